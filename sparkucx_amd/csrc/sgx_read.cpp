// sgx_read.cpp — the reduce side: ShuffleTransport.fetchBlocksByBlockIds
// (ucx/ShuffleTransport.scala:154-156) / BlockStoreClient.fetchBlocks
// (spark_3_0/UcxShuffleClient.scala:49-91) served from HBM, and what UcxShuffleReader.read
// does after the fetch (spark_3_0/UcxShuffleReader.scala:137-191): deserialize (Kryo, LZ4),
// sort by key (keyOrdering), group / sum (aggregator).
#include "sgx_engine.h"

#include <algorithm>
#include <cstring>
#include <vector>

using namespace sgx;

static constexpr int64_t ITEM_BYTES = 64 * 1024;

// ------------------------------------------------------------------------------------
// fetchBlocksByBlockIds
// ------------------------------------------------------------------------------------
int sgx::fetch_impl(sgx_engine *e, Ctx &c, Shuffle &s, const int64_t *map_ids, const int32_t *reduce_ids, int64_t n,
                    void *dst, int64_t dst_cap, int32_t dst_mem_kind, int64_t *out_lengths, bool sync,
                    std::vector<std::shared_ptr<void>> *keep) {
    struct Src {
        const void *p;
        int64_t len;
        hipEvent_t ready;
        const MapOut *pad = nullptr;  // a padded map's block: gathered from its fragments
        int32_t part = 0;
    };
    // snapshot the shuffle's rounds and the maps asked for (references keep them alive)
    std::vector<std::shared_ptr<Round>> rounds;
    std::map<int64_t, std::shared_ptr<MapOut>> maps;
    {
        std::lock_guard<std::mutex> lk(s.mu);
        rounds = s.rounds;
        for (int64_t i = 0; i < n; ++i) {
            auto mt = s.maps.find(map_ids[i]);
            if (mt != s.maps.end()) maps[map_ids[i]] = mt->second;
        }
    }
    std::map<int64_t, std::vector<int64_t>> map_off;  // per local map: partition byte offsets
    std::map<int64_t, bool> map_pad;                  // per local map: read through its fragments
    std::vector<Src> srcs((size_t)n);
    // a padded map's fragments are copied a dword at a time at least: a destination that is
    // not 4-byte aligned reads the map's contiguous copy instead
    const bool dst_al4 = ((uintptr_t)dst & 3) == 0 || dst_mem_kind != SGX_MEM_DEVICE;
    int64_t total = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t mid = map_ids[i];
        const int32_t r = reduce_ids[i];
        if (r < 0 || r >= s.R) return fail_msg(SGX_ERR_INVALID, "reduceId %d out of range [0, %d)", r, s.R);
        bool found = false;
        // received blocks (newest round first)
        for (auto rt = rounds.rbegin(); rt != rounds.rend() && !found; ++rt) {
            Round &rd = **rt;
            if (r < rd.r0 || r >= rd.r1) continue;
            for (size_t j = 0; j < rd.map_ids.size(); ++j) {
                if (rd.map_ids[j] != mid) continue;
                srcs[(size_t)i] = Src{rd.block_ptr(j, r), rd.lens[j * (size_t)s.R + (size_t)r], rd.done.ev};
                found = true;
                break;
            }
        }
        if (!found) {
            auto mt = maps.find(mid);
            if (mt != maps.end()) {
                MapOut &m = *mt->second;
                auto ot = map_off.find(mid);
                if (ot == map_off.end()) {
                    std::lock_guard<std::mutex> lk(m.mu);
                    if (m.open) return fail_msg(SGX_ERR_STATE, "map %lld is still open", (long long)mid);
                    SGX_TRY(finish_lengths(e, c, s, m));
                    // (only a fill needs the contiguous copy; a size query reads lengths)
                    if (m.padded && !dst_al4 && dst) SGX_TRY(materialize(e, c, s, m));
                    std::vector<int64_t> o((size_t)s.R + 1, 0);
                    for (int32_t q = 0; q < s.R; ++q) o[(size_t)q + 1] = o[(size_t)q] + m.lengths[(size_t)q];
                    ot = map_off.emplace(mid, std::move(o)).first;
                    map_pad[mid] = m.padded && !m.dense_valid;
                }
                const int64_t bl = ot->second[(size_t)r + 1] - ot->second[(size_t)r];
                if (map_pad[mid])
                    srcs[(size_t)i] = Src{nullptr, bl, m.done.ev, &m, r};
                else
                    srcs[(size_t)i] = Src{(const char *)m.view() + ot->second[(size_t)r], bl, m.done.ev};
                found = true;
            }
        }
        if (!found)
            return fail_msg(SGX_ERR_NOT_FOUND, "shuffle_%d_%lld_%d is not registered", s.id, (long long)mid, r);
        out_lengths[i] = srcs[(size_t)i].len;
        total += srcs[(size_t)i].len;
    }
    if (total > dst_cap)
        return fail_msg(SGX_ERR_INVALID, "destination capacity %lld < %lld bytes", (long long)dst_cap, (long long)total);
    if (total > 0 && !dst) return fail_msg(SGX_ERR_INVALID, "dst is NULL");
    if (total == 0) return SGX_OK;
    hipStream_t st = c.st;
    // every source must be complete: wait on each distinct producer event once
    std::vector<hipEvent_t> waited;
    for (int64_t i = 0; i < n; ++i) {
        hipEvent_t ev = srcs[(size_t)i].ready;
        if (ev && std::find(waited.begin(), waited.end(), ev) == waited.end()) {
            HIP_TRY(hipStreamWaitEvent(st, ev, 0));
            waited.push_back(ev);
        }
    }
    // one gather launch: {src, dst, bytes} pieces of <= 64 KiB, back to back in request
    // order (the reader asks reducer-major, map-minor: the canonical per-reducer sequence)
    const bool dev_dst = dst_mem_kind == SGX_MEM_DEVICE;
    char *gdst = (char *)dst;
    if (!dev_dst) {
        SGX_TRY(c.gather_stage.ensure((size_t)total));
        gdst = (char *)c.gather_stage.p;
    }
    int64_t npieces = 0, nfrag = 0;
    int maxG = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (srcs[(size_t)i].pad) {
            ++nfrag;
            maxG = std::max(maxG, (int)srcs[(size_t)i].pad->frag_G);
        } else {
            npieces += (srcs[(size_t)i].len + ITEM_BYTES - 1) / ITEM_BYTES;
        }
    }
    // [pieces x 3][fragment descriptors], one host-to-device copy
    const int64_t nwords = npieces * 3 + nfrag * FRAG_DESC_WORDS;
    SGX_TRY(c.gather_items.ensure((size_t)nwords * 8));
    SGX_TRY(c.items_dev.ensure((size_t)nwords * 8));
    // the pinned item list is rewritten only after the previous gather's copy has landed
    HIP_TRY(hipStreamSynchronize(st));
    int64_t *gi = (int64_t *)c.gather_items.p, k = 0, off = 0;
    int64_t *fd = gi + npieces * 3, nf = 0;
    bool al16 = ((uintptr_t)gdst & 15) == 0, al4 = ((uintptr_t)gdst & 3) == 0;
    for (int64_t i = 0; i < n; ++i) {
        if (const MapOut *pm = srcs[(size_t)i].pad) {
            const int64_t len = (int64_t)s.R * pm->frag_G;
            const uint32_t *fstart = (const uint32_t *)pm->frag.p;
            int64_t *d = fd + FRAG_DESC_WORDS * nf++;
            d[0] = (int64_t)(uintptr_t)pm->data.p;
            d[1] = (int64_t)(uintptr_t)fstart;
            d[2] = (int64_t)(uintptr_t)(fstart + len);
            d[3] = (int64_t)(uintptr_t)(fstart + 2 * len);
            d[4] = (int64_t)(uintptr_t)(gdst + off);
            d[5] = srcs[(size_t)i].part;
            d[6] = pm->frag_G;
            d[7] = s.rb;
            off += srcs[(size_t)i].len;
            continue;
        }
        const char *sp = (const char *)srcs[(size_t)i].p;
        for (int64_t done = 0; done < srcs[(size_t)i].len; done += ITEM_BYTES, ++k) {
            const int64_t b = std::min<int64_t>(ITEM_BYTES, srcs[(size_t)i].len - done);
            gi[3 * k] = (int64_t)(uintptr_t)(sp + done);
            gi[3 * k + 1] = (int64_t)(uintptr_t)(gdst + off + done);
            gi[3 * k + 2] = b;
            const uintptr_t bits = (uintptr_t)(sp + done) | (uintptr_t)(off + done) | (uintptr_t)b;
            al16 = al16 && (bits & 15) == 0;
            al4 = al4 && (bits & 3) == 0;
        }
        off += srcs[(size_t)i].len;
    }
    hipEvent_t g0 = e->ev(), g1 = e->ev();
    HIP_TRY(hipEventRecord(g0, st));
    HIP_TRY(hipMemcpyAsync(c.items_dev.p, gi, (size_t)nwords * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_gather_items((const int64_t *)c.items_dev.p, npieces, al16 ? 16 : al4 ? 4 : 1, st));
    SGX_TRY(debug_sync(e, st, "k_gather_items"));
    HIP_TRY(launch_gather_frags((const int64_t *)c.items_dev.p + npieces * 3, nfrag, maxG, st));
    SGX_TRY(debug_sync(e, st, "k_gather_frags"));
    HIP_TRY(hipEventRecord(g1, st));
    e->record_stage(SGX_STAGE_REGROUP, g0, g1);
    if (!dev_dst) HIP_TRY(hipMemcpyAsync(dst, gdst, (size_t)total, hipMemcpyDeviceToHost, st));
    if (keep) {
        for (auto &r : rounds) keep->push_back(r);
        for (auto &kv : maps) keep->push_back(kv.second);
    }
    if (sync) HIP_TRY(hipStreamSynchronize(st));
    return SGX_OK;
}

extern "C" int sgx_fetch_blocks(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids,
                                const int32_t *reduce_ids, int64_t n, void *dst, int64_t dst_cap,
                                int32_t dst_mem_kind, int64_t *out_lengths) {
    sgx::TraceRange trace_("sgx_fetch_blocks");
    if (!e || (n > 0 && (!map_ids || !reduce_ids || !out_lengths))) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    return fetch_impl(e, *c, *s, map_ids, reduce_ids, n, dst, dst_cap, dst_mem_kind, out_lengths, true, nullptr);
}

// ------------------------------------------------------------------------------------
// records of a partition range (deserialized), sorting, grouping
// ------------------------------------------------------------------------------------
// The canonical block list of reducers [r0, r1) x maps: reducer-major, map order as given.
static void canonical_blocks(const int64_t *map_ids, int64_t nmaps, int32_t r0, int32_t r1, std::vector<int64_t> &mids,
                             std::vector<int32_t> &rids) {
    const int64_t nreq = (int64_t)(r1 - r0) * nmaps;
    mids.resize((size_t)nreq);
    rids.resize((size_t)nreq);
    for (int32_t r = r0; r < r1; ++r)
        for (int64_t j = 0; j < nmaps; ++j) {
            mids[(size_t)((r - r0) * nmaps + j)] = map_ids[j];
            rids[(size_t)((r - r0) * nmaps + j)] = r;
        }
}

// Gather the canonical blocks of reducers [r0, r1) x maps into c.sort_buf[0] as records (a
// Kryo shuffle's stream -- LZ4-decompressed first when compressed -- is decoded on the GPU on
// the way); c.sort_buf[1] is sized to match.  *nrec = records.  Synchronous.
static int records_impl(sgx_engine *e, Ctx &c, Shuffle &s, const int64_t *map_ids, int64_t nmaps, int32_t r0,
                        int32_t r1, int64_t *nrec) {
    if (r0 < 0 || r1 > s.R || r0 > r1)
        return fail_msg(SGX_ERR_INVALID, "partition range [%d, %d) outside [0, %d)", r0, r1, s.R);
    if (nmaps < 0 || (nmaps > 0 && !map_ids)) return fail_msg(SGX_ERR_INVALID, "bad map list");
    const int rb = s.rb;
    std::vector<int64_t> mids, lens;
    std::vector<int32_t> rids;
    canonical_blocks(map_ids, nmaps, r0, r1, mids, rids);
    const int64_t nreq = (int64_t)mids.size();
    lens.resize((size_t)nreq);
    std::vector<std::shared_ptr<void>> keep;
    // size query (fails with SGX_ERR_INVALID on capacity, after filling the lengths)
    int rc = fetch_impl(e, c, s, mids.data(), rids.data(), nreq, nullptr, 0, SGX_MEM_DEVICE, lens.data(), false, nullptr);
    if (rc != SGX_OK && rc != SGX_ERR_INVALID) return rc;
    int64_t total = 0;
    for (int64_t L : lens) total += L;
    hipStream_t st = c.st;
    // records per partition, in the gather's (reducer-major) order, for the sorted read's
    // segmented window pass; unknown for a Kryo stream until it is decoded
    c.gather_part_recs.clear();
    if (s.ser != SGX_SER_KRYO && nmaps > 0) {
        c.gather_part_recs.assign((size_t)(r1 - r0), 0);
        for (int64_t i = 0; i < nreq; ++i) c.gather_part_recs[(size_t)(i / nmaps)] += lens[(size_t)i] / rb;
    }
    if (s.ser == SGX_SER_KRYO) {
        // the fetched Kryo stream (blocks back to back are one valid stream) -> records
        *nrec = 0;
        if (s.lz4_block > 0 && total > 0) {
            // a compressed shuffle: fetch the LZ4 frames, decompress them into the Kryo input
            // (LZ4BlockInputStream, same stream, so no host round trip between the two)
            SGX_TRY(c.fetch_tmp.ensure((size_t)total));
            SGX_TRY(fetch_impl(e, c, s, mids.data(), rids.data(), nreq, c.fetch_tmp.p, total, SGX_MEM_DEVICE,
                               lens.data(), false, &keep));
            int64_t dec = 0;
            // every fetched block is one partition stream: walk them in parallel
            SGX_TRY(lz4_unframe_impl(e, c, c.fetch_tmp.p, total, &c.kryo_in, nullptr, 0, &dec, lens.data(), nreq));
            total = dec;
        }
        const int64_t cap = total / 4;  // a record takes >= 4 bytes
        SGX_TRY(c.sort_buf[0].ensure((size_t)cap * 16));
        if (total == 0) return SGX_OK;
        if (s.lz4_block == 0) {
            SGX_TRY(c.kryo_in.ensure((size_t)total + 64));
            SGX_TRY(fetch_impl(e, c, s, mids.data(), rids.data(), nreq, c.kryo_in.p, total, SGX_MEM_DEVICE,
                               lens.data(), false, &keep));
        }
        const int64_t tiles = kryo_deser16_tiles(total);
        SGX_TRY(c.kryo_work.ensure(24 + (size_t)kryo_work_bytes(tiles)));
        HIP_TRY(hipMemsetAsync(c.kryo_work.p, 0, 24, st));  // error word, record count
        uint32_t *tick = (uint32_t *)c.kryo_work.p;
        int64_t *cnt_dev = (int64_t *)((char *)c.kryo_work.p + 16);
        uint64_t *status = (uint64_t *)((char *)c.kryo_work.p + 24);
        hipEvent_t k0 = e->ev(), k1 = e->ev();
        HIP_TRY(hipEventRecord(k0, st));
        HIP_TRY(launch_kryo_deser16(c.kryo_in.p, total, c.sort_buf[0].p, cap, status, tick, cnt_dev, st));
        SGX_TRY(debug_sync(e, st, "Kryo decoder"));
        HIP_TRY(hipEventRecord(k1, st));
        e->record_stage(SGX_STAGE_DESERIALIZE, k0, k1);
        uint32_t herr[4];
        int64_t hcnt = 0;
        HIP_TRY(hipMemcpyAsync(herr, tick, 16, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&hcnt, cnt_dev, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (herr[1] & 1u) return fail_msg(SGX_ERR_TIMEOUT, "Kryo decoder look-back spin gave up");
        if (herr[1] & 2u) return fail_msg(SGX_ERR_INVALID, "fetched blocks are not a Kryo stream of (Long, Long) pairs");
        if (hcnt < 0 || hcnt > cap) return fail_msg(SGX_ERR_HIP, "internal error: Kryo record count %lld", (long long)hcnt);
        if (hcnt >= (int64_t)INT32_MAX) return fail_msg(SGX_ERR_INVALID, "%lld records exceed one read", (long long)hcnt);
        *nrec = hcnt;
        SGX_TRY(c.sort_buf[1].ensure((size_t)hcnt * 16));
        return SGX_OK;
    }
    const int64_t n = total / rb;
    if (n >= (int64_t)INT32_MAX) return fail_msg(SGX_ERR_INVALID, "%lld records exceed one sorted read", (long long)n);
    *nrec = n;
    SGX_TRY(c.sort_buf[0].ensure((size_t)total));
    SGX_TRY(c.sort_buf[1].ensure((size_t)total));
    if (n == 0) return SGX_OK;
    SGX_TRY(fetch_impl(e, c, s, mids.data(), rids.data(), nreq, c.sort_buf[0].p, total, SGX_MEM_DEVICE, lens.data(),
                       false, &keep));
    HIP_TRY(hipStreamSynchronize(st));  // `keep` holds the sources until here
    return SGX_OK;
}

// Stable sort of the n records in c.sort_buf[0]: LSD digit passes that are the map side's
// own K1-K4 with an internal digit partitioner (R = 256, KIND_DIGIT), least significant byte
// first -- i64 keys (bytes 0..7, the top byte sign-flipped) or TeraSort's 10-byte big-endian
// keys (bytes 9..0) -- then, with `by_partition`, one pass by the shuffle's partitioner
// (skipped for an ascending RangePartitioner, whose partition order is key order).  One read
// of the keys histograms every digit; a digit with a single non-empty bucket is the identity
// permutation and is skipped (unless SGX_FLAG_SORT_ALL_DIGITS).
int sgx::sort_records(sgx_engine *e, Ctx &c, const Shuffle &s, int64_t n, bool by_partition, const void **sorted,
                      int32_t nparts, void *final_dst) {
    const int rb = s.rb;
    if (rb != 16 && rb != 100)
        return fail_msg(SGX_ERR_UNSUPPORTED, "sorted read needs 16 B (Long, Long) or 100 B TeraSort records, not %d B",
                        rb);
    *sorted = c.sort_buf[0].p;
    if (n == 0) return SGX_OK;
    hipStream_t st = c.st;
    constexpr int MAXP = 12;
    SGX_TRY(c.sort_err.ensure(MAXP * 4));
    HIP_TRY(hipMemsetAsync(c.sort_err.p, 0, MAXP * 4, st));
    uint32_t *errs = (uint32_t *)c.sort_err.p;
    hipEvent_t t0 = e->ev(), t1 = e->ev();
    HIP_TRY(hipEventRecord(t0, st));
    const int ndig = rb == 16 ? 8 : 10;
    SGX_TRY(c.digit_hist.ensure((size_t)ndig * 256 * 4));
    const bool skip = !(e->flags & SGX_FLAG_SORT_ALL_DIGITS);
    int cur = 0, np = 0;
    const bool range_asc = s.kind != SGX_PART_HASH && s.asc;
    // Bucket path: a window of the key's top varying bits, sized so a bucket (P, window)
    // holds ~64 records, taken in <= 10-bit LSD passes (KIND_KEY_BITS), then the pass by the
    // partitioner, then every bucket sorted on chip (launch_bucket_sort) -- 2-4 passes instead
    // of up to 8-10 digit passes + 1.  Skewed keys (the top varying byte's largest value
    // holding > 1/16 of the records) keep the digit passes, whose trivial digits are skipped.
    // (a read of one partition needs no pass by the partitioner: every record has the same one)
    const bool use_p = by_partition && !range_asc && s.R > 1 && nparts != 1;
    // Segmented passes: the gather of a fixed-codec read left partition p's records
    // contiguous (c.gather_part_recs), so every LSD pass can run inside each partition's segment
    // -- pieces of <= SEG_PIECE records, K4's SEG mode from per-piece offsets -- and the final
    // pass by the partitioner disappears.
    constexpr int64_t SEG_PIECE = 1 << 17;
    const std::vector<int64_t> &gpr = c.gather_part_recs;
    int64_t gpr_sum = 0;
    for (int64_t x : gpr) gpr_sum += x;
    const bool seg_ok = use_p && rb == 16 && !(e->flags & SGX_FLAG_NO_SEG_WINDOW) && nparts > 0 &&
                        (int64_t)gpr.size() == (int64_t)nparts && gpr_sum == n;
    bool seg_planned = false;
    int64_t seg_npieces = 0;
    const int64_t *seg_desc = nullptr;
    const uint32_t *seg_nd = nullptr;
    uint32_t *seg_cnt = nullptr, *seg_offs = nullptr;
    const int64_t *seg_base = nullptr;
    const int32_t *seg_pk = nullptr;
    auto seg_plan = [&]() -> int {
        if (seg_planned) return SGX_OK;
        const int64_t nseg = (int64_t)gpr.size();
        int64_t npieces = 0;
        for (int64_t x : gpr) npieces += (x + SEG_PIECE - 1) / SEG_PIECE;
        // [desc 4 x npieces i64][seg_base nseg i64][pk nseg+1 i32][ndesc | seg_end u32][cnt][offs]
        auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
        const size_t b_desc = al((size_t)std::max<int64_t>(npieces, 1) * 32), b_base = al((size_t)nseg * 8);
        const size_t b_pk = al((size_t)(nseg + 1) * 4), b_sc = 256;
        const size_t b_cnt = al((size_t)std::max<int64_t>(npieces, 1) * 1024 * 4);
        const size_t host = b_desc + b_base + b_pk + b_sc;
        SGX_TRY(c.seg_work.ensure(host + 2 * b_cnt));
        SGX_TRY(c.seg_desc_host.ensure(host));
        char *hw = (char *)c.seg_desc_host.p;
        int64_t *hd = (int64_t *)hw, *hb = (int64_t *)(hw + b_desc);
        int32_t *hpk = (int32_t *)(hw + b_desc + b_base);
        uint32_t *hsc = (uint32_t *)(hw + b_desc + b_base + b_pk);
        int64_t k = 0, pos = 0;
        for (int64_t sg = 0; sg < nseg; ++sg) {
            hb[sg] = pos;
            hpk[sg] = (int32_t)k;
            const int64_t x = gpr[(size_t)sg];
            for (int64_t b = 0; b < x; b += SEG_PIECE, ++k) {
                hd[4 * k] = pos + b;
                hd[4 * k + 1] = 0;
                hd[4 * k + 2] = k;  // K4's "segment" index: this piece's own offsets (G = 1)
                hd[4 * k + 3] = 0;
            }
            pos += x;
        }
        hpk[nseg] = (int32_t)k;
        hsc[0] = (uint32_t)npieces;
        hsc[1] = (uint32_t)n;
        char *dw = (char *)c.seg_work.p;
        HIP_TRY(hipMemcpyAsync(dw, hw, host, hipMemcpyHostToDevice, st));
        seg_desc = (const int64_t *)dw;
        seg_base = (const int64_t *)(dw + b_desc);
        seg_pk = (const int32_t *)(dw + b_desc + b_base);
        seg_nd = (const uint32_t *)(dw + b_desc + b_base + b_pk);
        seg_cnt = (uint32_t *)(dw + host);
        seg_offs = (uint32_t *)(dw + host + b_cnt);
        seg_npieces = npieces;
        seg_planned = true;
        return SGX_OK;
    };
    // The keys' first read: the digit histograms (which bytes vary, skew), and -- when the
    // segmented bucket path is possible -- in the same pass every piece's histogram of the
    // window that path takes if the keys' top byte varies (k_piece_digit_hist); the window pass
    // below uses those counts when the guess holds instead of counting again.
    const double rp = use_p ? (double)(nparts > 0 ? std::min(nparts, s.R) : s.R) : 1.0;
    int kbits0 = 0;  // the window width the bucket path takes (before the top byte's cap)
    while (kbits0 < 30 && (double)n / (rp * (double)(1ull << kbits0)) > 64.0) ++kbits0;
    PartParams spec{};
    bool spec_counted = false;
    if (seg_ok && skip && !(e->flags & SGX_FLAG_NO_BUCKET_SORT) && s.kind == SGX_PART_HASH && kbits0 >= 1 &&
        kbits0 <= 10) {
        SGX_TRY(seg_plan());
        if (seg_npieces > 0) {
            spec.kind = KIND_KEY_BITS;
            spec.R = 1u << kbits0;
            spec.nbits = (uint32_t)kbits0;
            spec.dshift = (uint32_t)(64 - kbits0);
            spec.dflip = 1u;
            HIP_TRY(launch_piece_digit_hist(c.sort_buf[0].p, n, seg_desc, seg_npieces, spec, seg_cnt,
                                            (uint32_t *)c.digit_hist.p, st));
            spec_counted = true;
        }
    }
    if (!spec_counted) HIP_TRY(launch_digit_hist(c.sort_buf[0].p, n, rb, (uint32_t *)c.digit_hist.p, e->num_cus, st));
    std::vector<uint32_t> dh((size_t)ndig * 256);
    HIP_TRY(hipMemcpyAsync(dh.data(), c.digit_hist.p, dh.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    // one segmented pass c.sort_buf[cur] -> c.sort_buf[cur ^ 1] by kp (KIND_KEY_BITS / KIND_DIGIT)
    auto seg_pass = [&](PartParams kp, uint32_t *err) -> int {
        SGX_TRY(seg_plan());
        if (seg_npieces == 0) return SGX_OK;
        const ScatterGeom geo = scatter_geom16_wc(kp.R);
        if (geo.items == 0) return fail_msg(SGX_ERR_HIP, "internal error: no write-combining geometry for %u", kp.R);
        kp.mbits = (uint32_t)geo.mbits;
        // the counts of the first read, when this is the guessed window over the unsorted buffer
        const bool have = spec_counted && cur == 0 && kp.kind == KIND_KEY_BITS && kp.R == spec.R &&
                          kp.dshift == spec.dshift && kp.dflip == spec.dflip;
        spec_counted = false;
        if (!have) HIP_TRY(launch_piece_hist(c.sort_buf[cur].p, n, seg_desc, seg_npieces, kp, seg_cnt, st));
        HIP_TRY(launch_seg_offsets(seg_cnt, seg_base, seg_pk, (int64_t)gpr.size(), kp.R, seg_offs, st));
        HIP_TRY(launch_scatter16_seg(c.sort_buf[cur].p, c.sort_buf[cur ^ 1].p, n, kp, seg_offs, 1, seg_desc, seg_nd,
                                     seg_nd + 1, (int)seg_npieces, geo, err, st));
        return debug_sync(e, st, "segmented sort pass");
    };
    if (skip && !(e->flags & SGX_FLAG_NO_BUCKET_SORT) && (use_p ? s.kind == SGX_PART_HASH : true)) {
        int top_byte = -1;  // most significant varying key byte, as a bit position of the window
        uint32_t maxbin = 0;
        for (int d = ndig - 1; d >= 0 && top_byte < 0; --d) {
            const int byte = rb == 16 ? d : 9 - d;
            uint32_t mx = 0;
            for (int b = 0; b < 256; ++b) mx = std::max(mx, dh[(size_t)byte * 256 + (size_t)b]);
            if (mx == (uint32_t)n) continue;  // constant byte
            maxbin = mx;
            top_byte = byte;
        }
        // window top bit: 16 B -> 8 * (byte + 1) of the sign-flipped Long; 100 B -> the first 8
        // key bytes big-endian, byte j ends at bit 64 - 8 j (bytes 8, 9 are outside the window)
        const int top = top_byte < 0 ? 64 : (rb == 16 ? 8 * (top_byte + 1) : (top_byte < 8 ? 64 - 8 * top_byte : -1));
        const int kbits = std::min(kbits0, std::max(top, 0));
        // (buckets must fit the bucket sort's halo: 255 records for 16 B, 127 for 100 B)
        const double max_avg = rb == 16 ? 128.0 : 64.0;
        const bool eligible = top_byte >= 0 && top > 0 && (uint64_t)maxbin * 16 <= (uint64_t)n &&
                              (double)n / (rp * (double)(1ull << kbits)) <= max_avg;
        if (eligible) {
            const int lo = top - kbits;
            // Segmented form: the gather left every partition's records
            // contiguous, so one stable pass by the window bits inside each partition's segment
            // replaces the window pass + the pass by the partitioner.
            bool seg_done = false;
            if (seg_ok && kbits >= 1 && kbits <= 10) {
                PartParams kp{};
                kp.kind = KIND_KEY_BITS;
                kp.R = 1u << kbits;
                kp.nbits = (uint32_t)kbits;
                kp.dshift = (uint32_t)lo;
                kp.dflip = 1u;
                SGX_TRY(seg_pass(kp, errs + np));
                cur ^= 1;
                ++np;
                seg_done = true;
            }
            for (int b0 = lo; b0 < top && !seg_done; b0 += 10) {  // least significant window chunk first
                const int cb = std::min(10, top - b0);
                PartParams kp{};
                kp.kind = KIND_KEY_BITS;
                kp.R = 1u << cb;
                kp.nbits = (uint32_t)cb;
                kp.dshift = (uint32_t)b0;
                kp.dflip = rb == 16 ? 1u : 0u;
                SGX_TRY(partition_pass(e, c, c.sort_buf[cur].p, c.sort_buf[cur ^ 1].p, n, rb, kp, (int32_t)kp.R,
                                       KIND_KEY_BITS, nullptr, errs + np, false));
                cur ^= 1;
                ++np;
            }
            if (use_p && !seg_done) {
                SGX_TRY(partition_pass(e, c, c.sort_buf[cur].p, c.sort_buf[cur ^ 1].p, n, rb, s.pp, s.R, s.kind,
                                       nullptr, errs + np, false));
                cur ^= 1;
                ++np;
            }
            // the last pass straight into the caller's device buffer when it has one (a sorted read
            // into HBM: no copy of the result afterwards)
            void *bout = final_dst ? final_dst : c.sort_buf[cur ^ 1].p;
            HIP_TRY(launch_bucket_sort(c.sort_buf[cur].p, bout, n, rb, s.pp, use_p ? 1 : 0,
                                       (uint32_t)lo, (uint32_t)kbits, errs + np, st));
            SGX_TRY(debug_sync(e, st, "bucket sort"));
            ++np;
            uint32_t herr[MAXP];
            HIP_TRY(hipMemcpyAsync(herr, c.sort_err.p, MAXP * 4, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            for (int i = 0; i < np; ++i) {
                if (herr[i] & 1u) return fail_msg(SGX_ERR_TIMEOUT, "sort pass %d: scan look-back spin gave up", i);
                if (herr[i] & 2u) return fail_msg(SGX_ERR_HIP, "sort pass %d: a scatter destination was out of range", i);
            }
            if (!(herr[np - 1] & 4u)) {
                HIP_TRY(hipEventRecord(t1, st));
                e->record_stage(SGX_STAGE_SORT, t0, t1);
                *sorted = bout;
                return SGX_OK;
            }
            // a bucket too long for the chip: the digit passes below finish from the bucket
            // sort's input (stable passes: any stable order of the input sorts the same)
            HIP_TRY(hipMemsetAsync(c.sort_err.p, 0, MAXP * 4, st));
            np = 0;
        }
    }
    // LSD digit passes (8-bit digits, least significant first); a digit whose histogram has
    // one non-empty bucket is the identity permutation and is skipped
    for (int d = 0; d < ndig; ++d) {
        const int byte = rb == 16 ? d : 9 - d;  // digit d of the LSD order
        bool trivial = false;
        for (int b = 0; b < 256; ++b)
            if (dh[(size_t)byte * 256 + (size_t)b] == (uint32_t)n) trivial = true;
        if (trivial && skip) continue;
        ++np;
        PartParams dp{};
        dp.kind = KIND_DIGIT;
        dp.R = DIGIT_R;
        dp.nbits = 8;
        dp.dshift = rb == 16 ? 8u * (uint32_t)d : 8u * (uint32_t)(9 - d);
        dp.dflip = (rb == 16 && d == 7) ? 0x80u : 0u;
        if (seg_ok)
            SGX_TRY(seg_pass(dp, errs + np - 1));
        else
            SGX_TRY(partition_pass(e, c, c.sort_buf[cur].p, c.sort_buf[cur ^ 1].p, n, rb, dp, (int32_t)DIGIT_R,
                                   KIND_DIGIT, nullptr, errs + np - 1, false));
        cur ^= 1;
    }
    if (use_p && !seg_ok) {
        SGX_TRY(partition_pass(e, c, c.sort_buf[cur].p, c.sort_buf[cur ^ 1].p, n, rb, s.pp, s.R, s.kind, nullptr,
                               errs + np, false));
        cur ^= 1;
        ++np;
    }
    HIP_TRY(hipEventRecord(t1, st));
    e->record_stage(SGX_STAGE_SORT, t0, t1);
    uint32_t herr[MAXP];
    HIP_TRY(hipMemcpyAsync(herr, c.sort_err.p, MAXP * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (int i = 0; i < np; ++i) {
        if (herr[i] & 1u) return fail_msg(SGX_ERR_TIMEOUT, "sort pass %d: scan look-back spin gave up", i);
        if (herr[i] & 2u) return fail_msg(SGX_ERR_HIP, "sort pass %d: a scatter destination was out of range", i);
    }
    *sorted = c.sort_buf[cur].p;
    return SGX_OK;
}

int sgx::group_records(sgx_engine *e, Ctx &c, const void *sorted, int64_t n, int32_t agg, int64_t *ngroups,
                       int64_t **keys, int64_t **starts, int64_t **vals) {
    hipStream_t st = c.st;
    *ngroups = 0;
    // one pass (k_group_fused): outputs sized for the worst case (every record its own group)
    if (n >= (int64_t)1 << 31) return fail_msg(SGX_ERR_UNSUPPORTED, "grouping %lld records (limit 2^31 - 1)", (long long)n);
    const int64_t tiles = group_tiles(n);
    SGX_TRY(c.grp_out.ensure((size_t)std::max<int64_t>(n, 1) * 24));
    int64_t *dkeys = (int64_t *)c.grp_out.p, *dstarts = dkeys + std::max<int64_t>(n, 1),
            *dvals = dstarts + std::max<int64_t>(n, 1);
    // [ticket, err | ngroups | two status words per tile]
    SGX_TRY(c.grp_status.ensure((size_t)(16 + tiles * 16)));
    uint32_t *ticket_err = (uint32_t *)c.grp_status.p;
    int64_t *dng = (int64_t *)((char *)c.grp_status.p + 8);
    hipEvent_t t0 = e->ev(), t1 = e->ev();
    HIP_TRY(hipEventRecord(t0, st));
    int64_t ng = 0;
    if (n > 0) {
        HIP_TRY(hipMemsetAsync(c.grp_status.p, 0, (size_t)(16 + tiles * 16), st));
        HIP_TRY(launch_group_fused(sorted, n, agg == SGX_AGG_SUM, (uint64_t *)((char *)c.grp_status.p + 16), ticket_err,
                                   ticket_err + 1, dkeys, starts ? dstarts : nullptr, dvals, dng, st));
        uint32_t terr[2] = {0, 0};
        HIP_TRY(hipMemcpyAsync(&ng, dng, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(terr, ticket_err, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (terr[1] & 1u) return fail_msg(SGX_ERR_TIMEOUT, "group scan look-back spin gave up");
    }
    HIP_TRY(hipEventRecord(t1, st));
    e->record_stage(SGX_STAGE_GROUP, t0, t1);
    *ngroups = ng;
    *keys = dkeys;
    if (starts) *starts = dstarts;
    *vals = dvals;
    return SGX_OK;
}

// (A pinned, multi-threaded staging of copies into pageable memory was measured against
// this in round 6: 34 vs 32 ms for groupByKey's 1.5 GB into mapped pages, 64 vs 70 ms into
// fresh ones -- the runtime's copy kept)
static int copy_out(Ctx &c, void *dst, const void *src, int64_t bytes, int32_t mem_kind) {
    if (bytes <= 0) return SGX_OK;
    HIP_TRY(hipMemcpyAsync(dst, src, (size_t)bytes,
                           mem_kind == SGX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c.st));
    return SGX_OK;
}

// Common entry checks of the reads; *s and *c on success.
// ------------------------------------------------------------------------------------
// size query + fill: reuse of the size query's result (Ctx::ReadCache)
// ------------------------------------------------------------------------------------
enum { RC_RECORDS = 0, RC_SORTED = 1, RC_GROUPED = 2 };

static bool rc_hit(const Ctx &c, uint64_t epoch, int kind, int agg, int32_t sid, const int64_t *maps, int64_t nmaps,
                   int32_t r0, int32_t r1) {
    const Ctx::ReadCache &k = c.rc;
    return k.ops + 1 == c.ops && k.epoch == epoch && k.kind == kind && k.agg == agg && k.sid == sid && k.r0 == r0 &&
           k.r1 == r1 && (int64_t)k.maps.size() == nmaps && (nmaps == 0 || std::equal(k.maps.begin(), k.maps.end(), maps));
}

static void rc_store(Ctx &c, uint64_t epoch, int kind, int agg, int32_t sid, const int64_t *maps, int64_t nmaps,
                     int32_t r0, int32_t r1, int64_t n, int64_t ng, const void *sorted, int64_t *keys, int64_t *starts,
                     int64_t *vals) {
    Ctx::ReadCache &k = c.rc;
    k.ops = c.ops;
    k.epoch = epoch;
    k.kind = kind;
    k.agg = agg;
    k.sid = sid;
    k.r0 = r0;
    k.r1 = r1;
    k.maps.assign(maps, maps + nmaps);
    k.n = n;
    k.ng = ng;
    k.sorted = sorted;
    k.keys = keys;
    k.starts = starts;
    k.vals = vals;
}

static int read_entry(sgx_engine *e, int32_t shuffle_id, int32_t mem_kind, std::shared_ptr<Shuffle> *s, Ctx **c) {
    if (mem_kind != SGX_MEM_HOST && mem_kind != SGX_MEM_DEVICE) return fail_msg(SGX_ERR_INVALID, "unknown mem_kind %d", mem_kind);
    *s = e->find_shuffle(shuffle_id);
    if (!*s) return SGX_ERR_STATE;
    HIP_TRY(hipSetDevice(e->device));
    *c = e->ctx();
    return *c ? SGX_OK : SGX_ERR_HIP;
}

extern "C" int sgx_read_sorted(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                               int32_t start_partition, int32_t end_partition, void *dst, int64_t dst_cap,
                               int32_t dst_mem_kind, int64_t *out_bytes) {
    sgx::TraceRange trace_("sgx_read_sorted");
    if (!e || !out_bytes) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    std::shared_ptr<Shuffle> s;
    Ctx *c = nullptr;
    SGX_TRY(read_entry(e, shuffle_id, dst_mem_kind, &s, &c));
    const int rb = s->rb;
    const uint64_t epoch = e->epoch.load();
    if (!dst && dst_cap == 0 && s->ser == SGX_SER_KRYO) {  // size query: decoded records, sorted and kept
        int64_t n = 0;
        const void *sorted = nullptr;
        SGX_TRY(records_impl(e, *c, *s, map_ids, nmaps, start_partition, end_partition, &n));
        SGX_TRY(sort_records(e, *c, *s, n, true, &sorted, end_partition - start_partition));
        rc_store(*c, epoch, RC_SORTED, 0, shuffle_id, map_ids, nmaps, start_partition, end_partition, n, 0, sorted,
                 nullptr, nullptr, nullptr);
        *out_bytes = n * rb;
        return SGX_OK;
    }
    if (!dst && dst_cap == 0) {  // size query: lengths only
        if (start_partition < 0 || end_partition > s->R || start_partition > end_partition || nmaps < 0 ||
            (nmaps > 0 && !map_ids))
            return fail_msg(SGX_ERR_INVALID, "bad partition range or map list");
        std::vector<int64_t> mids, lens;
        std::vector<int32_t> rids;
        canonical_blocks(map_ids, nmaps, start_partition, end_partition, mids, rids);
        lens.resize(mids.size());
        int rc = fetch_impl(e, *c, *s, mids.data(), rids.data(), (int64_t)mids.size(), nullptr, 0, SGX_MEM_DEVICE,
                            lens.data(), false, nullptr);
        if (rc != SGX_OK && rc != SGX_ERR_INVALID) return rc;
        int64_t total = 0;
        for (int64_t L : lens) total += L;
        *out_bytes = total;
        return SGX_OK;
    }
    int64_t n = 0;
    const void *sorted = nullptr;
    if (rc_hit(*c, epoch, RC_SORTED, 0, shuffle_id, map_ids, nmaps, start_partition, end_partition)) {
        n = c->rc.n;
        sorted = c->rc.sorted;
    } else {
        SGX_TRY(records_impl(e, *c, *s, map_ids, nmaps, start_partition, end_partition, &n));
        if (n * rb > dst_cap)
            return fail_msg(SGX_ERR_INVALID, "destination capacity %lld < %lld bytes", (long long)dst_cap,
                            (long long)(n * rb));
        // a device destination takes the sort's last pass directly
        const bool direct = dst && dst_mem_kind == SGX_MEM_DEVICE && ((uintptr_t)dst & 15) == 0 &&
                            dst != c->sort_buf[0].p && dst != c->sort_buf[1].p;
        SGX_TRY(sort_records(e, *c, *s, n, true, &sorted, end_partition - start_partition, direct ? dst : nullptr));
    }
    *out_bytes = n * rb;
    c->last_read_records = n;
    if (n * rb > dst_cap)
        return fail_msg(SGX_ERR_INVALID, "destination capacity %lld < %lld bytes", (long long)dst_cap,
                        (long long)(n * rb));
    if (n > 0 && !dst) return fail_msg(SGX_ERR_INVALID, "dst is NULL");
    if (sorted != dst) SGX_TRY(copy_out(*c, dst, sorted, n * rb, dst_mem_kind));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SGX_OK;
}

extern "C" int sgx_read_records(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                                int32_t start_partition, int32_t end_partition, void *dst, int64_t dst_cap,
                                int32_t dst_mem_kind, int64_t *out_bytes) {
    sgx::TraceRange trace_("sgx_read_records");
    if (!e || !out_bytes) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    std::shared_ptr<Shuffle> s;
    Ctx *c = nullptr;
    SGX_TRY(read_entry(e, shuffle_id, dst_mem_kind, &s, &c));
    const int rb = s->rb;
    const uint64_t epoch = e->epoch.load();
    int64_t n = 0;
    if (rc_hit(*c, epoch, RC_RECORDS, 0, shuffle_id, map_ids, nmaps, start_partition, end_partition))
        n = c->rc.n;  // the records are still in c->sort_buf[0]
    else
        SGX_TRY(records_impl(e, *c, *s, map_ids, nmaps, start_partition, end_partition, &n));
    *out_bytes = n * rb;
    c->last_read_records = n;
    if (!dst && dst_cap == 0) {  // size query
        rc_store(*c, epoch, RC_RECORDS, 0, shuffle_id, map_ids, nmaps, start_partition, end_partition, n, 0,
                 c->sort_buf[0].p, nullptr, nullptr, nullptr);
        return SGX_OK;
    }
    if (n * rb > dst_cap)
        return fail_msg(SGX_ERR_INVALID, "destination capacity %lld < %lld bytes", (long long)dst_cap,
                        (long long)(n * rb));
    if (n > 0 && !dst) return fail_msg(SGX_ERR_INVALID, "dst is NULL");
    SGX_TRY(copy_out(*c, dst, c->sort_buf[0].p, n * rb, dst_mem_kind));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SGX_OK;
}

extern "C" int sgx_read_grouped(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                                int32_t start_partition, int32_t end_partition, int32_t agg, int64_t *keys,
                                int64_t *group_starts, int64_t *values, int64_t cap_groups, int64_t cap_values,
                                int32_t mem_kind, int64_t *out_groups, int64_t *out_values) {
    sgx::TraceRange trace_("sgx_read_grouped");
    if (!e || !out_groups || !out_values) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    if (agg != SGX_AGG_GROUP && agg != SGX_AGG_SUM) return fail_msg(SGX_ERR_INVALID, "unknown aggregation %d", agg);
    std::shared_ptr<Shuffle> s;
    Ctx *c = nullptr;
    SGX_TRY(read_entry(e, shuffle_id, mem_kind, &s, &c));
    if (s->rb != 16)
        return fail_msg(SGX_ERR_UNSUPPORTED, "grouped read needs 16 B (Long, Long) records, not %d B", s->rb);
    // a map-side-combined shuffle holds combiners: only combineCombinersByKey (sum) applies
    if (s->combine == SGX_AGG_SUM && agg != SGX_AGG_SUM)
        return fail_msg(SGX_ERR_UNSUPPORTED, "shuffle %d was combined map-side (sum): read it with SGX_AGG_SUM",
                        shuffle_id);
    const uint64_t epoch = e->epoch.load();
    int64_t n = 0, ng = 0;
    int64_t *dkeys = nullptr, *dstarts = nullptr, *dvals = nullptr;
    if (rc_hit(*c, epoch, RC_GROUPED, agg, shuffle_id, map_ids, nmaps, start_partition, end_partition)) {
        n = c->rc.n;
        ng = c->rc.ng;
        dkeys = c->rc.keys;
        dstarts = c->rc.starts;
        dvals = c->rc.vals;
    } else {
        SGX_TRY(records_impl(e, *c, *s, map_ids, nmaps, start_partition, end_partition, &n));
        const void *sorted = nullptr;
        SGX_TRY(sort_records(e, *c, *s, n, true, &sorted, end_partition - start_partition));
        SGX_TRY(group_records(e, *c, sorted, n, agg, &ng, &dkeys, &dstarts, &dvals));
    }
    const int64_t nvals = agg == SGX_AGG_GROUP ? n : ng;
    c->last_read_records = n;  // the shuffled records the aggregation consumed
    *out_groups = ng;
    *out_values = nvals;
    if (!keys && cap_groups == 0 && cap_values == 0) {  // size query
        rc_store(*c, epoch, RC_GROUPED, agg, shuffle_id, map_ids, nmaps, start_partition, end_partition, n, ng, nullptr,
                 dkeys, dstarts, dvals);
        return SGX_OK;
    }
    if (ng > cap_groups || nvals > cap_values)
        return fail_msg(SGX_ERR_INVALID, "capacity (%lld groups, %lld values) < (%lld, %lld)", (long long)cap_groups,
                        (long long)cap_values, (long long)ng, (long long)nvals);
    if (n == 0) return SGX_OK;
    if (!keys || !values || (agg == SGX_AGG_GROUP && !group_starts)) return fail_msg(SGX_ERR_INVALID, "NULL output array");
    SGX_TRY(copy_out(*c, keys, dkeys, ng * 8, mem_kind));
    if (group_starts) SGX_TRY(copy_out(*c, group_starts, dstarts, ng * 8, mem_kind));
    SGX_TRY(copy_out(*c, values, dvals, nvals * 8, mem_kind));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SGX_OK;
}

// The records (before any aggregation) the calling thread's last sgx_read_records / _sorted /
// _grouped consumed: what the reference's reader counts with incRecordsRead, one per shuffled
// record ahead of the aggregator (spark_3_0/UcxShuffleReader.scala:148-162).
extern "C" int sgx_last_read_records(sgx_engine *e, int64_t *out) {
    if (!e || !out) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    *out = c->last_read_records;
    return SGX_OK;
}
