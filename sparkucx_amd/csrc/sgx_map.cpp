// sgx_map.cpp — the map side: getWriter(...).write(records) + commitAllPartitions
// (spark_3_0/UcxShuffleManager.scala:32-53; ucx/NvkvShuffleMapOutputWriter.scala:105-148).
//
//   sgx_write_map    one batch: K1+K2 histogram -> K3 scan -> K4 stable scatter on the calling
//                    thread's stream, then (dep.serializer = Kryo) the Kryo framing kernels;
//                    with dep.mapSideCombine the records are first combined per key (sort by
//                    key within partition + segmented sum + repartition).
//   sgx_map_begin / _append / _commit   a map task whose records arrive in several batches
//                    (spills): every batch is partitioned on arrival, the commit concatenates
//                    the batches per partition in append order.
//   finish_lengths   long[R] partition lengths (commitAllPartitions' return value) and the
//                    published bytes: fixed records, the Kryo stream, or its LZ4 frames.
#include "sgx_engine.h"

#include <algorithm>
#include <cstring>

using namespace sgx;

// ------------------------------------------------------------------------------------
// one stable partition pass
// ------------------------------------------------------------------------------------
// K1+K2 hist -> K3 scan -> K4 scatter of `n` records of `rb` bytes from device memory `in`
// to `out` under partitioner `spp` (R partitions, `kind`), asynchronous on the context's
// stream.  The (R+1) record offsets and the device error word land in `host_off` (R+2 u32,
// pinned) when given; the error word alone in `err_slot` (device) when given; the device
// offsets stay in c.last_off_dev until the context's next pass.
int sgx::partition_pass(sgx_engine *e, Ctx &c, const void *in, void *out, int64_t n, int rb, const PartParams &spp0,
                        int32_t R, int32_t kind, uint32_t *host_off, uint32_t *err_slot, bool stats,
                        const ChunkTable *ct) {
    PartParams spp = spp0;
    spp.chunks = ct ? ct->dev : nullptr;
    hipStream_t st = c.st;
    // K4 choice (every choice is byte-identical):
    //   hash, 16 B, R <= 1024   write-combining staged kernel (whole 128 B lines only)
    //   hash, 16 B, R > 1024    lane-ordered staged kernel
    //   range, 16 B             ballot-matched staged kernel (slot -> partition search)
    //   100 B                   LDS-staged dword-stream kernel (R <= 2048), else per-lane copy
    ScatterGeom geo = rb == 16 ? scatter_geom16((uint32_t)R, e->sc_waves, e->sc_items)
                               : scatter_geom_wide((uint32_t)R, rb);
    if (rb == 16 && kind == SGX_PART_HASH && e->rank_mode == SGX_RANK_ORDERED) {
        const ScatterGeom o = scatter_geom16_ord((uint32_t)R, e->sc_waves, e->sc_items);
        if (o.items) geo = o;
        if (!(e->flags & SGX_FLAG_NO_WRITE_COMBINING) && e->sc_waves == 0 && e->sc_items == 0) {
            const ScatterGeom w = scatter_geom16_wc((uint32_t)R);
            if (w.items) geo = w;
        }
    }
    if (rb != 16 && !(e->flags & SGX_FLAG_NO_WIDE_STAGED) && e->lds_order_ok && ((uintptr_t)in & 15) == 0) {
        const ScatterGeom w2 = scatter_geom_wide2((uint32_t)R, rb, kind, spp.nb);
        if (w2.items) geo = w2;
    }
    // the reduce side's digit / key-window passes run on the write-combining / wide-record
    // kernels, or on the per-lane ballot-matched kernel when the engine-start check of the
    // lane-ordered ranking failed (sgx_create)
    if ((kind == KIND_DIGIT || kind == KIND_KEY_BITS) && !e->lds_order_ok) {
        geo = scatter_geom_wide((uint32_t)R, rb);
    } else if (kind == KIND_DIGIT || kind == KIND_KEY_BITS) {
        if (rb == 16) geo = scatter_geom16_wc((uint32_t)R);
        if (geo.waves < WC_GEOM_BASE && geo.waves != WIDE2_GEOM_TAG)
            return fail_msg(SGX_ERR_UNSUPPORTED, "digit pass on %d B records at this alignment", rb);
    }
    // R > 1024 (power of two, hash, 16 B): the hybrid two-level split -- level 1 writes the
    // hot partitions straight to the output and the cold ones into S = R / 64
    // super-partitions, level 2 splits each super into Q = 64; both write-combining, whole
    // lines only, instead of one pass whose runs leave L2 as partial lines (sgx_kernels.hip,
    // "Two-level split scatter", "Hybrid split")
    const bool split = rb == 16 && kind == SGX_PART_HASH && R > 1024 && (R & (R - 1)) == 0 && R <= 4096 &&
                       e->rank_mode == SGX_RANK_ORDERED && e->sc_waves == 0 && e->sc_items == 0 &&
                       !(e->flags & (SGX_FLAG_NO_WRITE_COMBINING | SGX_FLAG_NO_SPLIT_SCATTER));
    constexpr int32_t Q = 64;
    const int32_t S = split ? R / Q : 0;
    ScatterGeom geo1{}, geo2{};
    if (split) {
        geo1 = scatter_geom16_wc((uint32_t)(SPLIT_HOT_CAP + S));
        geo2 = scatter_geom16_wc((uint32_t)Q);
        geo1.lds_bytes += ((size_t)R * 2 + 15) & ~(size_t)15;  // the partition -> stream table
        if (geo1.items == 0 || geo2.items == 0 || geo1.lds_bytes > 160 * 1024)
            return fail_msg(SGX_ERR_UNSUPPORTED, "split scatter geometry for R=%d", R);
        geo1.items = 8;  // 12 new records per lane spill registers in this kernel; 8 do not
        geo1.tile = 8 * 512;
        geo = geo1;
    }
    if (geo.items == 0)
        return fail_msg(SGX_ERR_UNSUPPORTED, "no scatter geometry (waves %d, items %d) fits R=%d", e->sc_waves,
                        e->sc_items, R);
    const int tile = geo.tile;
    int64_t chunk = n > 0 ? (n + e->G - 1) / e->G : 1;
    chunk = (chunk + tile - 1) / tile * tile;
    int G = n > 0 ? (int)((n + chunk - 1) / chunk) : 1;
    if (ct && n > 0) {  // a streaming map's chunks (cut by the commit on this geometry's tile)
        if (split || ct->chunk % tile != 0)
            return fail_msg(SGX_ERR_HIP, "internal error: chunk table of %lld records on a tile of %d",
                            (long long)ct->chunk, tile);
        chunk = ct->chunk;
        G = ct->G;
    }
    const int64_t len = (int64_t)R * G;
    const int64_t tiles = scan_tiles(len);
    const int64_t len1 = (int64_t)S * G;
    const int64_t tiles1 = split ? scan_tiles(len1) : 0;
    SGX_TRY(c.offs.ensure((size_t)len * 4));
    // one work block, zeroed by ONE memset (each fill / copy between kernels costs ~5-10 µs):
    // [counts u32 x R*G][ticket u32 | pad][look-back status u64 x tiles]
    // [partition offsets u32 x (R+1) | error] -- the error word sits right after the
    // offsets so one copy lands both on the host -- [ticket | status of the split's scan]
    const size_t counts_bytes = ((size_t)len * 4 + 15) & ~(size_t)15;
    const size_t status_bytes = ((size_t)(16 + tiles * 8) + 15) & ~(size_t)15;
    const size_t off_bytes = ((size_t)(R + 2) * 4 + 15) & ~(size_t)15;
    const size_t status1_bytes = split ? ((size_t)(16 + tiles1 * 8) + 15) & ~(size_t)15 : 0;
    const size_t work_bytes = counts_bytes + status_bytes + off_bytes + 2 * status1_bytes;
    SGX_TRY(c.work.ensure(work_bytes));
    uint32_t *counts = (uint32_t *)c.work.p;
    uint32_t *ticket = (uint32_t *)((char *)c.work.p + counts_bytes);
    uint64_t *status = (uint64_t *)((char *)ticket + 16);
    uint32_t *part_off_dev = (uint32_t *)((char *)ticket + status_bytes);
    uint32_t *err = part_off_dev + R + 1;
    uint32_t *ticket1 = (uint32_t *)((char *)part_off_dev + off_bytes);
    uint64_t *status1 = (uint64_t *)((char *)ticket1 + 16);
    uint32_t *ticket2 = (uint32_t *)((char *)ticket1 + status1_bytes);  // the piece numbering's scan
    uint64_t *status2 = (uint64_t *)((char *)ticket2 + 16);
    c.last_off_dev = part_off_dev;
    // the split's scratch: [csum u32 x S*G][offs1 u32 x S*G][flags u32 x S*G][idx u32 x S*G]
    // [part_off1 u32 x (S+2) | npieces u32 x 4][desc i64 x 4*S*G][cur1 u32 x (HOT+S)*G]
    // [stream_of u16 x R][hot_part i32 x HOT], and the level-1 output of the cold partitions
    uint32_t *csum = nullptr, *offs1 = nullptr, *part_off1 = nullptr, *npieces = nullptr, *pflags = nullptr,
             *pidx = nullptr, *cur1 = nullptr;
    int64_t *desc = nullptr;
    uint16_t *stream_of = nullptr;
    int32_t *hot_part = nullptr;
    if (split) {
        const size_t a = ((size_t)len1 * 4 + 15) & ~(size_t)15, b = ((size_t)(S + 6) * 4 + 15) & ~(size_t)15;
        const size_t cb = ((size_t)(SPLIT_HOT_CAP + S) * G * 4 + 15) & ~(size_t)15;
        const size_t tb = ((size_t)R * 2 + 15) & ~(size_t)15;
        SGX_TRY(c.split_work.ensure(4 * a + b + (size_t)len1 * 32 + cb + tb + SPLIT_HOT_CAP * 4));
        csum = (uint32_t *)c.split_work.p;
        offs1 = (uint32_t *)((char *)c.split_work.p + a);
        pflags = (uint32_t *)((char *)c.split_work.p + 2 * a);
        pidx = (uint32_t *)((char *)c.split_work.p + 3 * a);
        part_off1 = (uint32_t *)((char *)c.split_work.p + 4 * a);
        npieces = part_off1 + S + 2;
        desc = (int64_t *)((char *)c.split_work.p + 4 * a + b);
        cur1 = (uint32_t *)((char *)desc + (size_t)len1 * 32);
        stream_of = (uint16_t *)((char *)cur1 + cb);
        hot_part = (int32_t *)((char *)stream_of + tb);
        SGX_TRY(c.split_tmp.ensure((size_t)std::max<int64_t>(n, 1) * 16));
    }
    HIP_TRY(hipMemsetAsync(c.work.p, 0, work_bytes, st));

    // stage events: consecutive stages share their boundary event (every timing marker
    // between two kernels measured ~5 µs of idle GPU)
    hipEvent_t h0 = e->ev(), h1 = e->ev(), c1 = e->ev(), x1 = e->ev();
    HIP_TRY(hipEventRecord(h0, st));
    if (n > 0) HIP_TRY(launch_hist(in, n, rb, chunk, G, spp, counts, st, e->hist_mode, true));
    SGX_TRY(debug_sync(e, st, "K1+K2 k_hist"));
    HIP_TRY(hipEventRecord(h1, st));
    HIP_TRY(launch_scan((const uint32_t *)counts, (uint32_t *)c.offs.p, len, status, ticket, err, part_off_dev, G, R,
                        st));
    SGX_TRY(debug_sync(e, st, "K3 k_scan"));
    PartParams lpp = spp;
    lpp.mbits = (uint32_t)geo.mbits;
    if (split && n > 0) {
        // per map, on the device: the hot partitions (the SPLIT_HOT_CAP largest) and the
        // partition -> stream table; level-1 cursors (a hot stream: its final offsets; a cold
        // super: a scan of its cold partitions' per-chunk counts); level-2 pieces from those
        HIP_TRY(launch_hot_select(part_off_dev, R, Q, stream_of, hot_part, st));
        HIP_TRY(launch_super_counts_cold(counts, stream_of, csum, S, Q, G, st));
        HIP_TRY(launch_scan(csum, offs1, len1, status1, ticket1, err, part_off1, G, S, st));
        HIP_TRY(launch_hot_cursors((const uint32_t *)c.offs.p, hot_part, offs1, cur1, S, G, st));
        // level-2 pieces: cut from the cold records' count (on the device), about one per CU
        const int64_t pieces = std::max<int64_t>(1, (int64_t)e->num_cus - S);
        HIP_TRY(launch_seg_desc(offs1, S, G, part_off1 + S, pieces, desc, pflags, pidx, status2, ticket2, err, npieces,
                                st));
        SGX_TRY(debug_sync(e, st, "split scan / pieces"));
        HIP_TRY(hipEventRecord(c1, st));
        PartParams p1 = spp;
        p1.kind = KIND_HOT_SPLIT;
        p1.R = (uint32_t)(SPLIT_HOT_CAP + S);
        p1.dshift = (uint32_t)__builtin_ctz((unsigned)R);  // the full partition id's bits
        p1.dir = stream_of;
        p1.mbits = (uint32_t)geo1.mbits;
        HIP_TRY(launch_scatter(in, out, n, rb, chunk, G, p1, cur1, geo1, err, st, c.split_tmp.p,
                               (uint32_t)SPLIT_HOT_CAP));
        SGX_TRY(debug_sync(e, st, "K4 split level 1"));
        PartParams p2 = spp;
        p2.kind = KIND_HASH_POW2;
        p2.R = (uint32_t)Q;
        p2.mbits = (uint32_t)geo2.mbits;
        const int grid = (int)(S + pieces + 1);  // >= the pieces: one per super + every cut
        HIP_TRY(launch_scatter16_seg(c.split_tmp.p, out, n, p2, (const uint32_t *)c.offs.p, G, desc, npieces + 1,
                                     part_off1 + S, grid, geo2, err, st));
        SGX_TRY(debug_sync(e, st, "K4 split level 2"));
    } else {
        HIP_TRY(hipEventRecord(c1, st));
        if (n > 0) HIP_TRY(launch_scatter(in, out, n, rb, chunk, G, lpp, (const uint32_t *)c.offs.p, geo, err, st));
        SGX_TRY(debug_sync(e, st, "K4 scatter"));
    }
    HIP_TRY(hipEventRecord(x1, st));
    // (R+1) offsets then the error word, one copy
    if (host_off) HIP_TRY(hipMemcpyAsync(host_off, part_off_dev, (size_t)(R + 2) * 4, hipMemcpyDeviceToHost, st));
    if (err_slot) HIP_TRY(hipMemcpyAsync(err_slot, err, 4, hipMemcpyDeviceToDevice, st));
    if (stats) {
        e->record_stage(SGX_STAGE_HIST, h0, h1);
        e->record_stage(SGX_STAGE_SCAN, h1, c1);
        e->record_stage(SGX_STAGE_SCATTER, c1, x1);
    } else {
        e->release_events({h0, h1, c1, x1});
    }
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// single-pass padded write
// ------------------------------------------------------------------------------------
// Whether the map is written padded: hash partitioner, 16 B fixed-codec records, R within the
// write-combining K4 (<= 1024), the default kernels, no communicator at all (an exchange sends
// contiguous bytes, so a padded map would need its contiguous copy first; a one-rank
// communicator is the self-exchange stand-in for the multi-rank path and keeps its layout), big enough for
// the skipped histogram to matter, and no earlier overflow in this shuffle.
// R in (1024, 4096], a power of two: the hybrid two-level split of partition_pass, padded.
static bool split_ok(sgx_engine *e, int32_t R) {
    return R > 1024 && R <= 4096 && (R & (R - 1)) == 0 &&
           !(e->flags & (SGX_FLAG_NO_WRITE_COMBINING | SGX_FLAG_NO_SPLIT_SCATTER));
}

// TeraSort's 100 B records under a RangePartitioner over 10-byte keys take the same path with the
// LDS-staged wide-record K4 (its input 16 B-aligned, as that kernel needs).
static bool use_padded(sgx_engine *e, const Shuffle &s, const void *in, int64_t n) {
    // a Kryo shuffle's 16 B records too: the serializer reads them through the fragment table
    // and publishes its contiguous stream (the map itself is then contiguous to every consumer)
    const bool kryo16 = s.ser == SGX_SER_KRYO && s.rb == 16 && s.kind == SGX_PART_HASH;
    if (s.R < 2 || (s.ser != SGX_SER_FIXED && !kryo16) || s.combine != -1) return false;
    if (e->flags & SGX_FLAG_NO_PADDED_MAP) return false;
    if (e->rank_mode != SGX_RANK_ORDERED || !e->lds_order_ok || e->sc_waves || e->sc_items) return false;
    // a communicator sends padded maps by the direct peer gather, straight from their fragments
    // (sgx_exchange.cpp p2p_data); without it (SGX_FLAG_NO_P2P_EXCHANGE, or after the peer
    // gather could not map a peer's buffer) sends are contiguous byte ranges and the write
    // stays two-pass
    const bool comm = e->nranks > 1 || e->comm || e->host_comm;
    if ((comm && ((e->flags & SGX_FLAG_NO_P2P_EXCHANGE) || e->p2p_off.load())) || n < e->pad_min || s.pad_failed.load()) return false;
    if (s.rb == 16 && s.kind == SGX_PART_HASH && s.R > 1024)  // the padded two-level split
        return split_ok(e, s.R);
    if (s.rb == 16 && s.kind == SGX_PART_HASH)
        return !(e->flags & SGX_FLAG_NO_WRITE_COMBINING) && scatter_geom16_wc((uint32_t)s.R).items != 0;
    if (s.rb == 100 && s.kind == SGX_PART_RANGE_BYTES10)
        return !(e->flags & SGX_FLAG_NO_WIDE_STAGED) && ((uintptr_t)in & 15) == 0 &&
               scatter_geom_wide2((uint32_t)s.R, 100, s.kind, s.nb).items != 0;
    return false;
}

// The map's geometry: chunk / G exactly as partition_pass cuts them (the fallback's kernels
// and the padded kernels share it), the sample stride and the output capacity.
struct PadGeom {
    ScatterGeom geo;
    int64_t chunk = 0, sampled = 0, olim = -1;
    int G = 0, stride = 1;
};

static PadGeom pad_geom(sgx_engine *e, const Shuffle &s, int64_t n, const ChunkTable *ct = nullptr) {
    PadGeom pg;
    const int32_t R = s.R;
    if (s.rb == 16 && R > 1024) {  // the split's level 1 (its tile decides the chunks)
        pg.geo = scatter_geom16_wc((uint32_t)(SPLIT_HOT_CAP + R / 64));
        pg.geo.lds_bytes += ((size_t)R * 2 + 15) & ~(size_t)15;  // the partition -> stream table
        pg.geo.items = 8;
        pg.geo.tile = 8 * 512;
    } else {
        pg.geo = s.rb == 16 ? scatter_geom16_wc((uint32_t)R) : scatter_geom_wide2((uint32_t)R, s.rb, s.kind, s.nb);
    }
    const int tile = pg.geo.tile;
    int64_t chunk = n > 0 ? (n + e->G - 1) / e->G : 1;
    pg.chunk = (chunk + tile - 1) / tile * tile;
    pg.G = n > 0 ? (int)((n + pg.chunk - 1) / pg.chunk) : 1;
    // about 2^16 sampled groups of 8 records or more, one group in PAD_SAMPLE_STRIDE_MAX at most
    // (C1: one 128 B line in 128, 34 MB of the 4.3 GB map)
    pg.stride = (int)std::min<int64_t>(PAD_SAMPLE_STRIDE_MAX, std::max<int64_t>(1, ((n + 7) / 8) >> 16));
    pg.sampled = pad_sampled_records(n, pg.stride);
    if (ct) {  // a streaming map: its chunks, each sampled on its own (k_pad_sample)
        if (ct->chunk % tile != 0) return PadGeom{};
        pg.chunk = ct->chunk;
        pg.G = ct->G;
        pg.sampled = 0;
        for (int64_t l : ct->len) pg.sampled += pad_sampled_records(l, pg.stride);
    }
    pg.olim = pad_capacity_bound(n, R, pg.chunk, pg.G, pg.sampled);
    if (s.rb == 16 && R > 1024 && pg.olim >= 0) {
        // the level-1 scratch (cold super-partitions' sub-bins) and the output share one bound
        const int64_t o1 = pad_capacity_bound(n, R / 64, pg.chunk, pg.G, pg.sampled);
        pg.olim = o1 < 0 ? -1 : std::max(pg.olim, o1);
    }
    return pg;
}

// The hybrid two-level split (partition_pass), padded: the hot partitions --
// chosen from the sampled counts -- stream from level 1 into their final sub-bins, the others
// into sub-bins of their super-partition in a scratch buffer; level 2 reads the scratch's
// (super, chunk) fragments of 16 supers and one chunk per workgroup and writes each cold
// partition's records into ITS final sub-bin of that chunk.  Then, as in padded_pass: K3 over the final counts, and a guarded
// two-pass fallback (K1+K2, K3, the single lane-ordered K4).
#ifndef SGX_SPLIT_PRE_STREAM  // (A/B builds: 0 runs the split's front on the main stream)
#define SGX_SPLIT_PRE_STREAM 1
#endif
static int padded_split_pass(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m, const void *in, int64_t n,
                             const PadGeom &pg) {
    hipStream_t st = c.st;
    const int32_t R = s.R;
    constexpr int32_t Q = 64;
    const int32_t S = R / Q;
    constexpr int32_t HOT = SPLIT_HOT_CAP;
    const int G = pg.G;
    const int64_t len = (int64_t)R * G, tiles = scan_tiles(len);
    const uint32_t olim = (uint32_t)pg.olim;
    // this write's work slot: the tail that last read it (two writes ago) must have run.  The
    // front (sample, cut, capacities, cursors) runs on the pre stream, which waits for that
    // tail only -- not for the previous write's level 2 on the main stream -- and for the
    // input when the engine staged it on the main stream
    const int slot = c.pad_slot;
    c.pad_slot ^= 1;
    hipStream_t pre = SGX_SPLIT_PRE_STREAM ? c.st_pre : st;
    if (c.pad_done[slot].ev) HIP_TRY(hipStreamWaitEvent(pre, c.pad_done[slot].ev, 0));
    if (in == c.input_stage.p) {
        HIP_TRY(c.pre_in.record(st));
        HIP_TRY(hipStreamWaitEvent(pre, c.pre_in.ev, 0));
    }
    // the fallback's chunks (one wave each: the zero-LDS histogram and scatter)
    const int64_t chunk_fb = std::max<int64_t>(1, (n + e->G - 1) / e->G);
    const int G_fb = (int)((n + chunk_fb - 1) / chunk_fb);
    const int64_t len_fb = (int64_t)R * G_fb, tiles_fb = scan_tiles(len_fb);
    SGX_TRY(m.data.ensure((size_t)olim * 16));
    SGX_TRY(m.frag.ensure((size_t)len * 12 + 16));
    uint32_t *fstart = (uint32_t *)m.frag.p, *foff = fstart + len, *cnt = foff + len;
    SGX_TRY(c.pad_offs[slot].ensure((size_t)len_fb * 8));  // the fallback's offsets, then its cursors
    SGX_TRY(c.split_tmp.ensure((size_t)olim * 16));
    // [fallback counts][fallback ticket | status][offsets R+1 | error | padded flags]
    // [padded scan ticket | status][est R][pcap R], one memset
    auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const size_t counts_bytes = al((size_t)len_fb * 4);
    const size_t status_fb_bytes = al((size_t)(16 + tiles_fb * 8));
    const size_t off_bytes = al((size_t)(R + 3) * 4);
    const size_t status_bytes = al((size_t)(16 + tiles * 8));
    const size_t rbytes = al((size_t)R * 4);
    const size_t work_bytes = counts_bytes + status_fb_bytes + off_bytes + status_bytes + 2 * rbytes;
    SGX_TRY(c.pad_work[slot].ensure(work_bytes));
    char *w = (char *)c.pad_work[slot].p;
    uint32_t *counts_fb = (uint32_t *)w;
    uint32_t *ticket_fb = (uint32_t *)(w + counts_bytes);
    uint64_t *status_fb = (uint64_t *)((char *)ticket_fb + 16);
    uint32_t *part_off_dev = (uint32_t *)(w + counts_bytes + status_fb_bytes);
    uint32_t *err = part_off_dev + R + 1, *err_pad = part_off_dev + R + 2;
    uint32_t *ticket_pad = (uint32_t *)((char *)part_off_dev + off_bytes);
    uint64_t *status_pad = (uint64_t *)((char *)ticket_pad + 16);
    uint32_t *est = (uint32_t *)((char *)ticket_pad + status_bytes);
    uint32_t *pcap = (uint32_t *)((char *)est + rbytes);
    c.last_off_dev = part_off_dev;
    // the split's scratch: [stream_of u16 R][hot_part i32 HOT][est1 S][cap1 S][fstart1 S*G]
    // [cnt1 (HOT+S)*G][cur1 (HOT+S)*G][capS HOT+S]
    const int64_t ns = (int64_t)(HOT + S);
    const size_t b_so = al((size_t)R * 2), b_hp = al((size_t)HOT * 4), b_s = al((size_t)S * 4);
    const size_t b_sg = al((size_t)S * G * 4), b_st = al((size_t)ns * G * 4), b_cs = al((size_t)ns * 4);
    SGX_TRY(c.split_pad[slot].ensure(b_so + b_hp + 2 * b_s + b_sg + 2 * b_st + b_cs));
    char *x = (char *)c.split_pad[slot].p;
    uint16_t *stream_of = (uint16_t *)x;
    int32_t *hot_part = (int32_t *)(x += b_so);
    uint32_t *est1 = (uint32_t *)(x += b_hp);
    uint32_t *cap1 = (uint32_t *)(x += b_s);
    uint32_t *fstart1 = (uint32_t *)(x += b_s);
    uint32_t *cnt1 = (uint32_t *)(x += b_sg);
    uint32_t *cur1 = (uint32_t *)(x += b_st);
    uint32_t *capS = (uint32_t *)(x += b_st);
    hipEvent_t h0 = e->ev(), h1 = e->ev(), l0 = e->ev(), c1 = e->ev(), x1 = e->ev();
    HIP_TRY(hipEventRecord(h0, pre));
    HIP_TRY(hipMemsetAsync(w, 0, work_bytes, pre));
    HIP_TRY(launch_pad_sample(in, n, 16, pg.stride, s.pp, est, pre));
    HIP_TRY(launch_hot_select(nullptr, R, Q, stream_of, hot_part, pre, est));
    HIP_TRY(launch_pad_caps(est, R, pg.sampled, pg.chunk, G, olim, pcap, fstart, err_pad, pre));
    HIP_TRY(launch_cold_super_est(est, stream_of, S, Q, est1, pre));
    HIP_TRY(launch_pad_caps(est1, S, pg.sampled, pg.chunk, G, olim, cap1, fstart1, err_pad, pre));
    HIP_TRY(launch_hot_cursors(fstart, hot_part, fstart1, cur1, S, G, pre, pcap, cap1, capS));
    SGX_TRY(debug_sync(e, pre, "padded split: sample / selection / capacities"));
    HIP_TRY(hipEventRecord(h1, pre));
    HIP_TRY(c.pre_done[slot].record(pre));
    HIP_TRY(hipStreamWaitEvent(st, c.pre_done[slot].ev, 0));
    HIP_TRY(hipEventRecord(l0, st));
    PartParams p1 = s.pp;
    p1.kind = KIND_HOT_SPLIT;
    p1.R = (uint32_t)(HOT + S);
    p1.dshift = (uint32_t)__builtin_ctz((unsigned)R);
    p1.dir = stream_of;
    p1.mbits = (uint32_t)pg.geo.mbits;
    p1.olim = olim;
    p1.pad_cnt = cnt1;
    p1.pad_cap = capS;
    HIP_TRY(launch_scatter(in, m.data.p, n, 16, pg.chunk, G, p1, cur1, pg.geo, err_pad, st, c.split_tmp.p,
                           (uint32_t)HOT));
    SGX_TRY(debug_sync(e, st, "K4 padded split level 1"));
    // level 2: a workgroup per (group of `pack` supers, chunk), its 64 pack streams the
    // group's partitions (pid & (64 pack - 1)), the group's fragments of that chunk read back to
    // back
    const int pack = std::min<int>(S, (int)SPLIT_PACK_MAX);
    const ScatterGeom geo2 = scatter_geom16_wc((uint32_t)(Q * pack));
    PartParams p2 = s.pp;
    p2.kind = KIND_HASH_POW2;
    p2.R = (uint32_t)(Q * pack);
    p2.mbits = (uint32_t)geo2.mbits;
    p2.olim = olim;
    p2.pad_cnt = cnt;
    p2.pad_cap = pcap;
    p2.frag_start = fstart1;
    p2.frag_cnt = cnt1 + (int64_t)HOT * G;
    p2.pack = (uint32_t)pack;
    const int grid2 = (S / pack) * G;
    HIP_TRY(launch_scatter16_seg(c.split_tmp.p, m.data.p, n, p2, fstart, G, nullptr, nullptr, nullptr, grid2, geo2,
                                 err_pad, st));
    SGX_TRY(debug_sync(e, st, "K4 padded split level 2"));
    HIP_TRY(launch_hot_counts(cnt1, hot_part, G, cnt, st));
    HIP_TRY(hipEventRecord(c1, st));
    // the tail on the second stream, behind level 2: K3 over the final counts (one wave per
    // tile), then the two-pass fallback -- a histogram, a scan, a scatter, each a no-op unless
    // *err_pad has PAD_OVERFLOW -- and the offsets to the host.  Every kernel of it is LDS-free,
    // so it runs beside the next write's level 1 instead of waiting for its CUs
    hipStream_t tl = c.st_tail;
    HIP_TRY(hipStreamWaitEvent(tl, c1, 0));
    HIP_TRY(launch_scan_wave(cnt, foff, len, status_pad, ticket_pad, err, part_off_dev, G, R, tl));
    uint32_t *offs_fb = (uint32_t *)c.pad_offs[slot].p, *cur_fb = offs_fb + len_fb;
    HIP_TRY(launch_hist16_fallback(in, n, chunk_fb, G_fb, s.pp, counts_fb, err_pad, tl));
    HIP_TRY(launch_scan_wave(counts_fb, offs_fb, len_fb, status_fb, ticket_fb, err, part_off_dev, G_fb, R, tl,
                             err_pad));
    HIP_TRY(launch_scatter16_fallback(in, m.data.p, n, chunk_fb, G_fb, s.pp, offs_fb, cur_fb, err_pad, err, tl, 16));
    SGX_TRY(debug_sync(e, tl, "padded split scan / fallback"));
    HIP_TRY(hipEventRecord(x1, tl));
    HIP_TRY(hipMemcpyAsync(m.part_off.p, part_off_dev, (size_t)(R + 3) * 4, hipMemcpyDeviceToHost, tl));
    HIP_TRY(c.pad_done[slot].record(tl));
    c.tail_slot = slot;
    e->record_stage(SGX_STAGE_HIST, h0, h1);
    e->record_stage(SGX_STAGE_SCATTER, l0, c1);
    e->record_stage(SGX_STAGE_SCAN, c1, x1);
    m.pad_try = true;
    m.frag_G = G;
    return SGX_OK;
}

// 100 B TeraSort records: sample -> sub-bin capacities -> K4 into the sub-bins (final counts out) -> K3 over the
// counts (contiguous positions + index offsets), then the two-pass K1+K2 -> K3 -> K4 into the
// same buffer, every kernel of it guarded on the padded K4's overflow bit (a no-op launch
// otherwise).  Asynchronous on the context's stream; (R+1) offsets, the error word and the
// padded K4's flag word land in m.part_off.
static int padded_pass_wide(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m, const void *in, int64_t n,
                            const PadGeom &pg, const ChunkTable *ct) {
    hipStream_t st = c.st;
    const int32_t R = s.R;
    const int G = pg.G;
    const int64_t len = (int64_t)R * G, tiles = scan_tiles(len);
    const uint32_t olim = (uint32_t)pg.olim;
    const int rb = s.rb;
    // this write's work slot: the tail that last read it (two writes ago) must have run
    const int slot = c.pad_slot;
    c.pad_slot ^= 1;
    if (c.pad_done[slot].ev) HIP_TRY(hipStreamWaitEvent(st, c.pad_done[slot].ev, 0));
    SGX_TRY(m.data.ensure((size_t)olim * (size_t)rb));
    SGX_TRY(m.frag.ensure((size_t)len * 12 + 16));
    uint32_t *fstart = (uint32_t *)m.frag.p, *foff = fstart + len, *cnt = foff + len;
    SGX_TRY(c.pad_offs[slot].ensure((size_t)len * 4));
    // one work block, one memset: [fallback counts R*G][fallback ticket | status]
    // [offsets R+1 | error | padded flags][padded scan ticket | status][est R][pcap R]
    const size_t counts_bytes = ((size_t)len * 4 + 15) & ~(size_t)15;
    const size_t status_bytes = ((size_t)(16 + tiles * 8) + 15) & ~(size_t)15;
    const size_t off_bytes = ((size_t)(R + 3) * 4 + 15) & ~(size_t)15;
    const size_t rbytes = ((size_t)R * 4 + 15) & ~(size_t)15;
    const size_t work_bytes = counts_bytes + 2 * status_bytes + off_bytes + 2 * rbytes;
    SGX_TRY(c.pad_work[slot].ensure(work_bytes));
    char *w = (char *)c.pad_work[slot].p;
    uint32_t *counts_fb = (uint32_t *)w;
    uint32_t *ticket_fb = (uint32_t *)(w + counts_bytes);
    uint64_t *status_fb = (uint64_t *)((char *)ticket_fb + 16);
    uint32_t *part_off_dev = (uint32_t *)(w + counts_bytes + status_bytes);
    uint32_t *err = part_off_dev + R + 1, *err_pad = part_off_dev + R + 2;
    uint32_t *ticket_pad = (uint32_t *)((char *)part_off_dev + off_bytes);
    uint64_t *status_pad = (uint64_t *)((char *)ticket_pad + 16);
    uint32_t *est = (uint32_t *)((char *)ticket_pad + status_bytes);
    uint32_t *pcap = (uint32_t *)((char *)est + rbytes);
    uint32_t *offs_fb = (uint32_t *)c.pad_offs[slot].p;
    c.last_off_dev = part_off_dev;
    HIP_TRY(hipMemsetAsync(w, 0, work_bytes, st));
    hipEvent_t h0 = e->ev(), h1 = e->ev(), c1 = e->ev(), x1 = e->ev();
    HIP_TRY(hipEventRecord(h0, st));
    PartParams bp = s.pp;  // the shuffle's partitioner over this map's input (chunk table or not)
    bp.chunks = ct ? ct->dev : nullptr;
    HIP_TRY(launch_pad_sample(in, n, rb, pg.stride, bp, est, st, pg.chunk, G));
    HIP_TRY(launch_pad_caps(est, R, pg.sampled, pg.chunk, G, olim, pcap, fstart, err_pad, st));
    SGX_TRY(debug_sync(e, st, "padded sample / capacities"));
    HIP_TRY(hipEventRecord(h1, st));
    PartParams kp = bp;
    kp.mbits = (uint32_t)pg.geo.mbits;
    kp.olim = olim;
    kp.pad_cnt = cnt;
    kp.pad_cap = pcap;
    HIP_TRY(launch_scatter(in, m.data.p, n, rb, pg.chunk, G, kp, fstart, pg.geo, err_pad, st));
    SGX_TRY(debug_sync(e, st, "K4 padded scatter"));
    HIP_TRY(hipEventRecord(c1, st));
    // the tail on the second stream, behind K4: K3 over the counts, then the two-pass
    // fallback, each kernel a no-op unless *err_pad has PAD_OVERFLOW, and the offsets to the host
    hipStream_t tl = c.st_tail;
    HIP_TRY(hipStreamWaitEvent(tl, c1, 0));
    HIP_TRY(launch_scan(cnt, foff, len, status_pad, ticket_pad, err, part_off_dev, G, R, tl));
    PartParams fp = bp;
    fp.guard = err_pad;
    HIP_TRY(launch_hist(in, n, rb, pg.chunk, G, fp, counts_fb, tl, e->hist_mode, true));
    HIP_TRY(launch_scan(counts_fb, offs_fb, len, status_fb, ticket_fb, err, part_off_dev, G, R, tl, err_pad));
    fp.mbits = (uint32_t)pg.geo.mbits;
    HIP_TRY(launch_scatter(in, m.data.p, n, rb, pg.chunk, G, fp, offs_fb, pg.geo, err, tl));
    SGX_TRY(debug_sync(e, tl, "padded scan / fallback"));
    HIP_TRY(hipEventRecord(x1, tl));
    HIP_TRY(hipMemcpyAsync(m.part_off.p, part_off_dev, (size_t)(R + 3) * 4, hipMemcpyDeviceToHost, tl));
    HIP_TRY(c.pad_done[slot].record(tl));
    c.tail_slot = slot;
    // stages: the sampled histogram stands where K1+K2 do, the scans (and the no-op fallback
    // launches) where K3 does
    e->record_stage(SGX_STAGE_HIST, h0, h1);
    e->record_stage(SGX_STAGE_SCATTER, h1, c1);
    e->record_stage(SGX_STAGE_SCAN, c1, x1);
    m.pad_try = true;
    m.frag_G = G;
    return SGX_OK;
}

// 16 B records (the write-combining K4): sample -> K4, which lays the sub-bins out itself from
// the sampled counts and writes every stream into its sub-bin (end positions out), on the
// context's stream -- nothing else runs ahead of the next write's K4.  Then, on the tail
// stream behind K4: the fragment table and the streams' counts (k_pad_finish, which also
// checks them against their capacities), K3 over the counts (contiguous positions + index
// offsets), the slot's reset for its next sample, and the overflow fallback (a no-op launch
// that takes no LDS unless a sub-bin overflowed).  Asynchronous; (R+1) offsets, the error
// word and the padded flag word land in m.part_off.
static int padded_pass16(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m, const void *in, int64_t n, const PadGeom &pg,
                         const ChunkTable *ct) {
    const int rb = s.rb;  // 16, or 100 (TeraSort's write-combining K4: wide_wc_padded_ok)
    const int32_t R = s.R;
    const int G = pg.G;
    const int64_t len = (int64_t)R * G, tiles = scan_tiles(len);
    const uint32_t olim = (uint32_t)pg.olim;
    auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
    // this write's slot: its sample block is free once the tail two writes ago reset it; the
    // rest of the slot is the tail stream's own (in order)
    const int slot = c.pad_slot;
    c.pad_slot ^= 1;
    // Overlapping writes (the default; sgx_set_overlap_writes): consecutive writes alternate
    // between two streams (slot 1 on the
    // pre stream, which the R > 1024 split uses for its front), so a write's sample and K4 start
    // on the CUs the previous write's last K4 workgroups leave, instead of behind its whole
    // grid (C1 1.794 -> 1.772 ms per write, C4 1.663 -> 1.634, profiles/r06/r06w_*; kernel
    // traces then time a K4 from its dispatch, waiting included: r06x).  A write on the pre
    // stream waits for what the call put on the main stream for it: the input's staging copy
    // and the all-to-all still reading the map's old bytes (a streaming commit's landing
    // copies: the whole main stream).
    hipStream_t st = c.st;
    if (e->overlap_writes.load() && slot == 1) {
        st = c.st_pre;
        if (ct || in == c.input_stage.p) {
            HIP_TRY(c.pre_in.record(c.st));
            HIP_TRY(hipStreamWaitEvent(st, c.pre_in.ev, 0));
        }
        if (m.read_done.ev) HIP_TRY(hipStreamWaitEvent(st, m.read_done.ev, 0));
    }
    if (c.pad_free[slot].ev) HIP_TRY(hipStreamWaitEvent(st, c.pad_free[slot].ev, 0));
    SGX_TRY(m.data.ensure((size_t)olim * (size_t)rb));
    SGX_TRY(m.frag.ensure((size_t)len * 12 + 16));
    uint32_t *fstart = (uint32_t *)m.frag.p, *foff = fstart + len, *cnt = foff + len;
    SGX_TRY(c.pad_offs[slot].ensure((size_t)len * 4));
    // the sample's block: [est R][flags | pad][layout: caps R, bases R]; est and flags are zero
    // when the sample starts (the slot's last tail reset them)
    const size_t rbytes = al((size_t)R * 4), zero_bytes = rbytes + 16;
    if (c.pad_crit[slot].cap < zero_bytes + 2 * rbytes) c.pad_crit_zeroed[slot] = 0;
    SGX_TRY(c.pad_crit[slot].ensure(zero_bytes + 2 * rbytes));
    char *cb = (char *)c.pad_crit[slot].p;
    uint32_t *est = (uint32_t *)cb, *flags = (uint32_t *)(cb + rbytes), *layout = (uint32_t *)(cb + zero_bytes);
    if (c.pad_crit_zeroed[slot] < zero_bytes) HIP_TRY(hipMemsetAsync(cb, 0, zero_bytes, st));
    c.pad_crit_zeroed[slot] = 0;  // until this write's tail has reset it
    // the tail's block: [offsets R+1 | error | flags copy][scan ticket | status]; k_pad_finish
    // zeroes what the scan needs zero: everything from the error word on
    const size_t off_bytes = al((size_t)(R + 3) * 4);
    const size_t status_bytes = al((size_t)(16 + tiles * 8));
    SGX_TRY(c.pad_work[slot].ensure(off_bytes + status_bytes));
    char *w = (char *)c.pad_work[slot].p;
    uint32_t *part_off_dev = (uint32_t *)w;
    uint32_t *err = part_off_dev + R + 1, *flags_copy = part_off_dev + R + 2;
    uint32_t *ticket_pad = (uint32_t *)(w + off_bytes);
    uint64_t *status_pad = (uint64_t *)((char *)ticket_pad + 16);
    c.last_off_dev = part_off_dev;
    hipEvent_t h0 = e->ev(), h1 = e->ev(), c1 = e->ev(), x1 = e->ev();
    HIP_TRY(hipEventRecord(h0, st));
    PartParams bp = s.pp;  // the shuffle's partitioner over this map's input (chunk table or not)
    bp.chunks = ct ? ct->dev : nullptr;
    HIP_TRY(launch_pad_sample(in, n, rb, pg.stride, bp, est, st, pg.chunk, G));
    SGX_TRY(debug_sync(e, st, "padded sample"));
    HIP_TRY(hipEventRecord(h1, st));
    PartParams kp = bp;
    kp.mbits = (uint32_t)pg.geo.mbits;
    kp.olim = olim;
    kp.pad_cnt = cnt;
    kp.pad_est = est;
    kp.pad_layout = layout;
    kp.pad_scale = (double)pg.chunk / (double)pg.sampled;
    kp.pad_a = 1.0 + kp.pad_scale;
    HIP_TRY(launch_scatter(in, m.data.p, n, rb, pg.chunk, G, kp, nullptr, pg.geo, flags, st));
    SGX_TRY(debug_sync(e, st, "K4 padded scatter"));
    HIP_TRY(hipEventRecord(c1, st));
    hipStream_t tl = c.st_tail;
    HIP_TRY(hipStreamWaitEvent(tl, c1, 0));
    HIP_TRY(launch_pad_finish(layout, R, G, olim, fstart, cnt, flags, err,
                              (int64_t)((off_bytes + status_bytes) / 4) - (R + 1), tl));
    HIP_TRY(launch_scan_wave(cnt, foff, len, status_pad, ticket_pad, err, part_off_dev, G, R, tl));
    HIP_TRY(launch_pad_reset(flags, flags_copy, est, R, tl));
    HIP_TRY(c.pad_free[slot].record(tl));
    c.pad_crit_zeroed[slot] = zero_bytes;
    HIP_TRY(launch_scatter16_fallback(in, m.data.p, n, pg.chunk, G, bp, foff, (uint32_t *)c.pad_offs[slot].p,
                                      flags_copy, err, tl, rb));
    SGX_TRY(debug_sync(e, tl, "padded tail"));
    HIP_TRY(hipEventRecord(x1, tl));
    HIP_TRY(hipMemcpyAsync(m.part_off.p, part_off_dev, (size_t)(R + 3) * 4, hipMemcpyDeviceToHost, tl));
    HIP_TRY(c.pad_done[slot].record(tl));
    c.tail_slot = slot;
    // stages: the sampled histogram stands where K1+K2 do, the tail where K3 does
    e->record_stage(SGX_STAGE_HIST, h0, h1);
    e->record_stage(SGX_STAGE_SCATTER, h1, c1);
    e->record_stage(SGX_STAGE_SCAN, c1, x1);
    m.pad_try = true;
    m.frag_G = G;
    return SGX_OK;
}

static int padded_pass(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m, const void *in, int64_t n, const PadGeom &pg,
                       const ChunkTable *ct = nullptr) {
    const bool own_layout = s.rb == 16 || wide_wc_padded_ok((uint32_t)s.R, s.nb, pg.chunk);
    return own_layout ? padded_pass16(e, c, s, m, in, n, pg, ct) : padded_pass_wide(e, c, s, m, in, n, pg, ct);
}

int sgx::materialize(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m) {
    if (!m.padded || m.dense_valid) return SGX_OK;
    const int32_t R = s.R;
    const int G = m.frag_G;
    const uint32_t *po = (const uint32_t *)m.part_off.p;
    SGX_TRY(m.dense.ensure((size_t)std::max<int64_t>(m.nrec * s.rb, 16)));
    std::vector<int64_t> desc((size_t)R * FRAG_DESC_WORDS);
    const int64_t len = (int64_t)R * G;
    const uint32_t *fstart = (const uint32_t *)m.frag.p;
    for (int32_t p = 0; p < R; ++p) {
        int64_t *d = &desc[(size_t)p * FRAG_DESC_WORDS];
        d[0] = (int64_t)(uintptr_t)m.data.p;
        d[1] = (int64_t)(uintptr_t)fstart;
        d[2] = (int64_t)(uintptr_t)(fstart + len);
        d[3] = (int64_t)(uintptr_t)(fstart + 2 * len);
        d[4] = (int64_t)(uintptr_t)((char *)m.dense.p + (size_t)po[p] * (size_t)s.rb);
        d[5] = p;
        d[6] = G;
        d[7] = s.rb;
    }
    SGX_TRY(c.items_dev.ensure(desc.size() * 8));
    HIP_TRY(hipStreamWaitEvent(c.st, m.done.ev, 0));
    HIP_TRY(hipMemcpyAsync(c.items_dev.p, desc.data(), desc.size() * 8, hipMemcpyHostToDevice, c.st));
    HIP_TRY(launch_gather_frags((const int64_t *)c.items_dev.p, R, G, c.st));
    SGX_TRY(debug_sync(e, c.st, "k_gather_frags (contiguous copy)"));
    HIP_TRY(m.done.record(c.st));
    HIP_TRY(hipStreamSynchronize(c.st));  // the descriptors are host memory of this frame
    m.dense_valid = true;
    return SGX_OK;
}

// Kryo framing of the partition-contiguous 16 B records just written (sgx_serde.hip), on
// the context's stream behind the scatter; byte offsets land in m.ser_off (pinned).
// rec_off_dev: device (R+1) u32 record offsets of m.data.
// rec_off_dev: (nseg+1) u32 record offsets of the stream's segments (the R partitions, or
// the (partition, spill) segments of SGX_WRITER_UNSAFE).
static int serialize_kryo(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m, const uint32_t *rec_off_dev, int32_t nseg,
                          bool padded = false) {
    hipStream_t st = c.st;
    const int64_t n = m.nrec;
    const int64_t tiles = kryo_ser16_tiles(n);
    const size_t offb = (size_t)(nseg + 1) * 8;
    SGX_TRY(m.ser.ensure((size_t)(20 * n + 16)));
    SGX_TRY(m.ser_work.ensure(offb + (size_t)kryo_work_bytes(tiles)));
    SGX_TRY(m.ser_off.ensure(offb));
    int64_t *off_dev = (int64_t *)m.ser_work.p;
    uint64_t *work = (uint64_t *)((char *)m.ser_work.p + offb);
    if (n == 0) HIP_TRY(hipMemsetAsync(off_dev, 0, offb, st));  // no tile writes them
    hipEvent_t k0 = e->ev(), k1 = e->ev();
    HIP_TRY(hipEventRecord(k0, st));
    // a padded write's records through its fragment table, unless its fallback ran (the flag
    // word behind the partition offsets: padded_pass / padded_split_pass)
    const int64_t nfrag = padded ? (int64_t)s.R * m.frag_G : 0;
    HIP_TRY(launch_kryo_ser16(m.data.p, n, m.ser.p, rec_off_dev, nseg, off_dev, work, st,
                              padded ? (const uint32_t *)m.frag.p : nullptr, nfrag,
                              padded ? rec_off_dev + s.R + 2 : nullptr));
    SGX_TRY(debug_sync(e, st, "Kryo serializer"));
    HIP_TRY(hipEventRecord(k1, st));
    e->record_stage(SGX_STAGE_SERIALIZE, k0, k1);
    HIP_TRY(hipMemcpyAsync(m.ser_off.p, off_dev, offb, hipMemcpyDeviceToHost, st));  // (nseg+1) byte offsets
    m.ser_valid = true;
    return SGX_OK;
}

// Map-side combine, SGX_AGG_SUM (ExternalSorter.insertAll with the aggregator's
// mergeValue; the canonical combiner order is (partition, key ascending)): the n records at
// `in` (device) are copied to the context's sort buffer, sorted stably by key and then by
// the shuffle's partitioner (LSD digit passes + one partition pass, sgx_read.cpp), grouped,
// summed (wrapping), packed back into {key, sum} records and partitioned into m.data (an
// identity permutation that yields the partition offsets through the usual machinery).
// Synchronous (the group count decides the output size).
static int combine_sum(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m, const void *in, int64_t n) {
    hipStream_t st = c.st;
    hipEvent_t t0 = e->ev(), t1 = e->ev();
    HIP_TRY(hipEventRecord(t0, st));
    SGX_TRY(c.sort_buf[0].ensure((size_t)std::max<int64_t>(n, 1) * 16));
    SGX_TRY(c.sort_buf[1].ensure((size_t)std::max<int64_t>(n, 1) * 16));
    if (n > 0) HIP_TRY(hipMemcpyAsync(c.sort_buf[0].p, in, (size_t)n * 16, hipMemcpyDeviceToDevice, st));
    const void *sorted = c.sort_buf[0].p;
    int64_t ng = 0;
    int64_t *keys = nullptr, *sums = nullptr;
    if (n > 0) {
        SGX_TRY(sort_records(e, c, s, n, true, &sorted));
        SGX_TRY(group_records(e, c, sorted, n, SGX_AGG_SUM, &ng, &keys, nullptr, &sums));
    }
    SGX_TRY(c.comb_buf.ensure((size_t)std::max<int64_t>(ng, 1) * 16));
    HIP_TRY(launch_pack_pairs(keys, sums, ng, c.comb_buf.p, st));
    m.nrec = ng;
    SGX_TRY(m.data.ensure((size_t)std::max<int64_t>(ng, 1) * 16));
    SGX_TRY(partition_pass(e, c, c.comb_buf.p, m.data.p, ng, 16, s.pp, s.R, s.kind, (uint32_t *)m.part_off.p,
                           nullptr, false));
    HIP_TRY(hipEventRecord(t1, st));
    e->record_stage(SGX_STAGE_COMBINE, t0, t1);
    return SGX_OK;
}

// After the records of a map are known (device `in`, n records, or already partitioned in
// m.data when `partitioned`): partition / combine, then frame.  Asynchronous except for the
// combine.  m.done is recorded behind the last kernel.
// ct: a streaming map's batches (deferred commit) as the input's chunks; the padded write
// then needs no_pad false, and a Kryo map framed per (partition, spill) segment (seg_spills > 1)
// gets its segment offsets from the pass's per-(partition, chunk) offsets (g0: each batch's
// first chunk, device).
static int run_map_pipeline(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m, const void *in, int64_t n,
                            bool partitioned, const uint32_t *part_dev, const ChunkTable *ct = nullptr,
                            bool no_pad = false, const int32_t *g0_dev = nullptr) {
    m.ready = false;
    m.ser_valid = false;
    m.comp_valid = false;
    m.pad_try = m.padded = m.rec_padded = m.dense_valid = false;
    const uint32_t *rec_off_dev = part_dev;
    int tail = -1;  // the padded write left its tail on c.st_tail (this slot's pad_done)
    PadGeom pg;
    if (!partitioned && !no_pad && use_padded(e, s, in, n)) pg = pad_geom(e, s, n, ct);
    if (s.combine == SGX_AGG_SUM) {
        SGX_TRY(combine_sum(e, c, s, m, partitioned ? m.data.p : in, n));
        rec_off_dev = c.last_off_dev;
    } else if (!partitioned && pg.olim >= n) {
        m.nrec = n;
        if (s.rb == 16 && s.R > 1024 && !ct) {
            SGX_TRY(padded_split_pass(e, c, s, m, in, n, pg));
        } else {
            SGX_TRY(padded_pass(e, c, s, m, in, n, pg, ct));
        }
        tail = c.tail_slot;
        rec_off_dev = c.last_off_dev;
    } else if (!partitioned) {
        m.nrec = n;
        SGX_TRY(m.data.ensure((size_t)std::max<int64_t>(n * s.rb, 16)));
        SGX_TRY(partition_pass(e, c, in, m.data.p, n, s.rb, s.pp, s.R, s.kind, (uint32_t *)m.part_off.p, nullptr,
                               true, ct));
        rec_off_dev = c.last_off_dev;
        if (ct && m.seg_spills > 1) {  // (partition, spill) segments from the (partition, chunk) offsets
            SGX_TRY(m.seg_off.ensure((size_t)((int64_t)s.R * m.seg_spills + 1) * 4));
            HIP_TRY(launch_spill_seg_offs((const uint32_t *)c.offs.p, rec_off_dev, s.R, n > 0 ? ct->G : 0,
                                          m.seg_spills, g0_dev, (uint32_t *)m.seg_off.p, c.st));
        }
    }
    if (s.ser == SGX_SER_KRYO && tail >= 0) {  // the serializer reads the tail's final bytes / offsets
        HIP_TRY(hipStreamWaitEvent(c.st, c.pad_done[tail].ev, 0));
        tail = -1;
    }
    if (s.ser == SGX_SER_KRYO) {
        if (m.seg_spills > 1)  // (partition, spill) segments, SGX_WRITER_UNSAFE
            SGX_TRY(serialize_kryo(e, c, s, m, (const uint32_t *)m.seg_off.p, s.R * m.seg_spills));
        else
            SGX_TRY(serialize_kryo(e, c, s, m, rec_off_dev, s.R, m.pad_try));
    }
    // the map is complete behind its last kernel: the tail's, when nothing followed it
    HIP_TRY(m.done.record(tail >= 0 ? c.st_tail : c.st));
    m.written = true;
    return SGX_OK;
}

int sgx::finish_lengths(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m) {
    if (m.ready) return SGX_OK;
    if (!m.written) return fail_msg(SGX_ERR_STATE, "map output was not committed");
    HIP_TRY(m.done.wait_host());
    if (m.deferred) {  // the commit's pass has read the batches
        m.spills.clear();
        m.landing.clear();
        m.land_used = 0;
    }
    const uint32_t *po = (const uint32_t *)m.part_off.p;
    if (m.pad_try) {
        // the padded write's own flag word: an overflow means the guarded two-pass fallback
        // rewrote the map contiguous (its errors are in the main word, checked below)
        const uint32_t fl = po[s.R + 2];
        const bool ovf = (fl & PAD_OVERFLOW) != 0;
        if (!ovf && fl) return fail_msg(SGX_ERR_HIP, "internal error: padded scatter flag %#x", fl);
        // (a Kryo map publishes its serialized stream: contiguous whatever its records were)
        m.padded = !ovf && s.ser == SGX_SER_FIXED;
        m.rec_padded = !ovf;
        if (ovf) s.pad_failed.store(true);
        m.pad_try = false;
    }
    if (po[s.R + 1] & 1u)
        return fail_msg(SGX_ERR_TIMEOUT, "scan look-back spin gave up (device flag %u)", po[s.R + 1]);
    if (po[s.R + 1] & 2u)
        return fail_msg(SGX_ERR_HIP, "internal error: a scatter destination was out of range (device flag %u)",
                        po[s.R + 1]);
    if ((int64_t)po[s.R] != m.nrec)
        return fail_msg(SGX_ERR_HIP, "partition offsets do not sum to the record count (%u vs %lld)", po[s.R],
                        (long long)m.nrec);
    m.lengths.assign((size_t)s.R, 0);
    const int32_t S = s.ser == SGX_SER_KRYO ? m.seg_spills : 1;  // segments per partition
    if (s.ser == SGX_SER_KRYO) {
        const int64_t *so = (const int64_t *)m.ser_off.p;
        int64_t prev = 0;
        for (int32_t p = 0; p < s.R; ++p) {
            m.lengths[(size_t)p] = so[(size_t)(p + 1) * S] - so[(size_t)p * S];
            if (so[(size_t)p * S] != prev || m.lengths[(size_t)p] < 0 ||
                m.lengths[(size_t)p] > 20 * ((int64_t)po[p + 1] - po[p]))
                return fail_msg(SGX_ERR_HIP, "internal error: Kryo partition offsets inconsistent at %d", p);
            prev = so[(size_t)(p + 1) * S];
        }
        m.out_bytes = so[(size_t)s.R * S];
    } else {
        for (int32_t p = 0; p < s.R; ++p) m.lengths[(size_t)p] = ((int64_t)po[p + 1] - (int64_t)po[p]) * s.rb;
        m.out_bytes = m.nrec * s.rb;
    }
    if (s.lz4_block > 0) {  // publish the LZ4-framed partition streams instead
        // the source is this write's Kryo stream, named explicitly: `comp` may still hold an
        // earlier attempt's frames
        // one LZ4 stream per segment: a partition (SortShuffleWriter), or a (partition, spill)
        // segment whose streams the partition concatenates in spill order (UnsafeShuffleWriter's
        // fast merge); the frames land partition-major, spill-minor
        const void *src = m.ser_valid ? m.ser.p : m.data.p;
        const int32_t nseg = s.R * S;
        std::vector<int64_t> offs((size_t)nseg + 1, 0);
        const int64_t *so = (const int64_t *)m.ser_off.p;
        if (S > 1) {
            for (int32_t i = 0; i <= nseg; ++i) offs[(size_t)i] = so[i];
        } else {
            for (int32_t p = 0; p < s.R; ++p) offs[(size_t)p + 1] = offs[(size_t)p] + m.lengths[(size_t)p];
        }
        std::vector<int64_t> clen((size_t)nseg, 0);
        m.comp_valid = false;
        SGX_TRY(lz4_frame_impl(e, c, src, offs.data(), nseg, s.lz4_block, &m.comp, nullptr, 0, clen.data()));
        int64_t total = 0;
        for (int32_t p = 0; p < s.R; ++p) {
            int64_t l = 0;
            for (int32_t b = 0; b < S; ++b) l += clen[(size_t)p * S + b];
            m.lengths[(size_t)p] = l;
            total += l;
        }
        m.out_bytes = total;
        m.comp_valid = true;
    }
    m.ready = true;
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// the map output slot of a (re-)attempt
// ------------------------------------------------------------------------------------
// A re-attempt of the same map replaces the previous output (the in-HBM analogue of the
// index commit; the file commit keeps "first valid attempt wins", sgx_write_index).  The
// slot's buffers are reused when nobody else holds the old output; otherwise (a reader or an
// exchange round still references it) a fresh output takes the slot and the old one lives
// until its last reference drops.  Returns with m->mu locked (lk).
static int claim_slot(Shuffle &s, int64_t map_id, std::shared_ptr<MapOut> *pm, std::unique_lock<std::mutex> *lk) {
    std::lock_guard<std::mutex> sl(s.mu);
    std::shared_ptr<MapOut> &slot = s.maps[map_id];
    if (!slot || slot.use_count() > 1) slot = std::make_shared<MapOut>();
    *pm = slot;
    *lk = std::unique_lock<std::mutex>(slot->mu);
    return SGX_OK;
}

static void drop_slot(Shuffle &s, int64_t map_id, const std::shared_ptr<MapOut> &m) {
    std::lock_guard<std::mutex> sl(s.mu);
    auto it = s.maps.find(map_id);
    if (it != s.maps.end() && it->second == m) s.maps.erase(it);
}

static int check_batch(const Shuffle &s, const void *records, int64_t n, int32_t rb, int32_t mem_kind) {
    if (rb != s.rb) return fail_msg(SGX_ERR_INVALID, "record_bytes %d != registered %d", rb, s.rb);
    if (n < 0 || n >= (int64_t)UINT32_MAX) return fail_msg(SGX_ERR_INVALID, "nrecords %lld out of range", (long long)n);
    if (n > 0 && !records) return fail_msg(SGX_ERR_INVALID, "records is NULL");
    if (mem_kind != SGX_MEM_HOST && mem_kind != SGX_MEM_DEVICE && mem_kind != SGX_MEM_DEVICE_RETAINED)
        return fail_msg(SGX_ERR_INVALID, "unknown mem_kind %d", mem_kind);
    return SGX_OK;
}

// device pointer of a batch (host batches are staged through the context's buffer)
static int device_input(Ctx &c, const void *records, int64_t bytes, int32_t mem_kind, const void **in) {
    *in = records;
    if (mem_kind == SGX_MEM_HOST && bytes > 0) SGX_TRY(c.stage_input(records, (size_t)bytes, c.st, in));
    return SGX_OK;
}

extern "C" int sgx_write_map(sgx_engine *e, int32_t shuffle_id, int64_t map_id, const void *records,
                             int64_t n, int32_t rb, int32_t mem_kind, int64_t *out_lengths) {
    sgx::TraceRange trace_("sgx_write_map");
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    SGX_TRY(check_batch(*s, records, n, rb, mem_kind));
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    std::shared_ptr<MapOut> m;
    std::unique_lock<std::mutex> lk;
    SGX_TRY(claim_slot(*s, map_id, &m, &lk));
    // the previous attempt's kernels and any all-to-all still reading its bytes come first
    HIP_TRY(m->done.wait_host());
    if (m->read_done.ev) HIP_TRY(hipStreamWaitEvent(c->st, m->read_done.ev, 0));
    m->written = false;
    m->exchanged = false;
    m->open = false;
    m->deferred = false;
    m->spills.clear();
    m->seg_spills = 1;
    SGX_TRY(m->part_off.ensure((size_t)(s->R + 3) * 4));
    const void *in = nullptr;
    int rc = device_input(*c, records, n * rb, mem_kind, &in);
    if (rc == SGX_OK) rc = run_map_pipeline(e, *c, *s, *m, in, n, false, nullptr);
    if (rc == SGX_OK && out_lengths) {
        rc = finish_lengths(e, *c, *s, *m);
        if (rc == SGX_OK) std::memcpy(out_lengths, m->lengths.data(), sizeof(int64_t) * (size_t)s->R);
    }
    if (rc != SGX_OK && !m->written) {
        lk.unlock();
        drop_slot(*s, map_id, m);
    }
    return rc;
}

// ------------------------------------------------------------------------------------
// streaming map outputs
// ------------------------------------------------------------------------------------
// Deferred batches: sgx_map_append only lands the batch in HBM (a host batch
// through PCIe, a device batch copied, a retained device batch not at all) and the commit
// partitions every batch in ONE pass, with a chunk table in place of a contiguous input --
// the padded single-pass write where sgx_write_map would take it, else the two-pass one.  The
// map-side kernels that take a chunk table: the write-combining 16 B K4 (hash, R <= 1024) and
// the wide-record K4s (TeraSort), with their histogram and sample.
static bool deferred_ok(sgx_engine *e, const Shuffle &s) {
    if ((e->flags & SGX_FLAG_NO_DEFERRED_APPEND) || s.combine != -1) return false;
    if (e->rank_mode != SGX_RANK_ORDERED || !e->lds_order_ok || e->sc_waves || e->sc_items) return false;
    if (s.rb == 16 && s.kind == SGX_PART_HASH && s.R <= 1024)
        return !(e->flags & SGX_FLAG_NO_WRITE_COMBINING) && scatter_geom16_wc((uint32_t)s.R).items != 0;
    if (s.rb == 100 && s.kind == SGX_PART_RANGE_BYTES10)
        return !(e->flags & SGX_FLAG_NO_WIDE_STAGED) && scatter_geom_wide2((uint32_t)s.R, 100, s.kind, s.nb).items != 0;
    return false;
}

// the deferred commit's landing segments, and the pinned staging pieces of host batches
constexpr size_t LANDING_SEGMENT_BYTES = 512ull << 20;
constexpr int64_t HOST_STAGE_BYTES = 64ll << 20;

// the K4 tile the deferred commit cuts its chunks on (partition_pass / pad_geom pick the same
// geometry for these shuffles)
static int deferred_tile(const Shuffle &s) {
    return s.rb == 16 ? scatter_geom16_wc((uint32_t)s.R).tile : scatter_geom_wide2((uint32_t)s.R, 100, s.kind, s.nb).tile;
}

// The commit of deferred batches: chunks of at most `chunk` records (the map cut like one
// contiguous batch: about one per CU, a multiple of the tile), every batch into chunks of
// its own, the last one partial; byte offsets from the first non-empty batch.  The table
// ([2G] i64, then [S] i32 first chunk of every batch) goes to the device on the context's
// stream from the map's pinned buffer.
static int commit_deferred(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m, int64_t total) {
    const int rb = s.rb;
    const int32_t S = (int32_t)m.spills.size();
    const void *base = nullptr;
    for (auto &sp : m.spills)
        if (sp->nrec > 0) {
            base = sp->src;
            break;
        }
    m.seg_spills = (s.writer == SGX_WRITER_UNSAFE && s.ser == SGX_SER_KRYO && s.lz4_block > 0 && S > 1) ? S : 1;
    if (total == 0) {
        m.open = false;
        if (m.seg_spills > 1) {  // every (partition, spill) segment is empty
            const size_t sb = (size_t)((int64_t)s.R * m.seg_spills + 1) * 4;
            SGX_TRY(m.seg_off.ensure(sb));
            HIP_TRY(hipMemsetAsync(m.seg_off.p, 0, sb, c.st));
        }
        return run_map_pipeline(e, c, s, m, nullptr, 0, false, nullptr);
    }
    const int tile = deferred_tile(s);
    int64_t chunk = (total + e->G - 1) / e->G;
    chunk = (chunk + tile - 1) / tile * tile;
    ChunkTable ct;
    ct.chunk = chunk;
    std::vector<int64_t> tab;
    std::vector<int32_t> g0((size_t)S, 0);
    // regions: a batch, or a run of landed batches back to back in one landing segment (one
    // region, chunked as if one batch) -- except for per-(partition, spill) framing, which
    // needs every batch's first chunk
    struct Region {
        const char *src;
        int64_t nrec;
    };
    std::vector<Region> regions;
    for (int32_t b = 0; b < S; ++b) {
        const Spill &sp = *m.spills[(size_t)b];
        if (sp.nrec == 0) continue;
        const char *src = (const char *)sp.src;
        if (m.seg_spills == 1 && sp.landed && b > 0 && m.spills[(size_t)b - 1]->landed && !regions.empty() &&
            regions.back().src + regions.back().nrec * rb == src) {
            regions.back().nrec += sp.nrec;
            continue;
        }
        regions.push_back(Region{src, sp.nrec});
    }
    for (int32_t b = 0, r = 0; b < S; ++b) {  // first chunk of every batch (per-batch regions)
        g0[(size_t)b] = (int32_t)ct.len.size();
        if (m.seg_spills > 1 && m.spills[(size_t)b]->nrec > 0) {
            const Region &rg = regions[(size_t)r++];
            for (int64_t j = 0; j < rg.nrec; j += chunk) {
                tab.push_back((int64_t)(rg.src - (const char *)base) + j * rb);
                tab.push_back(std::min<int64_t>(chunk, rg.nrec - j));
                ct.len.push_back(tab.back());
            }
        }
    }
    if (m.seg_spills == 1)
        for (const Region &rg : regions)
            for (int64_t j = 0; j < rg.nrec; j += chunk) {
                tab.push_back((int64_t)(rg.src - (const char *)base) + j * rb);
                tab.push_back(std::min<int64_t>(chunk, rg.nrec - j));
                ct.len.push_back(tab.back());
            }
    ct.G = (int)ct.len.size();
    const size_t tb = tab.size() * 8, bytes = tb + (size_t)S * 4;
    SGX_TRY(m.chunk_host.ensure(bytes));
    SGX_TRY(m.chunk_dev.ensure(bytes));
    std::memcpy(m.chunk_host.p, tab.data(), tb);
    std::memcpy((char *)m.chunk_host.p + tb, g0.data(), (size_t)S * 4);
    HIP_TRY(hipMemcpyAsync(m.chunk_dev.p, m.chunk_host.p, bytes, hipMemcpyHostToDevice, c.st));
    ct.dev = (const int64_t *)m.chunk_dev.p;
    m.open = false;
    // UnsafeShuffleWriter's per-(partition, spill) LZ4 streams need contiguous records (the
    // serializer's segment offsets come from the two-pass scan)
    SGX_TRY(run_map_pipeline(e, c, s, m, base, total, false, nullptr, &ct, m.seg_spills > 1,
                             (const int32_t *)((const char *)m.chunk_dev.p + tb)));
    return SGX_OK;
}

extern "C" int sgx_map_begin(sgx_engine *e, int32_t shuffle_id, int64_t map_id) {
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    HIP_TRY(hipSetDevice(e->device));
    std::shared_ptr<MapOut> m;
    std::unique_lock<std::mutex> lk;
    SGX_TRY(claim_slot(*s, map_id, &m, &lk));
    HIP_TRY(m->done.wait_host());
    if (m->read_done.ev) HIP_TRY(m->read_done.wait_host());
    m->written = false;
    m->exchanged = false;
    m->ready = false;
    m->open = true;
    m->deferred = false;
    m->seg_spills = 1;
    m->spills.clear();
    m->landing.clear();
    m->land_used = 0;
    return SGX_OK;
}

extern "C" int sgx_map_append(sgx_engine *e, int32_t shuffle_id, int64_t map_id, const void *records, int64_t n,
                              int32_t rb, int32_t mem_kind) {
    sgx::TraceRange trace_("sgx_map_append");
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    std::shared_ptr<Shuffle> s;
    std::shared_ptr<MapOut> m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    SGX_TRY(check_batch(*s, records, n, rb, mem_kind));
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!m->open) return fail_msg(SGX_ERR_STATE, "map %lld of shuffle %d is not open (sgx_map_begin)",
                                  (long long)map_id, shuffle_id);
    if (m->spills.empty()) m->deferred = deferred_ok(e, *s);
    std::unique_ptr<Spill> sp(new Spill());
    sp->nrec = n;
    if (m->deferred) {  // land the batch; the commit partitions every batch in one pass
        const int64_t bytes = n * rb;
        if (mem_kind == SGX_MEM_DEVICE_RETAINED && ((uintptr_t)records & 15) == 0) {
            sp->src = records;  // read in place at the commit
        } else if (bytes > 0) {
            // into the landing area, right behind the last landed batch (16 B-aligned starts)
            if (m->landing.empty() || m->landing.back()->cap < m->land_used + (size_t)bytes) {
                std::unique_ptr<DevBuf> seg(new DevBuf());
                SGX_TRY(seg->ensure(std::max<size_t>((size_t)bytes, LANDING_SEGMENT_BYTES)));
                m->landing.push_back(std::move(seg));
                m->land_used = 0;
            }
            char *dst = (char *)m->landing.back()->p + m->land_used;
            m->land_used += ((size_t)bytes + 15) & ~(size_t)15;
            if (mem_kind == SGX_MEM_HOST) {
                // through the two pinned buffers: the copy to HBM runs while the caller fills
                // its next batch (the caller's buffer is free once it is in pinned memory)
                for (int64_t off = 0; off < bytes; off += HOST_STAGE_BYTES) {
                    const size_t piece = (size_t)std::min<int64_t>(HOST_STAGE_BYTES, bytes - off);
                    const int slot = c->host_slot;
                    c->host_slot ^= 1;
                    HIP_TRY(c->host_up[slot].wait_host());
                    SGX_TRY(c->host_stage[slot].ensure(piece));
                    host_copy_parallel((char *)c->host_stage[slot].p, (const char *)records + off, piece);
                    HIP_TRY(hipMemcpyAsync(dst + off, c->host_stage[slot].p, piece, hipMemcpyHostToDevice, c->st));
                    HIP_TRY(c->host_up[slot].record(c->st));
                }
            } else {
                HIP_TRY(hipMemcpyAsync(dst, records, (size_t)bytes, hipMemcpyDeviceToDevice, c->st));
                HIP_TRY(hipStreamSynchronize(c->st));  // the caller's device buffer is free again on return
            }
            sp->src = dst;
            sp->landed = true;
        }
        m->spills.push_back(std::move(sp));
        return SGX_OK;
    }
    const void *in = nullptr;
    SGX_TRY(device_input(*c, records, n * rb, mem_kind, &in));
    SGX_TRY(sp->data.ensure((size_t)std::max<int64_t>(n * rb, 16)));
    SGX_TRY(m->part_off.ensure((size_t)(s->R + 3) * 4));
    uint32_t *po = (uint32_t *)m->part_off.p;
    SGX_TRY(partition_pass(e, *c, in, sp->data.p, n, rb, s->pp, s->R, s->kind, po, nullptr, true));
    HIP_TRY(hipStreamSynchronize(c->st));
    if (po[s->R + 1] != 0 || (int64_t)po[s->R] != n)
        return fail_msg(SGX_ERR_HIP, "internal error: batch partition pass failed (flag %u)", po[s->R + 1]);
    sp->lengths.resize((size_t)s->R);
    for (int32_t p = 0; p < s->R; ++p) sp->lengths[(size_t)p] = (int64_t)po[p + 1] - po[p];  // records
    m->spills.push_back(std::move(sp));
    return SGX_OK;
}

extern "C" int sgx_map_commit(sgx_engine *e, int32_t shuffle_id, int64_t map_id, int64_t *out_lengths) {
    sgx::TraceRange trace_("sgx_map_commit");
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    std::shared_ptr<Shuffle> s;
    std::shared_ptr<MapOut> m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    std::lock_guard<std::mutex> lk(m->mu);
    if (!m->open) return fail_msg(SGX_ERR_STATE, "map %lld of shuffle %d is not open", (long long)map_id, shuffle_id);
    const int32_t R = s->R;
    const int rb = s->rb;
    int64_t total = 0;
    for (auto &sp : m->spills) total += sp->nrec;
    if (total >= (int64_t)UINT32_MAX)
        return fail_msg(SGX_ERR_INVALID, "map %lld holds %lld records (>= 2^32)", (long long)map_id, (long long)total);
    if (m->deferred) {
        SGX_TRY(m->part_off.ensure((size_t)(R + 3) * 4));
        SGX_TRY(commit_deferred(e, *c, *s, *m, total));
        if (out_lengths) {  // (finish_lengths frees the batches once the pass is done)
            SGX_TRY(finish_lengths(e, *c, *s, *m));
            std::memcpy(out_lengths, m->lengths.data(), sizeof(int64_t) * (size_t)R);
        }
        return SGX_OK;
    }
    // merged partition offsets (records): partition-major, batches in append order
    SGX_TRY(m->part_off.ensure((size_t)(R + 3) * 4));
    uint32_t *po = (uint32_t *)m->part_off.p;
    std::vector<int64_t> items;
    int64_t off = 0;
    std::vector<int64_t> bo(m->spills.size(), 0);  // running offset inside each batch
    for (int32_t p = 0; p < R; ++p) {
        po[p] = (uint32_t)off;
        for (size_t b = 0; b < m->spills.size(); ++b) {
            const int64_t cnt = m->spills[b]->lengths[(size_t)p];
            const int64_t bytes = cnt * rb;
            for (int64_t d = 0; d < bytes; d += 65536) {
                items.push_back((int64_t)(uintptr_t)((char *)m->spills[b]->data.p + bo[b] * rb + d));
                items.push_back(off * rb + d);  // destination offset, rebased below
                items.push_back(std::min<int64_t>(65536, bytes - d));
            }
            bo[b] += cnt;
            off += cnt;
        }
    }
    po[R] = (uint32_t)off;
    po[R + 1] = 0;
    // UnsafeShuffleWriter's fast merge frames every (partition, spill) segment on its own:
    // record offsets of the segments, partition-major, spill-minor (the merged layout)
    const int32_t S = (int32_t)m->spills.size();
    m->seg_spills = (s->writer == SGX_WRITER_UNSAFE && s->ser == SGX_SER_KRYO && s->lz4_block > 0 && S > 1) ? S : 1;
    if (m->seg_spills > 1) {
        const size_t nseg = (size_t)R * S;
        SGX_TRY(c->seg_host.ensure((nseg + 1) * 4));
        uint32_t *so = (uint32_t *)c->seg_host.p;
        uint32_t o = 0;
        for (int32_t p = 0; p < R; ++p)
            for (int32_t b = 0; b < S; ++b) {
                so[(size_t)p * S + b] = o;
                o += (uint32_t)m->spills[(size_t)b]->lengths[(size_t)p];
            }
        so[nseg] = o;
        SGX_TRY(m->seg_off.ensure((nseg + 1) * 4));
        HIP_TRY(hipMemcpyAsync(m->seg_off.p, so, (nseg + 1) * 4, hipMemcpyHostToDevice, c->st));
    }
    // the merged records, then the usual pipeline on an already partitioned map
    SGX_TRY(m->data.ensure((size_t)std::max<int64_t>(total * rb, 16)));
    m->nrec = total;
    const int64_t nitems = (int64_t)items.size() / 3;
    for (int64_t i = 0; i < nitems; ++i) items[3 * i + 1] += (int64_t)(uintptr_t)m->data.p;
    if (nitems > 0) {
        SGX_TRY(c->gather_items.ensure((size_t)nitems * 24));
        SGX_TRY(c->items_dev.ensure((size_t)nitems * 24));
        std::memcpy(c->gather_items.p, items.data(), (size_t)nitems * 24);
        HIP_TRY(hipMemcpyAsync(c->items_dev.p, c->gather_items.p, (size_t)nitems * 24, hipMemcpyHostToDevice, c->st));
        HIP_TRY(launch_gather_items((const int64_t *)c->items_dev.p, nitems, rb % 16 == 0 ? 16 : 4, c->st));
    }
    // device copy of the merged offsets (the Kryo framing reads them)
    SGX_TRY(c->work.ensure((size_t)(R + 2) * 4));
    HIP_TRY(hipMemcpyAsync(c->work.p, po, (size_t)(R + 2) * 4, hipMemcpyHostToDevice, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));  // the pinned offsets are rewritten by the pipeline
    m->open = false;
    SGX_TRY(run_map_pipeline(e, *c, *s, *m, m->data.p, total, true, (const uint32_t *)c->work.p));
    m->spills.clear();
    if (out_lengths) {
        SGX_TRY(finish_lengths(e, *c, *s, *m));
        std::memcpy(out_lengths, m->lengths.data(), sizeof(int64_t) * (size_t)R);
    }
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// lengths / data
// ------------------------------------------------------------------------------------
extern "C" int sgx_map_lengths(sgx_engine *e, int32_t shuffle_id, int64_t map_id, int64_t *out) {
    if (!e || !out) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    std::shared_ptr<Shuffle> s;
    std::shared_ptr<MapOut> m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    std::lock_guard<std::mutex> lk(m->mu);
    SGX_TRY(finish_lengths(e, *c, *s, *m));
    std::memcpy(out, m->lengths.data(), sizeof(int64_t) * (size_t)s->R);
    return SGX_OK;
}

extern "C" int sgx_map_data(sgx_engine *e, int32_t shuffle_id, int64_t map_id, void **ptr, int64_t *bytes) {
    if (!e || !ptr || !bytes) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    std::shared_ptr<Shuffle> s;
    std::shared_ptr<MapOut> m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    std::lock_guard<std::mutex> lk(m->mu);
    SGX_TRY(finish_lengths(e, *c, *s, *m));
    SGX_TRY(materialize(e, *c, *s, *m));
    *ptr = const_cast<void *>(m->view());
    *bytes = m->out_bytes;
    return SGX_OK;
}

extern "C" int sgx_map_layout(sgx_engine *e, int32_t shuffle_id, int64_t map_id, int32_t *out_layout) {
    if (!e || !out_layout) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    std::shared_ptr<Shuffle> s;
    std::shared_ptr<MapOut> m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    std::lock_guard<std::mutex> lk(m->mu);
    SGX_TRY(finish_lengths(e, *c, *s, *m));
    *out_layout = m->padded       ? SGX_LAYOUT_PADDED
                  : m->rec_padded ? SGX_LAYOUT_SERIALIZED_PADDED
                                  : SGX_LAYOUT_CONTIGUOUS;
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// IndexShuffleBlockResolver.writeIndexFileAndCommit (IndexShuffleBlockResolver.scala:161-217)
// ------------------------------------------------------------------------------------
extern "C" int sgx_write_index(sgx_engine *e, int32_t shuffle_id, int64_t map_id, const char *index_path,
                               const char *data_path, int64_t *out_lengths) {
    sgx::TraceRange trace_("sgx_write_index");
    if (!e || !index_path || !data_path) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    std::shared_ptr<Shuffle> s;
    std::shared_ptr<MapOut> m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    std::lock_guard<std::mutex> lk(m->mu);
    SGX_TRY(finish_lengths(e, *c, *s, *m));
    SGX_TRY(materialize(e, *c, *s, *m));
    std::vector<uint8_t> host((size_t)m->out_bytes);
    if (m->out_bytes) HIP_TRY(hipMemcpy(host.data(), m->view(), (size_t)m->out_bytes, hipMemcpyDeviceToHost));
    return commit_index_files(index_path, data_path, s->R, m->lengths.data(), host.data(), m->out_bytes, out_lengths);
}
