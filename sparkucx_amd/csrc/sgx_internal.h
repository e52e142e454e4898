// sgx_internal.h — shared between the HIP kernels (sgx_kernels.hip) and the engine
// (sgx_engine.cpp).  Not part of the public ABI (that is include/sgx.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sgx_host.h"

namespace sgx {

// Partitioner description as seen by the kernels (built by the engine from the shuffle's
// registration; see sgx_engine.cpp make_part_params).
struct PartParams {
    int32_t kind;        // SGX_PART_*
    uint32_t R;          // number of partitions
    uint32_t mg_m;       // Granlund-Montgomery magic for u32 mod R (R >= 2): see mod_params()
    uint32_t mg_s;       //   and its shift, ceil(log2 R) - 1
    uint32_t c31;        // 2^31 mod R (HashPartitioner's signed-int correction)
    uint32_t nbits;      // bits needed to hold a partition id (ceil log2 R), >= 1
    int32_t nb;          // range bounds count (R - 1)
    int32_t ascending;   // RangePartitioner.ascending
    uint32_t mbits;      // K4 peer-table width for this launch (0 = ballots only)
    const void *bounds;  // device: int64[nb] (RANGE_I64) or Key10[nb] (RANGE_BYTES10)
    uint32_t dshift;     // KIND_DIGIT: bit offset of the digit in the record's first 12 bytes (LE)
    uint32_t dflip;      // KIND_DIGIT: XORed into the digit (0x80 = sign flip of an i64 key's top byte)
    // range kinds: directory of the bounds by the key's top RDIR_BITS bits (device u16
    // [2^RDIR_BITS + 1]: dir[j] = first bound whose top bits are >= j), or null when the bounds
    // need the JDK binary search's exact path (duplicates with more than 128 bounds)
    const uint16_t *dir;
    // ---- single-pass padded map output (sgx_map.cpp padded_pass) ----
    // guard: non-null -> the kernel (k_hist, k_scatter16_wc) runs only when *guard holds
    // PAD_OVERFLOW, i.e. it is the two-pass fallback of a padded write whose bins overflowed
    const uint32_t *guard;
    // K4 output capacity in records (0 = n): the padded output is larger than the input
    uint32_t olim;
    // K4 padded: final record count of every (partition, chunk) stream out [R][G], checked
    // against pad_cap[p] (the sub-bin capacity of partition p); an overflow sets PAD_OVERFLOW
    uint32_t *pad_cnt;
    const uint32_t *pad_cap;
    // K4 padded, sub-bins laid out by K4 itself (pad_est non-null, 16 B write-combining K4):
    // every workgroup turns the sampled counts est[R] into capacities cap[p] (mu = est * scale,
    // cap = mu + PAD_SIGMAS * sqrt(a * mu + 16) + 8, a whole line) and bases pbase[p] =
    // sum_{q<p} G cap[q]; stream (p, g) starts at min(pbase[p] + g cap[p], olim); workgroup 0
    // publishes {cap[R], pbase[R]} in pad_layout; the epilogue writes every stream's END
    // position to pad_cnt (k_pad_finish turns them into counts and checks the capacities)
    const uint32_t *pad_est;
    uint32_t *pad_layout;
    double pad_scale, pad_a;
    // ---- streaming map (sgx_map_append batches written in one pass at sgx_map_commit) ----
    // chunk table: chunk g's records start at byte chunks[2g] from the kernel's input pointer
    // and number chunks[2g+1] (every chunk inside one batch); null: chunk g = records
    // [g * chunk, min(n, (g + 1) * chunk)) of one contiguous input
    const int64_t *chunks;
    // ---- the padded split's level 2 (k_scatter16_wc SEG + WC_PADDED): workgroup b = k G + g
    // reads the level-1 fragments of supers k pack .. k pack + pack - 1 in chunk g -- fragment
    // (s, g) = frag_cnt[s G + g] records from frag_start[s G + g] -- as one sequence; its R =
    // 64 pack streams are the partitions k R .. k R + R - 1 (pack <= SPLIT_PACK_MAX)
    const uint32_t *frag_start, *frag_cnt;
    uint32_t pack;
};
constexpr uint32_t SPLIT_PACK_MAX = 16;
// Error-word bits shared by the map-side kernels and the engine.
constexpr uint32_t ERR_SPIN = 1u;          // a look-back spin gave up
constexpr uint32_t ERR_SCATTER_OOB = 2u;   // a scatter destination was out of range
constexpr uint32_t PAD_OVERFLOW = 0x100u;  // a padded sub-bin overflowed: the two-pass fallback ran
// Padded map output: one line in PAD_SAMPLE_STRIDE_MAX (128 B = 8 records) at most is read by
// the sampled histogram; sub-bin capacity = mu + PAD_SIGMAS * sqrt(a * mu + 16) + 8, rounded up
// to a whole line (a = 1 + chunk / sampled records: the chunk's own Poisson spread plus the
// sample's estimation error).
#ifndef SGX_PAD_SAMPLE_STRIDE_MAX  // (A/B builds: -DSGX_PAD_SAMPLE_STRIDE_MAX=512)
#define SGX_PAD_SAMPLE_STRIDE_MAX 128
#endif
constexpr int PAD_SAMPLE_STRIDE_MAX = SGX_PAD_SAMPLE_STRIDE_MAX;
constexpr double PAD_SIGMAS = 6.5;
constexpr int RDIR_BITS = 10;
constexpr int RDIR_N = (1 << RDIR_BITS) + 1;
constexpr size_t RDIR_BYTES = ((size_t)RDIR_N * 2 + 15) & ~(size_t)15;
// Internal partition kind of the reduce side's LSD radix passes: pid = 8-bit digit of the
// key (R = 256), see PartParams::dshift / dflip.  Never registered through the C ABI.
constexpr int KIND_DIGIT = 200;
// Kernel-internal kind: HashPartitioner with a power-of-two R (pid = (k_lo ^ k_hi) & (R - 1)).
constexpr int KIND_HASH_POW2 = 100;
constexpr uint32_t DIGIT_R = 256;
// Internal partition kind of the two-level split scatter (hash, power-of-two R > 1024):
// pid = ((k_lo ^ k_hi) >> dshift) & (R - 1), i.e. the top log2(R) bits of the full
// power-of-two HashPartitioner id (its "super-partition"), with R super-partitions.
constexpr int KIND_HASH_BITS = 300;
// Internal kind of the sorted read's bucket passes: pid = (W >> dshift) & (R - 1) over the
// key's 64-bit order window W -- a 16 B record's signed Long key with its sign flipped
// (dflip = 1), or a 100 B record's first 8 key bytes big-endian (dflip = 0).
constexpr int KIND_KEY_BITS = 400;
// Internal kind of the hybrid split's level 1 (hash, power-of-two R > 1024): pid = stream of
// the record's partition (k_lo ^ k_hi) & (2^dshift - 1), looked up in the per-map table
// PartParams::dir (u16 [2^dshift], staged in LDS): the hot partitions' own streams
// [0, SPLIT_HOT_CAP), then one stream per cold super-partition of 64 partitions.
constexpr int KIND_HOT_SPLIT = 500;
#ifndef SGX_SPLIT_HOT_CAP
#define SGX_SPLIT_HOT_CAP 704
#endif
constexpr int SPLIT_HOT_CAP = SGX_SPLIT_HOT_CAP;  // + S <= 64 cold supers: <= 768 level-1 streams (LDS)

// Granlund-Montgomery parameters of mod_u32 (sgx_kernels.hip) for 2 <= R < 2^31:
// l = ceil(log2 R), m = floor(2^32 (2^l - R) / R) + 1, shift = l - 1.
inline void mod_params(uint32_t R, uint32_t *m, uint32_t *shift) {
    if (R < 2) { *m = 0; *shift = 0; return; }
    uint32_t l = 0;
    while ((1ull << l) < R) ++l;
    *m = (uint32_t)(((1ull << 32) * ((1ull << l) - R)) / R + 1);
    *shift = l - 1;
}

// 10-byte unsigned-lexicographic key, pre-split so tuple compare == byte compare.
struct Key10 {
    uint64_t hi;  // bytes 0..7 big-endian
    uint32_t lo;  // bytes 8..9 big-endian (<< 0)
    uint32_t pad;
};

// Tile geometry of the LDS-staged scatter (records per tile) for a partition count.
struct ScatterGeom {
    int waves;
    int items;  // records per lane per tile
    int tile;   // waves * items * 64
    size_t lds_bytes;
    int mbits;  // LDS peer-table width (0 = ballots only)
};
ScatterGeom scatter_geom16(uint32_t R, int force_waves = 0, int force_items = 0);
// Lane-ordered-ranking staged kernel (waves == ORD_GEOM_BASE + real waves, mbits == PP).
constexpr int ORD_GEOM_BASE = 2000;
ScatterGeom scatter_geom16_ord(uint32_t R, int force_waves = 0, int force_items = 0);
// Write-combining staged kernel (waves == WC_GEOM_BASE + real waves, items == new records
// per lane, mbits == stage slots per lane).
constexpr int WC_GEOM_BASE = 3000;
ScatterGeom scatter_geom16_wc(uint32_t R);
__host__ __device__ size_t scatter16_lds(uint32_t R, int waves, int items, int mbits);
ScatterGeom scatter_geom_wide(uint32_t R, int record_bytes);
// Wide-record staged kernel (100 B TeraSort records; waves == WIDE2_GEOM_TAG), items == 0
// when it does not apply (R > 2048, other widths, LDS).
constexpr int WIDE2_GEOM_TAG = -2;
ScatterGeom scatter_geom_wide2(uint32_t R, int record_bytes, int kind, int nb);

// Launchers (all asynchronous on `stream`).  counts / offs are [R][G] partition-major.
// counts: [R][G] u32, zeroed here unless `zeroed` (the caller's memset covered them).
// mode: HIST_ATOMIC (one LDS atomic per record) or HIST_BALLOT (wave-aggregated: one
// atomic per distinct partition id of a wave, peers found by ballots; 16 B hash only).
constexpr int HIST_ATOMIC = 0, HIST_BALLOT = 1;
hipError_t launch_hist(const void *in, int64_t n, int record_bytes, int64_t chunk, int G,
                       const PartParams &pp, uint32_t *counts, hipStream_t stream, int mode = 0,
                       bool zeroed = false);
// ticket: zeroed dispatch-order counter; err: sticky error word (bit 0: look-back gave up);
// guard: as PartParams::guard
hipError_t launch_scan(const uint32_t *counts, uint32_t *offs, int64_t len, uint64_t *status,
                       uint32_t *ticket, uint32_t *err, uint32_t *part_off, int G, int R,
                       hipStream_t stream, const uint32_t *guard = nullptr);
int64_t scan_tiles(int64_t len);
// The same scan (same tiles, statuses and results) with one wave per tile and no LDS: a
// padded write's tail runs it while the next map's K4 holds every CU's LDS, so its workgroups
// share CUs with that K4 instead of holding back some of its workgroups.
hipError_t launch_scan_wave(const uint32_t *counts, uint32_t *offs, int64_t len, uint64_t *status, uint32_t *ticket,
                            uint32_t *err, uint32_t *part_off, int G, int R, hipStream_t stream,
                            const uint32_t *guard = nullptr);
// the padded split's overflow fallback histogram: [R][G] counts of a contiguous 16 B input
// (hash partitioner), no LDS; a no-op unless *guard has PAD_OVERFLOW
hipError_t launch_hist16_fallback(const void *in, int64_t n, int64_t chunk, int G, const PartParams &pp,
                                  uint32_t *counts, const uint32_t *guard, hipStream_t stream);
// Padded map output.  launch_pad_sample: est[p] += records of partition p among
// every `stride`-th group of 8 records (est zeroed by the caller; hash partitioner over 16 B
// records, or RangePartitioner over 100 B TeraSort records; R <= 4096).  With a chunk table
// (pp.chunks, a streaming map) each of the G chunks (<= `chunk` records) is sampled on its own.
hipError_t launch_pad_sample(const void *in, int64_t n, int rb, int stride, const PartParams &pp, uint32_t *est,
                             hipStream_t stream, int64_t chunk = 0, int G = 0);
// The tail of a padded write whose K4 laid its sub-bins out itself (PartParams.pad_est):
// fstart[i] = min(pbase[p] + g cap[p], olim) from the published layout ([R] caps, [R] bases),
// cnt[i] = the end position K4 left there - fstart[i]; a count above its capacity sets
// PAD_OVERFLOW in *flags.  Also zeroes `zero` (nzero u32: the scan's ticket / status, its
// error word) for the kernels that follow on the stream.
hipError_t launch_pad_finish(const uint32_t *layout, int R, int G, uint32_t olim, uint32_t *fstart, uint32_t *cnt,
                             uint32_t *flags, uint32_t *zero, int64_t nzero, hipStream_t stream);
// *flags_out = *flags; then est[R], *flags = 0 (the slot's next sample and K4 start from zero).
hipError_t launch_pad_reset(uint32_t *flags, uint32_t *flags_out, uint32_t *est, int R, hipStream_t stream);
// The padded 16 B write's overflow fallback (a no-op unless *guard has PAD_OVERFLOW): the
// map's records into the contiguous layout, stream (p, g) from foff[p*G+g] on, stably, one
// wave per chunk and no LDS -- so its no-op launch takes no CU away from the next map's K4.
// cur: R*G u32 of scratch (the streams' cursors).
hipError_t launch_scatter16_fallback(const void *in, void *out, int64_t n, int64_t chunk, int G, const PartParams &pp,
                                     const uint32_t *foff, uint32_t *cur, const uint32_t *guard, uint32_t *err,
                                     hipStream_t stream, int rb = 16);  // rb 16 (hash) or 100 (TeraSort range)
// Whether a padded TeraSort map's K4 is the write-combining kernel (the one that lays its
// sub-bins out itself): R <= 1024, its LDS fits, chunks a multiple of its tile.
bool wide_wc_padded_ok(uint32_t R, int nb, int64_t chunk);
// (partition, spill) segment offsets of a streaming map committed in one pass (k_spill_seg_offs).
hipError_t launch_spill_seg_offs(const uint32_t *offs, const uint32_t *part_off, int R, int G, int S,
                                 const int32_t *g0, uint32_t *out, hipStream_t stream);
// The number of records launch_pad_sample reads (the estimate's denominator).
int64_t pad_sampled_records(int64_t n, int stride);
// Sub-bin capacities pcap[p] (records, a multiple of 8) from the sampled counts, and the
// stream starts fstart[p][g] = pbase[p] + g * pcap[p] (pbase: exclusive scan of G * pcap);
// a total above olim sets PAD_OVERFLOW in *err_pad.  R <= 4096.
hipError_t launch_pad_caps(const uint32_t *est, int R, int64_t sampled, int64_t chunk, int G, uint32_t olim,
                           uint32_t *pcap, uint32_t *fstart, uint32_t *err_pad, hipStream_t stream);
// Host bound of the padded output's records for any sample (>= every total launch_pad_caps
// can produce), or -1 when it does not fit 32-bit record offsets.
int64_t pad_capacity_bound(int64_t n, int R, int64_t chunk, int G, int64_t sampled);
// Gather of padded fragments: for each block b, fragments g in [0, G_b) of partition p_b of a
// padded map of rb-byte records -- src + rb * fstart[p*G+g], rb * cnt[p*G+g] bytes -- to
// dst + rb * (foff[p*G+g] - foff[p*G]).  desc[b] = {src, fstart, foff, cnt, dst, p, G_b, rb};
// G = the largest G_b.
constexpr int FRAG_DESC_WORDS = 8;
// the peer gather's system-scope L2 write-back (release) / invalidate (acquire) on every XCD
hipError_t launch_l2_fence(bool release, hipStream_t stream);
hipError_t launch_gather_frags(const int64_t *desc, int64_t nblocks, int G, hipStream_t stream,
                               int max_rows = 65535);  // max_rows: workgroups per fragment column
// Two-level split scatter (hash partitioner, power-of-two R > 1024, 16 B records):
// desc: the level-2 pieces cut from the level-1 offsets (offs1[S][G], u32) -- each piece a
// run of whole (super, chunk) blocks inside one super-partition, about `target` records --
// as {begin, -, super, first chunk} int64 quadruples (a piece ends at the next one's begin;
// cut every *total / pieces records, *total = the level-1 record count on the device),
// their count in npieces[1] (flags / idx: S*G u32 scratch; status / ticket: a zeroed scan
// work area of scan_tiles(S*G) tiles);
// launch_scatter16_seg: level 2, write-combining K4 with R = Q over the pieces, cursors
// offs[(super*Q + q)][chunk] of the single-level scan.
hipError_t launch_seg_desc(const uint32_t *offs1, int S, int G, const uint32_t *total, int64_t pieces, int64_t *desc,
                           uint32_t *flags, uint32_t *idx, uint64_t *status, uint32_t *ticket, uint32_t *err,
                           uint32_t *npieces, hipStream_t stream);
// seg_end: device count of the level-1 records the pieces cover (the last piece's end)
// With pp.pad_cnt (the padded split): one workgroup walks fragments blockIdx.x, + grid, ... of
// desc ({begin, end, super, chunk} each, *ndesc of them), every fragment's 64 streams starting
// at offs[(super*Q + q)][chunk] (their sub-bins) and their final counts going to pad_cnt.
hipError_t launch_scatter16_seg(const void *in, void *out, int64_t n, const PartParams &pp, const uint32_t *offs,
                                int G, const int64_t *desc, const uint32_t *ndesc, const uint32_t *seg_end, int grid,
                                const ScatterGeom &geo, uint32_t *err, hipStream_t stream);
// Hybrid split: from the partition offsets, stream_of[p] = hot index for
// about the SPLIT_HOT_CAP largest partitions (a coarse count histogram picks the cut; the hot
// ones numbered in id order), else SPLIT_HOT_CAP + p / Q; hot_part[h] = the partition of hot
// stream h (-1: unused).
// csum[s][g] = the cold partitions' counts summed per super-partition s and chunk g;
// cur1[(SPLIT_HOT_CAP + S) x G] = level-1 cursors: a hot stream's final offsets
// offs[p][g], a cold super's scratch offsets offs1[s][g].
// counts (optional): per-partition counts to select from instead of the offsets' differences
hipError_t launch_hot_select(const uint32_t *part_off, int R, int Q, uint16_t *stream_of, int32_t *hot_part,
                             hipStream_t stream, const uint32_t *counts = nullptr);
hipError_t launch_super_counts_cold(const uint32_t *counts, const uint16_t *stream_of, uint32_t *csum, int S, int Q,
                                    int G, hipStream_t stream);
// pcap / cap1 / capS: the padded split's sub-bin capacities (capS[stream] written when given)
hipError_t launch_hot_cursors(const uint32_t *offs, const int32_t *hot_part, const uint32_t *offs1, uint32_t *cur1,
                              int S, int G, hipStream_t stream, const uint32_t *pcap = nullptr,
                              const uint32_t *cap1 = nullptr, uint32_t *capS = nullptr);
// The padded split: est1[s] = cold partitions' sampled counts per super; level 2's
// fragment list desc[s*G+g] = {begin, end, s, g} of the level-1 scratch sub-bins (cnt1: the
// level-1 streams' counts, [HOT + S][G]); the hot partitions' final counts from level 1.
hipError_t launch_cold_super_est(const uint32_t *est, const uint16_t *stream_of, int S, int Q, uint32_t *est1,
                                 hipStream_t stream);
hipError_t launch_hot_counts(const uint32_t *cnt1, const int32_t *hot_part, int G, uint32_t *cnt, hipStream_t stream);
// The sorted read's last step: `in` is ordered by bucket = (P(key) << kbits) | key window
// bits [kshift, kshift + kbits) (P the shuffle's hash partitioner when use_p, else 0); every
// bucket is sorted stably by the full key on chip (16 B: signed Long; 100 B: 10-byte
// unsigned big-endian) into `out`.  A bucket longer than the kernel's cap sets bit 4 of *err
// and leaves `out` incomplete (the caller falls back to the LSD digit passes).
hipError_t launch_bucket_sort(const void *in, void *out, int64_t n, int rb, const PartParams &pp, int use_p,
                              uint32_t kshift, uint32_t kbits, uint32_t *err, hipStream_t stream);
// Engine-start self-check of the lane-ordered LDS atomics the ordered ranking relies on:
// *bad |= 1 on any violation (sgx_create).
hipError_t launch_lds_order_probe(uint32_t *bad, hipStream_t stream);
// out2 / hot_cap: KIND_HOT_SPLIT only -- streams >= hot_cap go to out2 (the split's scratch)
hipError_t launch_scatter(const void *in, void *out, int64_t n, int record_bytes, int64_t chunk,
                          int G, const PartParams &pp, const uint32_t *offs, const ScatterGeom &geo,
                          uint32_t *err, hipStream_t stream, void *out2 = nullptr, uint32_t hot_cap = 0);
// items: [n][3] int64 {src_off, dst_off, bytes}; all offsets/bytes multiples of `align`.
// LZ4BlockOutputStream framing (sgx_lz4.hip)
int lz4_lanes_per_workgroup();
int lz4_max_block();
// err: 4 int64 {flags, block, offset, length}, zeroed by the caller (see k_lz4_blocks).
// sizes[b] = 21 + payload bytes (RAW: the block's length); checks[b] = masked XXH32.
hipError_t launch_lz4_blocks(const uint8_t *stream, int64_t stream_len, const int64_t *blocks, int64_t nblocks,
                             int level, uint8_t *slots, int64_t slot_bytes, int32_t *sizes, uint32_t *checks,
                             int64_t *err, hipStream_t s);
hipError_t launch_lz4_gather(const uint8_t *stream, const int64_t *blocks, const uint8_t *slots, int64_t slot_bytes,
                             const int32_t *sizes, const uint32_t *checks, const int64_t *frame_off, int64_t nblocks,
                             const int64_t *end_off, int64_t nends, int level, uint8_t *dst, hipStream_t s);
hipError_t launch_lz4_walk(const uint8_t *in, int64_t nbytes, int64_t *desc, int64_t desc_cap, int64_t *info,
                           hipStream_t s);
// per-stream walk (see k_lz4_walk_streams): soff[nstreams + 1]; cnt [nstreams][2]; err: one
// u64, initialised to ~0 by the caller (min of position << 8 | code)
hipError_t launch_lz4_walk_streams(const uint8_t *in, const int64_t *soff, int64_t nstreams, int64_t *cnt,
                                   int64_t *desc, unsigned long long *err, bool write, hipStream_t s);
// force_lanes: compressed frames one lane per frame whatever their number (SGX_FLAG_LZ4_LANE_DECODE)
hipError_t launch_lz4_decode(const uint8_t *in, const int64_t *desc, int64_t nframes, uint8_t *out,
                             uint32_t *err, bool force_lanes, hipStream_t s);
hipError_t launch_copy_items(const void *src, void *dst, const int64_t *items, int64_t n_items,
                             int align, hipStream_t stream);
// items: [n][3] int64 {src address, dst address, bytes} (device memory on both sides).
hipError_t launch_gather_items(const int64_t *items, int64_t n_items, int align, hipStream_t stream);
// Reduce side (sgx_reduce.hip), key-sorted (Long, Long) records
hipError_t launch_digit_hist(const void *rec, int64_t n, int rb, uint32_t *hist, int num_cus, hipStream_t st);
// The sorted read's segmented passes (records already contiguous by partition): piece k =
// desc[4k..] = {begin, -, k, 0} up to the next piece's begin (the last: n), pieces of segment
// s = [pk[s], pk[s+1]); cnt[k * Q + q] = piece k's records in bucket q (KIND_KEY_BITS or
// KIND_DIGIT, Q = pp.R <= 1024); offs = per-segment exclusive scan, bucket-major,
// piece-minor, from seg_base[s] -- K4's SEG mode then runs with G = 1.
// The window histogram of every piece (KIND_KEY_BITS) and the 8 digit histograms of 16 B records
// in one pass (dhist zeroed here).
hipError_t launch_piece_digit_hist(const void *in, int64_t n, const int64_t *desc, int64_t npieces,
                                   const PartParams &pp, uint32_t *cnt, uint32_t *dhist, hipStream_t st);
hipError_t launch_piece_hist(const void *in, int64_t n, const int64_t *desc, int64_t npieces, const PartParams &pp,
                             uint32_t *cnt, hipStream_t st);
hipError_t launch_seg_offsets(const uint32_t *cnt, const int64_t *seg_base, const int32_t *pk, int64_t nseg, uint32_t Q,
                              uint32_t *offs, hipStream_t st);
// groupByKey / reduceByKey(_ + _) over key-sorted (Long, Long) records in one pass
// (sgx_reduce.hip, k_group_fused): keys[g], starts[g] (may be NULL), vals = every value (GROUP)
// or the group sums (SUM), *ngroups.  status: 2 * group_tiles(n) u64, ticket/err: zeroed.
int64_t group_tiles(int64_t n);
hipError_t launch_group_fused(const void *rec, int64_t n, bool sum, uint64_t *status, uint32_t *ticket, uint32_t *err,
                              int64_t *keys, int64_t *starts, int64_t *vals, int64_t *ngroups, hipStream_t st);
// keys[i], vals[i] -> 16 B records {key, value} (map-side combine output)
hipError_t launch_pack_pairs(const int64_t *keys, const int64_t *vals, int64_t n, void *out, hipStream_t st);
// RangePartitioner.sketch (sgx_sample.hip): reservoir of k keys of n records, XORShiftRandom
// state s0 (already hashSeed'ed), jump = [48][64] column-form powers M^(2^t) of one step.
int64_t reservoir_threads(int64_t n, int64_t k);
hipError_t launch_reservoir(const void *recs, int64_t n, int rb, int key_bytes, int64_t k, uint64_t s0,
                            const uint64_t *jump_dev, long long *winner, void *out_keys, hipStream_t st);
// RangePartitioner re-sampling (BernoulliSampler): flags[i] = nextDouble #i <= fraction, and a
// gather of the keys of selected record indices.
hipError_t launch_bernoulli_flags(int64_t n, double fraction, uint64_t s0, const uint64_t *jump_dev, uint8_t *flags,
                                  hipStream_t st);
hipError_t launch_gather_keys(const void *recs, int rb, int key_bytes, const int64_t *idx_dev, int64_t m,
                              void *out_keys, hipStream_t st);
// Kryo (Long, Long) framing (sgx_serde.hip): n partition-contiguous 16 B records -> their
// KryoSerializationStream bytes in `out` (capacity 20 n), partition byte offsets ser_off[R+1]
// from the record offsets rec_off[R+1].  A padded map's records come through its fragment
// table `frag` ([fstart | foff | cnt] x nfrag) unless *ovf has PAD_OVERFLOW (the fallback
// rewrote them contiguously).  Workspace `work` / `status`: kryo_work_bytes(tiles)
// bytes (tiles = kryo_ser16_tiles(n) / kryo_deser16_tiles(bytes)), no zeroing needed.
int64_t kryo_ser16_tiles(int64_t n);
int64_t kryo_work_bytes(int64_t tiles);  // the `status` workspace of either launcher
hipError_t launch_kryo_ser16(const void *in, int64_t n, void *out, const uint32_t *rec_off, int R, int64_t *ser_off,
                             uint64_t *work, hipStream_t st,
                             const uint32_t *frag = nullptr, int64_t nfrag = 0, const uint32_t *ovf = nullptr);
// Kryo (Long, Long) stream of `bytes` bytes (16 B-aligned, readable to bytes + 32) -> 16 B
// records (at most out_cap); *count_out = records; ticket_err[1] bit 1 = malformed stream.
int64_t kryo_deser16_tiles(int64_t bytes);
hipError_t launch_kryo_deser16(const void *in, int64_t bytes, void *out, int64_t out_cap, uint64_t *status,
                               uint32_t *ticket_err, int64_t *count_out, hipStream_t st);
hipError_t launch_gen_uniform16(void *dst, int64_t n, uint64_t seed, int64_t value_base,
                                hipStream_t stream);
hipError_t launch_gen_zipf16(void *dst, int64_t n, uint64_t seed, int64_t value_base,
                             const double *cdf, int64_t K, hipStream_t stream);
hipError_t launch_gen_terasort100(void *dst, int64_t n, uint64_t seed, int64_t index_base,
                                  hipStream_t stream);

}  // namespace sgx
