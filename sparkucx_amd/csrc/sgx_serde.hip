// Kryo framing of a (Long, Long) map output on the GPU.
//
// Spark writes a shuffle partition as the serializer's stream of its records; with
// spark.serializer = KryoSerializer and spark.shuffle.compress = false every (Long, Long)
// record is two kryo.writeClassAndObject calls (KryoSerializationStream.writeKey/writeValue,
// reached from ExternalSorter.writePartitionedMapOutput / UnsafeShuffleWriter behind
// UcxShuffleManager.getWriter, spark_3_0/UcxShuffleManager.scala:32-53):
//   [0x09]  class id of java.lang.Long (Kryo registers long as id 7; written varint(id + 2))
//   [zigzag varlong of the key]   LongSerializer: Output.writeLong(v, false) = writeVarLong,
//   [0x09]                        7 bits per byte, low first, 0x80 = more; after 8 such
//   [zigzag varlong of the value] bytes the 9th byte holds bits 56..63 whole.
// Long is a wrapper class, so reference tracking writes nothing.  A partition's bytes are
// its records' encodings back to back in map order; the index offsets
// (IndexShuffleBlockResolver.writeIndexFileAndCommit, :161-217) are byte offsets of that.
//
// Reduce-then-scan over the partition-contiguous 16 B records (K4's output): (1) every tile
// of 1024 records sums its records' encoded lengths, (2) one workgroup scans the tile sums
// into 64-bit byte prefixes, (3) every tile computes its records' offsets (block scan),
// encodes them into LDS at the output's 16 B phase and writes the tile out with 16 B stores
// (byte stores only for the two edge words it shares with its neighbours).  The tile that
// holds a partition's first record also writes that partition's byte offset.  HBM-bound:
// 16 B read twice + the encoded bytes written per record.
#include "sgx_internal.h"

namespace sgx {
namespace {

constexpr int KS_THREADS = 256, KS_ITEMS = 4, KS_TILE = KS_THREADS * KS_ITEMS;
constexpr int KS_MAXREC = 20;  // 2 class bytes + 2 x 9 varlong bytes

__device__ __forceinline__ uint64_t zigzag(uint64_t v) { return (v << 1) ^ (uint64_t)((int64_t)v >> 63); }

__device__ __forceinline__ uint32_t ks_wave_scan(uint32_t x, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    return x;
}

__device__ __forceinline__ uint32_t varlong_len(uint64_t z) {
    const uint32_t bits = 64u - (uint32_t)__clzll((long long)(z | 1ull));
    const uint32_t n = (bits + 6u) / 7u;
    return n > 9u ? 9u : n;
}

// The varlong bytes of z (length L = varlong_len(z)) as a 72-bit little-endian value:
// lo = the first 8 bytes (7-bit groups, 0x80 on every byte but the last), hi = the 9th.
__device__ __forceinline__ void varlong_bytes(uint64_t z, uint32_t L, uint64_t &lo, uint32_t &hi) {
    uint64_t e = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) e |= ((z >> (7 * i)) & 0x7Full) << (8 * i);
    const uint64_t cont = L >= 9 ? ~0ull : ((1ull << (8 * (L - 1))) - 1ull);  // bytes 0..L-2
    lo = e | (cont & 0x8080808080808080ull);
    hi = L >= 9 ? (uint32_t)(z >> 56) : 0u;
}

// w[0..2] |= (lo | hi << 64) << s, for 0 <= s <= 120 (bits), without dynamic indexing
__device__ __forceinline__ void or_shifted(uint64_t w[3], uint64_t lo, uint64_t hi, uint32_t s) {
    const uint32_t q = s >> 6, r = s & 63u;
    const uint64_t c0 = lo << r;
    const uint64_t c1 = (r ? lo >> (64 - r) : 0ull) | (hi << r);
    const uint64_t c2 = r ? hi >> (64 - r) : 0ull;
    w[0] |= q == 0 ? c0 : 0ull;
    w[1] |= q == 0 ? c1 : (q == 1 ? c0 : 0ull);
    w[2] |= q == 0 ? c2 : (q == 1 ? c1 : c0);
}


// Exclusive scan of per-tile u32 aggregates into u64 prefixes (one workgroup; a few
// hundred thousand tiles take tens of µs).  The serializer and decoder are reduce-then-scan:
// a single pass with decoupled look-back measured ~20 µs per tile of waiting on gfx950 (the
// status words are agent-coherent, i.e. they cross the XCDs' L2s), bounding both kernels by
// latency, not by HBM.
constexpr int TS_THREADS = 1024, TS_PER = 4, TS_BLOCK = TS_THREADS * TS_PER;
// Workspace after the tile sums: excl[tiles] (exclusive prefix within a block of TS_BLOCK
// tiles) | btot[ceil(tiles / TS_BLOCK)] (block totals).  k_ser_tile_info adds the totals of
// the blocks before each tile's (at most a few hundred values).
__global__ __launch_bounds__(TS_THREADS) void k_tile_scan64(const uint32_t *__restrict__ agg, int64_t ntiles,
                                                            uint64_t *__restrict__ excl, uint64_t *__restrict__ btot) {
    __shared__ uint64_t s_w[TS_THREADS / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t b = (int64_t)blockIdx.x * TS_BLOCK + (int64_t)tid * TS_PER;
    uint32_t v[TS_PER];
    uint64_t sum = 0;
#pragma unroll
    for (int i = 0; i < TS_PER; ++i) {
        v[i] = b + i < ntiles ? agg[b + i] : 0u;
        sum += v[i];
    }
    uint64_t x = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint64_t run = x - sum, tot = 0;
#pragma unroll
    for (uint32_t q = 0; q < TS_THREADS / 64; ++q) {
        if (q < w) run += s_w[q];
        tot += s_w[q];
    }
#pragma unroll
    for (int i = 0; i < TS_PER; ++i) {
        if (b + i < ntiles) excl[b + i] = run;
        run += v[i];
    }
    if (tid == 0) btot[blockIdx.x] = tot;
}

// The map's partitioned records: contiguous, or (a padded map) the fragments
// (p, g) = [fstart, + cnt) of the padded buffer in (p, g) order, foff their contiguous
// positions -- unless the padded write overflowed (*ovf & PAD_OVERFLOW: its fallback rewrote
// the map contiguously).  k_tile_frags first stores every tile's first fragment (one pass over
// the fragment table); a tile then stages the fragments covering its records in LDS (a tile of
// 1024 records meets a few dozen) and every record finds its own by a binary search there --
// no dependent global loads per record or per tile.  A tile that meets more (a run of empty
// fragments) searches the global table over the same range.
constexpr int KS_FRAGS = 256;
struct RecSrc {
    const uint4 *in;
    const uint32_t *fstart = nullptr, *foff = nullptr, *cnt = nullptr;  // padded map: R * G fragments
    int64_t nf = 0;
    const uint32_t *ovf = nullptr;
    const uint32_t *tile_f0 = nullptr;  // [tiles + 1]: the fragment holding each tile's first record
};
// a tile's fragments [f0, f0 + nfr) (registers: tile-uniform scalar loads) and their
// foff / fstart staged in LDS (2 x KS_FRAGS words the caller provides)
struct TileFrags {
    int64_t f0 = -1;  // -1: contiguous records
    int nfr = 0;
    uint32_t *s_foff = nullptr, *s_fstart = nullptr;
};
// tile_f0[t] = the nonempty fragment holding record t * KS_TILE (exactly one writer per
// tile), tile_f0[tiles] = nf - 1.  A no-op when the padded write overflowed.
__global__ __launch_bounds__(256) void k_tile_frags(RecSrc rs, int64_t tiles, uint32_t *__restrict__ tile_f0) {
    if (*rs.ovf & PAD_OVERFLOW) return;
    const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (f == 0) tile_f0[tiles] = (uint32_t)(rs.nf - 1);
    if (f >= rs.nf) return;
    const int64_t c = rs.cnt[f];
    if (c == 0) return;
    const int64_t a = rs.foff[f];
    for (int64_t t = (a + KS_TILE - 1) / KS_TILE; t <= (a + c - 1) / KS_TILE && t < tiles; ++t)
        tile_f0[t] = (uint32_t)f;
}

// the tile's fragment range (every thread; no LDS yet)
__device__ __forceinline__ TileFrags tile_frags(const RecSrc &rs, int64_t tile, uint32_t *lds) {
    TileFrags tf;
    if (!rs.foff || (*rs.ovf & PAD_OVERFLOW)) return tf;
    const uint32_t f0 = rs.tile_f0[tile], f1 = rs.tile_f0[tile + 1];
    tf.f0 = f0;
    tf.nfr = (int)(f1 - f0) + 1;
    tf.s_foff = lds;
    tf.s_fstart = lds + KS_FRAGS;
    return tf;
}
// whole block: stage the range in LDS; the caller's barrier publishes it
__device__ __forceinline__ void stage_frags(const RecSrc &rs, const TileFrags &tf, uint32_t tid) {
    if (tf.f0 < 0 || tf.nfr > KS_FRAGS) return;
    for (int j = (int)tid; j < tf.nfr; j += KS_THREADS) {
        tf.s_foff[j] = rs.foff[tf.f0 + j];
        tf.s_fstart[j] = rs.fstart[tf.f0 + j];
    }
}
__device__ __forceinline__ uint4 load_rec(const RecSrc &rs, const TileFrags &tf, int64_t i) {
    if (tf.f0 < 0) return rs.in[i];
    const uint32_t x = (uint32_t)i;
    int lo = 0, hi = tf.nfr;  // last j with foff[j] <= x (foff[0] <= t0 <= x)
    if (hi <= KS_FRAGS) {
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (tf.s_foff[mid] <= x) lo = mid;
            else hi = mid;
        }
        return rs.in[(int64_t)tf.s_fstart[lo] + (int64_t)(x - tf.s_foff[lo])];
    }
    const uint32_t *fo = rs.foff + tf.f0;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (fo[mid] <= x) lo = mid;
        else hi = mid;
    }
    return rs.in[(int64_t)rs.fstart[tf.f0 + lo] + (int64_t)(x - fo[lo])];
}

__global__ __launch_bounds__(KS_THREADS) void k_kryo_len16(RecSrc rs, int64_t n, uint32_t *__restrict__ agg) {
    __shared__ uint32_t s_w[KS_THREADS / 64];
    __shared__ uint32_t s_frag[2 * KS_FRAGS];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t t0 = (int64_t)blockIdx.x * KS_TILE;
    const int64_t tn = min((int64_t)KS_TILE, n - t0);
    const TileFrags tf = tile_frags(rs, blockIdx.x, s_frag);
    if (tf.f0 >= 0) {
        stage_frags(rs, tf, tid);
        __syncthreads();
    }
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < KS_ITEMS; ++k) {
        const int64_t i = (int64_t)k * KS_THREADS + tid;
        if (i < tn) {
            const uint4 r = load_rec(rs, tf, t0 + i);
            sum += 2u + varlong_len(zigzag((uint64_t)r.x | ((uint64_t)r.y << 32))) +
                   varlong_len(zigzag((uint64_t)r.z | ((uint64_t)r.w << 32)));
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_xor(sum, d, 64);
    if (lane == 0) s_w[w] = sum;
    __syncthreads();
    if (tid == 0) {
        uint32_t t = 0;
        for (int q = 0; q < KS_THREADS / 64; ++q) t += s_w[q];
        agg[blockIdx.x] = t;
    }
}

// Per serializer (decoder) tile: its 64-bit byte (token) prefix (the scan's in-block prefix + the totals of the
// blocks before) and the first segment whose first record is at or after the tile's start
// (lower bound of t0 in rec_off[0..R]), one thread per tile.  The serializer then needs two
// scalar loads instead of a wave's dependent search after its records land.
__global__ __launch_bounds__(256) void k_ser_tile_info(const uint64_t *__restrict__ excl,
                                                       const uint64_t *__restrict__ btot, int64_t tiles,
                                                       const uint32_t *__restrict__ rec_off, int R,
                                                       uint64_t *__restrict__ tbase, uint32_t *__restrict__ tp0) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= tiles) return;
    uint64_t b = excl[t];
    for (int64_t i = 0; i < t / TS_BLOCK; ++i) b += btot[i];
    tbase[t] = b;
    if (!rec_off) return;  // the decoder's tiles: the prefix only
    const int64_t t0 = t * KS_TILE;
    int lo = 0, hi = R + 1;  // first p with rec_off[p] >= t0
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)rec_off[mid] < t0) lo = mid + 1;
        else hi = mid;
    }
    tp0[t] = (uint32_t)lo;
}

// nontemporal stream stores, as the map's K4 (A/B: -DSGX_KRYO_NT=0): serialize 2.54 -> 2.51 ms
// at C1 (profiles/r05x_kryo_nt_ab.jsonl)
#ifndef SGX_KRYO_NT
#define SGX_KRYO_NT 1
#endif
__global__ __launch_bounds__(KS_THREADS) void k_kryo_ser16(RecSrc rs, int64_t n,
                                                           uint8_t *__restrict__ out,
                                                           const uint32_t *__restrict__ rec_off, int R,
                                                           int64_t *__restrict__ ser_off,
                                                           const uint64_t *__restrict__ tbase,
                                                           const uint32_t *__restrict__ tp0) {
    __shared__ __attribute__((aligned(16))) uint8_t s_len[KS_TILE];
    __shared__ __attribute__((aligned(16))) uint32_t s_off[KS_TILE];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[KS_TILE * KS_MAXREC + 16];
    __shared__ uint32_t s_wsum[KS_THREADS / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t tile = blockIdx.x;
    const int64_t t0 = (int64_t)tile * KS_TILE;
    const int64_t tn = min((int64_t)KS_TILE, n - t0);

    // the tile's byte prefix and the first partition that starts in it (k_ser_tile_info):
    // two tile-uniform scalar loads, in flight with the record loads
    const uint64_t B = tbase[tile];
    const int P0 = (int)tp0[tile];
    // a padded map's fragment range, staged in s_off (free until the offsets scan below)
    static_assert(2 * KS_FRAGS <= KS_TILE, "fragment staging fits s_off");
    const TileFrags tf = tile_frags(rs, tile, s_off);
    stage_frags(rs, tf, tid);
    for (uint32_t z = tid; z < (KS_TILE * KS_MAXREC + 16) / 16; z += KS_THREADS)
        ((uint4 *)s_out)[z] = make_uint4(0, 0, 0, 0);
    if (tf.f0 >= 0) __syncthreads();
    // lengths, coalesced loads (record t0 + k*256 + tid)
    uint4 rec[KS_ITEMS];
#pragma unroll
    for (int k = 0; k < KS_ITEMS; ++k) {
        const int64_t i = (int64_t)k * KS_THREADS + tid;
        rec[k] = i < tn ? load_rec(rs, tf, t0 + i) : make_uint4(0, 0, 0, 0);
        const uint64_t key = (uint64_t)rec[k].x | ((uint64_t)rec[k].y << 32);
        const uint64_t val = (uint64_t)rec[k].z | ((uint64_t)rec[k].w << 32);
        s_len[i] = i < tn ? (uint8_t)(2u + varlong_len(zigzag(key)) + varlong_len(zigzag(val))) : (uint8_t)0;
    }
    __syncthreads();
    // thread t owns records [KS_ITEMS t, KS_ITEMS (t+1)) for the scan
    uint32_t lv[KS_ITEMS], sum = 0;
#pragma unroll
    for (int j = 0; j < KS_ITEMS; ++j) {
        lv[j] = s_len[tid * KS_ITEMS + j];
        sum += lv[j];
    }
    const uint32_t incl = ks_wave_scan(sum, lane);
    if (lane == 63) s_wsum[w] = incl;
    __syncthreads();
    uint32_t run = incl - sum, agg = 0;
#pragma unroll
    for (uint32_t q = 0; q < KS_THREADS / 64; ++q) {
        if (q < w) run += s_wsum[q];
        agg += s_wsum[q];
    }
    {
#pragma unroll
        for (int j = 0; j < KS_ITEMS; ++j) { s_off[tid * KS_ITEMS + j] = run; run += lv[j]; }
    }
    __syncthreads();
    const uint32_t head = (uint32_t)(B & 15u);

    // encode into LDS at the output's 16 B phase: each record's <= 20 bytes are assembled
    // in registers (shifted to its dword phase) and OR-ed into the zeroed buffer, <= 6
    // ds_or_b32 per record (neighbours share edge dwords)
    uint32_t *s_out32 = (uint32_t *)s_out;
#pragma unroll
    for (int k = 0; k < KS_ITEMS; ++k) {
        const int64_t i = (int64_t)k * KS_THREADS + tid;
        if (i < tn) {
            const uint64_t zk = zigzag((uint64_t)rec[k].x | ((uint64_t)rec[k].y << 32));
            const uint64_t zv = zigzag((uint64_t)rec[k].z | ((uint64_t)rec[k].w << 32));
            const uint32_t Lk = varlong_len(zk), Lv = varlong_len(zv);
            uint64_t klo, vlo;
            uint32_t khi, vhi;
            varlong_bytes(zk, Lk, klo, khi);
            varlong_bytes(zv, Lv, vlo, vhi);
            const uint32_t p = head + s_off[i];
            const uint32_t ph = 8u * (p & 3u);
            uint64_t w[3] = {0ull, 0ull, 0ull};
            or_shifted(w, 0x09ull, 0ull, ph);
            or_shifted(w, klo, khi, ph + 8u);
            or_shifted(w, 0x09ull, 0ull, ph + 8u * (1u + Lk));
            or_shifted(w, vlo, vhi, ph + 8u * (2u + Lk));
            const uint32_t nd = ((p & 3u) + 2u + Lk + Lv + 3u) >> 2;
            uint32_t *dst = s_out32 + (p >> 2);
#pragma unroll
            for (int d = 0; d < 6; ++d)
                if ((uint32_t)d < nd) atomicOr(dst + d, (uint32_t)(w[d >> 1] >> (32 * (d & 1))));
        }
    }
    __syncthreads();

    // write [B, B + agg): whole 16 B words with vector stores, the edge words byte by byte
    const uint32_t span = head + agg;
    const uint32_t nwords = (span + 15u) / 16u;
    uint8_t *gbase = out + (B - head);
    for (uint32_t wd = tid; wd < nwords; wd += KS_THREADS) {
        const uint32_t lo = wd * 16u;
        if (lo >= head && lo + 16u <= span) {
#if SGX_KRYO_NT
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(((const v4u *)s_out)[wd], (v4u *)(gbase + lo));
#else
            *(uint4 *)(gbase + lo) = ((const uint4 *)s_out)[wd];
#endif
        } else {
            for (uint32_t b = max(lo, head); b < min(lo + 16u, span); ++b) gbase[b] = s_out[b];
        }
    }

    // byte offsets of the partitions whose first record is in this tile (the last tile also
    // writes those that start at n: the total)
    const int64_t t1 = t0 + tn;
    const bool last = t1 >= n;
    for (int p = P0 + (int)tid; p <= R; p += KS_THREADS) {
        const int64_t ro = (int64_t)rec_off[p];
        if (ro < t1) ser_off[p] = (int64_t)(B + s_off[ro - t0]);
        else if (last && ro == n) ser_off[p] = (int64_t)(B + agg);
        else break;
    }
}

// ------------------------------------------------------------------------------------
// Kryo (Long, Long) stream -> 16 B records (the reduce side of a Kryo shuffle: what
// KryoDeserializationStream.asKeyValueIterator does in UcxShuffleReader.read,
// spark_3_0/UcxShuffleReader.scala:137-145).
//
// The stream is [class][varlong][class][varlong]... and is locally tokenizable: a class
// byte (0x09) and a varlong's last byte have the top bit clear, every other varlong byte
// has it set -- except a 9-byte varlong's last byte, which may have it set; that byte is the
// 9th of a run of 9 high bytes (runs are at most 9 long: a varlong is framed by class
// bytes).  So "token end" = a low byte, or a high byte after 8 high bytes; every record
// holds exactly 4 token ends, and record k+1 starts right after token end 4k+3.
// Reduce-then-scan: (1) every tile of 16 KB counts its token ends, (2) the tile counts are
// scanned, (3) every tile stages its bytes in LDS, flags its token ends again (64 bytes per
// thread), and the thread holding token end 4k+3 parses record k+1 from the next byte
// (record 0 from byte 0) with a branch-free varlong decode.  Class bytes are checked,
// reads stay below B, writes below out_cap; err bit 1 = malformed stream.
// ------------------------------------------------------------------------------------
constexpr int KD_THREADS = 256, KD_BYTES = 64, KD_TILE = KD_THREADS * KD_BYTES;
constexpr int KD_STAGE = 16 + KD_TILE + 64;  // bytes [t0 - 16, t0 + KD_TILE + 64) of the stream

// The stage holds one pad dword after every 16 (64 bytes): a thread's bytes start 64 bytes
// after its neighbour's, so unpadded its window reads hit the same few banks as every
// other lane's; padded, lane t's dwords sit 17 t apart (distinct banks).
constexpr int KD_STAGE_DW = KD_STAGE / 4 + KD_STAGE / 64 + 8;
__device__ __forceinline__ uint32_t kd_pad(uint32_t dw) { return dw + (dw >> 4); }

// 24 bytes of the LDS stage from byte offset q (q + 28 <= KD_STAGE) as 3 little-endian u64
__device__ __forceinline__ void lds_window(const uint32_t *s32, uint32_t q, uint64_t W[3]) {
    const uint32_t b = q >> 2, sh = 8u * (q & 3u);
    uint32_t d[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) d[i] = s32[kd_pad(b + i)];
    uint32_t x[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = sh ? (d[i] >> sh) | (d[i + 1] << (32u - sh)) : d[i];
    W[0] = (uint64_t)x[0] | ((uint64_t)x[1] << 32);
    W[1] = (uint64_t)x[2] | ((uint64_t)x[3] << 32);
    W[2] = (uint64_t)x[4] | ((uint64_t)x[5] << 32);
}

// the 8 bytes at byte offset q (0 <= q <= 16) of the window, and the byte at q + 8
__device__ __forceinline__ uint64_t win8(const uint64_t W[3], uint32_t q) {
    const uint32_t r = 8u * (q & 7u);
    const uint64_t a = q < 8 ? W[0] : (q < 16 ? W[1] : W[2]);
    const uint64_t b = q < 8 ? W[1] : W[2];
    return r ? (a >> r) | (b << (64u - r)) : a;
}

// Kryo 4 Input.readVarLong(false) on 9 window bytes: lo = bytes 0..7, hi = byte 8.
__device__ __forceinline__ uint64_t varlong_decode(uint64_t lo, uint32_t hi, uint32_t &L) {
    const uint64_t m = ~lo & 0x8080808080808080ull;  // bytes without the continuation bit
    L = m ? (uint32_t)(__ffsll((long long)m) - 1) / 8u + 1u : 9u;
    const uint64_t keep = L >= 8 ? ~0ull : ((1ull << (8 * L)) - 1ull);
    const uint64_t x = lo & keep;
    uint64_t z = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) z |= ((x >> (8 * i)) & 0x7Full) << (7 * i);
    if (L == 9) z |= (uint64_t)(hi & 0xFFu) << 56;
    return (z >> 1) ^ (0ull - (z & 1ull));
}

// one (Long, Long) record at stage offset q (stream position p); false if malformed
__device__ __forceinline__ bool parse_pair_lds(const uint32_t *s32, uint32_t q, int64_t p, int64_t B,
                                               uint64_t kv[2]) {
    uint64_t W[3];
    lds_window(s32, q, W);
    uint32_t L1, L2;
    const uint64_t lo1 = win8(W, 1);
    kv[0] = varlong_decode(lo1, (uint32_t)(win8(W, 9) & 0xFFu), L1);
    const uint32_t c2 = 1u + L1;
    const uint32_t cls2 = (uint32_t)(win8(W, c2) & 0xFFu);
    kv[1] = varlong_decode(win8(W, c2 + 1u), (uint32_t)(win8(W, c2 + 9u) & 0xFFu), L2);
    return (W[0] & 0xFFu) == 0x09u && cls2 == 0x09u && p + 2 + (int64_t)L1 + (int64_t)L2 <= B;
}

// top bits of a dword's 4 bytes as a nibble (byte 0 -> bit 0): one multiply
__device__ __forceinline__ uint32_t top_bits4(uint32_t d) {
    return (((d >> 7) & 0x01010101u) * 0x10204080u) >> 28;
}

// token-end mask of the 64 bytes [p0, p0 + 64) given bytes [p0 - 16, p0 + 64) as q[0..4]:
// per 32-byte half, h = top bits of bytes [ph - 16, ph + 32) (48 bits, missing bytes 0);
// a byte ends a token if its top bit is clear or it and the 8 bytes before it are all high
__device__ __forceinline__ uint64_t tok_mask64(const uint4 q[5], int64_t p0, int64_t B) {
    uint32_t nib[20];
#pragma unroll
    for (int v = 0; v < 5; ++v) {
        nib[4 * v + 0] = top_bits4(q[v].x);
        nib[4 * v + 1] = top_bits4(q[v].y);
        nib[4 * v + 2] = top_bits4(q[v].z);
        nib[4 * v + 3] = top_bits4(q[v].w);
    }
    uint64_t tok = 0;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const int64_t ph = p0 + 32 * half;
        uint64_t h = 0;
#pragma unroll
        for (int k = 0; k < 12; ++k) h |= (uint64_t)nib[8 * half + k] << (4 * k);
        // bytes before the stream start or at / past B do not exist
        const int64_t lo = -(ph - 16), hi = B - (ph - 16);  // valid bit range [lo, hi)
        const uint64_t above = lo <= 0 ? ~0ull : (lo >= 64 ? 0ull : ~0ull << lo);
        const uint64_t below = hi >= 64 ? ~0ull : (hi <= 0 ? 0ull : (1ull << hi) - 1ull);
        h &= above & below;
        uint64_t a = h & (h << 1);
        a &= a << 2;
        a &= a << 4;
        a &= h << 8;  // bit i: bytes i-8 .. i all high
        const uint64_t t = ((~h | a) >> 16) & 0xFFFFFFFFull & below >> 16;
        tok |= t << (32 * half);
    }
    return tok;
}

__global__ __launch_bounds__(KD_THREADS) void k_kryo_tok(const uint8_t *__restrict__ in, int64_t B,
                                                         uint32_t *__restrict__ agg) {
    __shared__ uint32_t s_w[KD_THREADS / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t p0 = (int64_t)blockIdx.x * KD_TILE + (int64_t)tid * KD_BYTES;
    uint32_t cnt = 0;
    if (p0 < B) {  // bytes [p0 - 16, p0 + 64) are readable (the buffer holds B + 64)
        uint4 q[5];
#pragma unroll
        for (int v = 0; v < 5; ++v) {
            const int64_t g = p0 - 16 + 16 * v;
            q[v] = g >= 0 ? *(const uint4 *)(in + g) : make_uint4(0, 0, 0, 0);
        }
        cnt = (uint32_t)__popcll(tok_mask64(q, p0, B));
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
    if (lane == 0) s_w[w] = cnt;
    __syncthreads();
    if (tid == 0) {
        uint32_t t = 0;
        for (int q = 0; q < KD_THREADS / 64; ++q) t += s_w[q];
        agg[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(KD_THREADS) void k_kryo_deser16(const uint8_t *__restrict__ in, int64_t B,
                                                             uint4 *__restrict__ out, int64_t out_cap,
                                                             const uint64_t *__restrict__ tbase,
                                                             uint32_t *ticket_err, int64_t *count_out) {
    __shared__ uint32_t s32[KD_STAGE_DW];
    __shared__ uint32_t s_wsum[KD_THREADS / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t tile = blockIdx.x;
    const int64_t t0 = (int64_t)tile * KD_TILE;
    const int64_t p0 = t0 + (int64_t)tid * KD_BYTES;
    // stage [t0 - 16, t0 + KD_TILE + 64), padded (kd_pad): the buffer is readable to B + 64
    // (16 B-aligned); a 16 B chunk stays inside one 64 B group, so its dwords stay adjacent
    for (uint32_t i = tid; i < KD_STAGE / 16; i += KD_THREADS) {
        const int64_t g = t0 - 16 + 16 * (int64_t)i;
        const uint4 v = (g >= 0 && g + 16 <= B + 64) ? *(const uint4 *)(in + g) : make_uint4(0, 0, 0, 0);
        uint32_t *d = s32 + kd_pad(4 * i);
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    }
    __syncthreads();
    // this thread's token ends from its own bytes [p0 - 16, p0 + 64): stage dwords 16 t ..
    // 16 t + 19, at padded addresses 17 t + ... (distinct banks across the wave)
    uint4 q5[5];
#pragma unroll
    for (int v = 0; v < 5; ++v) {
        const uint32_t b = 16u * tid + 4u * v;
        q5[v] = make_uint4(s32[kd_pad(b)], s32[kd_pad(b + 1)], s32[kd_pad(b + 2)], s32[kd_pad(b + 3)]);
    }
    const uint64_t tok = tok_mask64(q5, p0, B);
    const uint32_t cnt = (uint32_t)__popcll(tok);
    const uint32_t incl = ks_wave_scan(cnt, lane);
    if (lane == 63) s_wsum[w] = incl;
    __syncthreads();
    uint32_t texcl = incl - cnt;
#pragma unroll
    for (uint32_t qq = 0; qq < KD_THREADS / 64; ++qq)
        if (qq < w) texcl += s_wsum[qq];
    const uint64_t c0 = tbase[tile] + texcl;  // global index of this thread's first token end
    bool bad = false;
    if (p0 == 0 && B > 0) {
        uint64_t kv[2];
        if (!parse_pair_lds(s32, 16u, 0, B, kv) || out_cap < 1) bad = true;
        else out[0] = make_uint4((uint32_t)kv[0], (uint32_t)(kv[0] >> 32), (uint32_t)kv[1], (uint32_t)(kv[1] >> 32));
    }
    // record ends = token ends of global index 3 mod 4: skip to the first, then every 4th
    // set bit (one iteration per record, so the lanes of a wave stay within one iteration)
    uint64_t m = tok;
    const uint32_t r0 = (3u - (uint32_t)(c0 & 3u)) & 3u;
    for (uint32_t i = 0; i < r0; ++i) m &= m - 1;
    for (uint64_t c = c0 + r0; m; c += 4) {
        const int j = __ffsll((long long)m) - 1;
        m &= m - 1;
        m &= m - 1;
        m &= m - 1;
        m &= m - 1;
        if (p0 + j + 1 >= B) continue;
        const int64_t k = (int64_t)(c >> 2) + 1;
        uint64_t kv[2];
        const uint32_t q = 16u + tid * KD_BYTES + (uint32_t)j + 1u;  // <= 16 + KD_TILE: window fits
        if (k >= out_cap || !parse_pair_lds(s32, q, p0 + j + 1, B, kv)) { bad = true; continue; }
        out[k] = make_uint4((uint32_t)kv[0], (uint32_t)(kv[0] >> 32), (uint32_t)kv[1], (uint32_t)(kv[1] >> 32));
    }
    if (p0 <= B - 1 && B - 1 < p0 + KD_BYTES) {  // the thread holding the last byte: totals
        const uint64_t cend = c0 + cnt;
        if (cend & 3u) bad = true;
        *count_out = (int64_t)(cend >> 2);
    }
    if (bad) atomicOr(&ticket_err[1], 2u);
}

}  // namespace

int64_t kryo_deser16_tiles(int64_t bytes) { return (bytes + KD_TILE - 1) / KD_TILE; }

int64_t kryo_work_bytes(int64_t tiles) {
    return (tiles + (tiles + TS_BLOCK - 1) / TS_BLOCK + 1) * 8 + tiles * 4 + (tiles + 1) * 4 + 8 + tiles * 12;
}

// workspace: excl[tiles] u64 | btot[nblk] u64 | agg[tiles] u32 | tile_f0[tiles + 1] u32 (the
// serializer of a padded map) | (8 B aligned) tbase[tiles] u64 | tp0[tiles] u32 (serializer)
static void work_split(uint64_t *ws, int64_t tiles, uint64_t **excl, uint64_t **btot, uint32_t **agg,
                       int64_t *nblk) {
    *nblk = (tiles + TS_BLOCK - 1) / TS_BLOCK;
    *excl = ws;
    *btot = ws + tiles;
    *agg = (uint32_t *)(ws + tiles + *nblk + 1);
}

// the tile-info arrays behind agg[tiles] | tile_f0[tiles + 1]
static void tile_info_split(uint32_t *agg, int64_t tiles, uint64_t **tbase, uint32_t **tp0) {
    *tbase = (uint64_t *)(((uintptr_t)(agg + 2 * tiles + 1) + 7) & ~(uintptr_t)7);
    *tp0 = (uint32_t *)(*tbase + tiles);
}

hipError_t launch_kryo_deser16(const void *in, int64_t bytes, void *out, int64_t out_cap, uint64_t *status,
                               uint32_t *ticket_err, int64_t *count_out, hipStream_t st) {
    if (bytes <= 0) return hipSuccess;
    const int64_t tiles = kryo_deser16_tiles(bytes);
    uint64_t *excl, *btot;
    uint32_t *agg;
    int64_t nblk;
    work_split(status, tiles, &excl, &btot, &agg, &nblk);
    hipLaunchKernelGGL(k_kryo_tok, dim3((unsigned)tiles), dim3(KD_THREADS), 0, st, (const uint8_t *)in, bytes, agg);
    hipLaunchKernelGGL(k_tile_scan64, dim3((unsigned)nblk), dim3(TS_THREADS), 0, st, (const uint32_t *)agg, tiles,
                       excl, btot);
    uint64_t *tbase;
    uint32_t *tp0;
    tile_info_split(agg, tiles, &tbase, &tp0);
    hipLaunchKernelGGL(k_ser_tile_info, dim3((unsigned)((tiles + 255) / 256)), dim3(256), 0, st,
                       (const uint64_t *)excl, (const uint64_t *)btot, tiles, nullptr, 0, tbase, tp0);
    hipLaunchKernelGGL(k_kryo_deser16, dim3((unsigned)tiles), dim3(KD_THREADS), 0, st, (const uint8_t *)in, bytes,
                       (uint4 *)out, out_cap, (const uint64_t *)tbase, ticket_err, count_out);
    return hipGetLastError();
}

int64_t kryo_ser16_tiles(int64_t n) { return (n + KS_TILE - 1) / KS_TILE; }

hipError_t launch_kryo_ser16(const void *in, int64_t n, void *out, const uint32_t *rec_off, int R, int64_t *ser_off,
                             uint64_t *work, hipStream_t st, const uint32_t *frag, int64_t nfrag,
                             const uint32_t *ovf) {
    if (n <= 0) return hipSuccess;
    if (frag && (nfrag <= 0 || nfrag >= (int64_t)INT32_MAX || !ovf)) return hipErrorInvalidValue;
    const int64_t tiles = kryo_ser16_tiles(n);
    uint64_t *excl, *btot;
    uint32_t *agg;
    int64_t nblk;
    work_split(work, tiles, &excl, &btot, &agg, &nblk);
    RecSrc rs;
    rs.in = (const uint4 *)in;
    if (frag) {  // [fstart nfrag][foff nfrag][cnt nfrag]
        rs.fstart = frag;
        rs.foff = frag + nfrag;
        rs.cnt = frag + 2 * nfrag;
        rs.nf = nfrag;
        rs.ovf = ovf;
        rs.tile_f0 = agg + tiles;
        hipLaunchKernelGGL(k_tile_frags, dim3((unsigned)((nfrag + 255) / 256)), dim3(256), 0, st, rs, tiles,
                           agg + tiles);
    }
    hipLaunchKernelGGL(k_kryo_len16, dim3((unsigned)tiles), dim3(KS_THREADS), 0, st, rs, n, agg);
    hipLaunchKernelGGL(k_tile_scan64, dim3((unsigned)nblk), dim3(TS_THREADS), 0, st, (const uint32_t *)agg, tiles,
                       excl, btot);
    uint64_t *tbase;
    uint32_t *tp0;
    tile_info_split(agg, tiles, &tbase, &tp0);
    hipLaunchKernelGGL(k_ser_tile_info, dim3((unsigned)((tiles + 255) / 256)), dim3(256), 0, st,
                       (const uint64_t *)excl, (const uint64_t *)btot, tiles, rec_off, R, tbase, tp0);
    hipLaunchKernelGGL(k_kryo_ser16, dim3((unsigned)tiles), dim3(KS_THREADS), 0, st, rs, n, (uint8_t *)out, rec_off, R,
                       ser_off, (const uint64_t *)tbase, (const uint32_t *)tp0);
    return hipGetLastError();
}

}  // namespace sgx
