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
// One pass over the partition-contiguous 16 B records (K4's output): a tile of 2048
// records computes every record's encoded length, scans them (block scan + decoupled
// look-back over tiles for the 64-bit byte prefix), encodes the tile into LDS at its final
// alignment, and writes it out with 16 B stores (byte stores only for the two edge words
// it shares with the neighbouring tiles).  The tile that holds a partition's first record
// also writes that partition's byte offset.  HBM-bound: 16 B read + the encoded bytes
// written per record.
#include "sgx_internal.h"

namespace sgx {
namespace {

constexpr int KS_THREADS = 256, KS_ITEMS = 8, KS_TILE = KS_THREADS * KS_ITEMS;
constexpr int KS_MAXREC = 20;  // 2 class bytes + 2 x 9 varlong bytes
constexpr uint64_t KS_AGG = 1ull << 62, KS_PRE = 2ull << 62, KS_VAL = (1ull << 62) - 1;

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


// Decoupled look-back by one whole wave (call from wave 0 only, every lane): publishes this
// tile's aggregate, then reads 64 predecessors' status words per step, from the nearest
// back; stops at the first inclusive prefix.  A walk of d tiles costs ~d/64 L2 round trips
// (one lane walking one tile per round trip made every tile wait ~tens of µs).  Returns the
// exclusive prefix (every lane); publishes the inclusive one.  Bounded spin -> err bit 0.
__device__ uint64_t wave_look_back(uint64_t *status, uint32_t tile, uint64_t agg, uint32_t lane, uint32_t *err) {
    if (tile == 0) {
        if (lane == 0) __hip_atomic_store(&status[0], KS_PRE | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&status[tile], KS_AGG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t excl = 0;
    int64_t j = (int64_t)tile - 1;  // lane l looks at tile j - l
    uint32_t spins = 0;
    while (true) {
        const int64_t idx = j - (int64_t)lane;
        const uint64_t st = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : KS_PRE;  // before tile 0: prefix 0
        const uint64_t flag = st & ~KS_VAL;
        const uint64_t pre = __ballot(flag == KS_PRE);
        const uint64_t notready = __ballot(flag == 0);
        const uint32_t last = pre ? (uint32_t)__ffsll((long long)pre) - 1u : 63u;  // lanes 0..last count
        const uint64_t upto = last == 63u ? ~0ull : ((1ull << (last + 1u)) - 1ull);
        if (notready & upto) {
            if (++spins > (1u << 24)) {
                if (lane == 0) atomicOr(err, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t v = lane <= last ? (st & KS_VAL) : 0ull;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        excl += v;
        if (pre) break;
        j -= 64;
    }
    if (lane == 0)
        __hip_atomic_store(&status[tile], KS_PRE | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

__global__ __launch_bounds__(KS_THREADS) void k_kryo_ser16(const uint4 *__restrict__ in, int64_t n,
                                                           uint8_t *__restrict__ out,
                                                           const uint32_t *__restrict__ rec_off, int R,
                                                           int64_t *__restrict__ ser_off, uint64_t *status,
                                                           uint32_t *ticket_err) {
    __shared__ __attribute__((aligned(16))) uint8_t s_len[KS_TILE];
    __shared__ __attribute__((aligned(16))) uint32_t s_off[KS_TILE];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[KS_TILE * KS_MAXREC + 16];
    __shared__ uint32_t s_tile, s_wsum[KS_THREADS / 64];
    __shared__ uint64_t s_base;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(&ticket_err[0], 1u);  // dispatch-order tiles: look-back progress
    __syncthreads();
    const uint32_t tile = s_tile;
    const int64_t t0 = (int64_t)tile * KS_TILE;
    const int64_t tn = min((int64_t)KS_TILE, n - t0);

    for (uint32_t z = tid; z < (KS_TILE * KS_MAXREC + 16) / 16; z += KS_THREADS)
        ((uint4 *)s_out)[z] = make_uint4(0, 0, 0, 0);
    // lengths, coalesced loads (record t0 + k*256 + tid)
    uint4 rec[KS_ITEMS];
#pragma unroll
    for (int k = 0; k < KS_ITEMS; ++k) {
        const int64_t i = (int64_t)k * KS_THREADS + tid;
        rec[k] = i < tn ? in[t0 + i] : make_uint4(0, 0, 0, 0);
        const uint64_t key = (uint64_t)rec[k].x | ((uint64_t)rec[k].y << 32);
        const uint64_t val = (uint64_t)rec[k].z | ((uint64_t)rec[k].w << 32);
        s_len[i] = i < tn ? (uint8_t)(2u + varlong_len(zigzag(key)) + varlong_len(zigzag(val))) : (uint8_t)0;
    }
    __syncthreads();
    // thread t owns records [8t, 8t+8) for the scan
    const uint2 l8 = ((const uint2 *)s_len)[tid];
    uint32_t lv[KS_ITEMS], sum = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        lv[j] = (l8.x >> (8 * j)) & 0xFFu;
        lv[4 + j] = (l8.y >> (8 * j)) & 0xFFu;
    }
#pragma unroll
    for (int j = 0; j < KS_ITEMS; ++j) sum += lv[j];
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
        uint32_t o[KS_ITEMS];
#pragma unroll
        for (int j = 0; j < KS_ITEMS; ++j) { o[j] = run; run += lv[j]; }
        ((uint4 *)s_off)[2 * tid] = make_uint4(o[0], o[1], o[2], o[3]);
        ((uint4 *)s_off)[2 * tid + 1] = make_uint4(o[4], o[5], o[6], o[7]);
    }
    // decoupled look-back over tiles (wave 0): 64-bit byte prefix
    if (w == 0) {
        const uint64_t excl = wave_look_back(status, tile, agg, lane, &ticket_err[1]);
        if (lane == 0) s_base = excl;
    }
    __syncthreads();
    const uint64_t B = s_base;
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
            *(uint4 *)(gbase + lo) = ((const uint4 *)s_out)[wd];
        } else {
            for (uint32_t b = max(lo, head); b < min(lo + 16u, span); ++b) gbase[b] = s_out[b];
        }
    }

    // byte offsets of the partitions whose first record is in this tile (the last tile also
    // writes those that start at n: the total)
    const int64_t t1 = t0 + tn;
    const bool last = t1 >= n;
    int lo = 0, hi = R + 1;  // first p with rec_off[p] >= t0
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)rec_off[mid] < t0) lo = mid + 1; else hi = mid;
    }
    for (int p = lo + (int)tid; p <= R; p += KS_THREADS) {
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
// holds exactly 4 token ends, and record k+1 starts right after token end 4k+3.  One pass:
// flag the token ends of a tile (32 bytes per thread), count them (block scan + decoupled
// look-back over tiles), and the thread holding token end 4k+3 parses record k+1 from the
// next byte (record 0 from byte 0).  Class bytes are checked, reads stay below B, writes
// below out_cap; err bit 1 = malformed stream, bit 0 = look-back gave up.
// ------------------------------------------------------------------------------------
constexpr int KD_THREADS = 256, KD_BYTES = 32, KD_TILE = KD_THREADS * KD_BYTES;

__device__ __forceinline__ bool parse_pair(const uint8_t *__restrict__ in, int64_t B, int64_t p, uint64_t *kv) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
        if (p >= B || in[p] != 0x09) return false;
        ++p;
        uint64_t z = 0;
        for (int i = 0; i < 9; ++i) {
            if (p >= B) return false;
            const uint64_t b = in[p++];
            if (i == 8) { z |= b << 56; break; }
            z |= (b & 0x7Full) << (7 * i);
            if (!(b & 0x80ull)) break;
        }
        kv[f] = (z >> 1) ^ (0ull - (z & 1ull));
    }
    return true;
}

__global__ __launch_bounds__(KD_THREADS) void k_kryo_deser16(const uint8_t *__restrict__ in, int64_t B,
                                                             uint4 *__restrict__ out, int64_t out_cap,
                                                             uint64_t *status, uint32_t *ticket_err,
                                                             int64_t *count_out) {
    __shared__ uint32_t s_tile, s_wsum[KD_THREADS / 64];
    __shared__ uint64_t s_base;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(&ticket_err[0], 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const int64_t p0 = (int64_t)tile * KD_TILE + (int64_t)tid * KD_BYTES;
    // bytes [p0 - 16, p0 + 32): the 8 before p0 decide whether an early high byte is a 9th
    uint4 q[3];
    q[0] = p0 >= 16 ? *(const uint4 *)(in + p0 - 16) : make_uint4(0, 0, 0, 0);
    q[1] = p0 < B ? *(const uint4 *)(in + p0) : make_uint4(0, 0, 0, 0);
    q[2] = p0 + 16 < B ? *(const uint4 *)(in + p0 + 16) : make_uint4(0, 0, 0, 0);
    uint64_t hi = 0;  // bit i: byte p0 - 16 + i has its top bit set (and exists)
#pragma unroll
    for (int v = 0; v < 3; ++v) {
        const uint32_t d[4] = {q[v].x, q[v].y, q[v].z, q[v].w};
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int i = v * 16 + c * 4 + b;
                const int64_t pos = p0 - 16 + i;
                if (pos >= 0 && pos < B && ((d[c] >> (8 * b + 7)) & 1u)) hi |= 1ull << i;
            }
    }
    uint32_t tok = 0;  // bit j: byte p0 + j ends a token
#pragma unroll
    for (int j = 0; j < KD_BYTES; ++j) {
        const int i = 16 + j;
        if (p0 + j >= B) break;
        const bool h = (hi >> i) & 1ull;
        const bool ninth = h && ((hi >> (i - 8)) & 0xFFull) == 0xFFull;
        if (!h || ninth) tok |= 1u << j;
    }
    const uint32_t cnt = (uint32_t)__popc(tok);
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) s_wsum[w] = incl;
    __syncthreads();
    uint32_t texcl = incl - cnt, agg = 0;
#pragma unroll
    for (uint32_t qq = 0; qq < KD_THREADS / 64; ++qq) {
        if (qq < w) texcl += s_wsum[qq];
        agg += s_wsum[qq];
    }
    if (w == 0) {
        const uint64_t excl = wave_look_back(status, tile, agg, lane, &ticket_err[1]);
        if (lane == 0) s_base = excl;
    }
    __syncthreads();
    uint64_t c = s_base + texcl;  // global index of this thread's first token end
    bool bad = false;
    if (p0 == 0 && B > 0) {
        uint64_t kv[2];
        if (!parse_pair(in, B, 0, kv) || out_cap < 1) bad = true;
        else out[0] = make_uint4((uint32_t)kv[0], (uint32_t)(kv[0] >> 32), (uint32_t)kv[1], (uint32_t)(kv[1] >> 32));
    }
    for (uint32_t m = tok; m; m &= m - 1, ++c) {
        const int j = __ffs(m) - 1;
        if ((c & 3u) != 3u || p0 + j + 1 >= B) continue;
        const int64_t k = (int64_t)(c >> 2) + 1;
        uint64_t kv[2];
        if (k >= out_cap || !parse_pair(in, B, p0 + j + 1, kv)) { bad = true; continue; }
        out[k] = make_uint4((uint32_t)kv[0], (uint32_t)(kv[0] >> 32), (uint32_t)kv[1], (uint32_t)(kv[1] >> 32));
    }
    if (p0 <= B - 1 && B - 1 < p0 + KD_BYTES) {  // the thread holding the last byte: totals
        if (c & 3u) bad = true;
        *count_out = (int64_t)(c >> 2);
    }
    if (bad) atomicOr(&ticket_err[1], 2u);
}

}  // namespace

int64_t kryo_deser16_tiles(int64_t bytes) { return (bytes + KD_TILE - 1) / KD_TILE; }

hipError_t launch_kryo_deser16(const void *in, int64_t bytes, void *out, int64_t out_cap, uint64_t *status,
                               uint32_t *ticket_err, int64_t *count_out, hipStream_t st) {
    if (bytes <= 0) return hipSuccess;
    const int64_t tiles = kryo_deser16_tiles(bytes);
    hipLaunchKernelGGL(k_kryo_deser16, dim3((unsigned)tiles), dim3(KD_THREADS), 0, st, (const uint8_t *)in, bytes,
                       (uint4 *)out, out_cap, status, ticket_err, count_out);
    return hipGetLastError();
}

int64_t kryo_ser16_tiles(int64_t n) { return (n + KS_TILE - 1) / KS_TILE; }

hipError_t launch_kryo_ser16(const void *in, int64_t n, void *out, const uint32_t *rec_off, int R, int64_t *ser_off,
                             uint64_t *status, uint32_t *ticket_err, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t tiles = kryo_ser16_tiles(n);
    hipLaunchKernelGGL(k_kryo_ser16, dim3((unsigned)tiles), dim3(KS_THREADS), 0, st, (const uint4 *)in, n,
                       (uint8_t *)out, rec_off, R, ser_off, status, ticket_err);
    return hipGetLastError();
}

}  // namespace sgx
