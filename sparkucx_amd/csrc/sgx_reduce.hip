// Reduce-side kernels: what UcxShuffleReader.read does after the fetch
// (shuffle/compat/spark_3_0/UcxShuffleReader.scala:137-191) for (Long, Long) records whose
// reducer runs are already sorted by key (sgx_read_sorted's LSD digit passes):
//
//   * groupByKey  -- Aggregator.combineValuesByKey with CompactBuffer (mapSideCombine =
//     false): one group per distinct key, values in arrival order (map order, then record
//     order: the canonical sequence of SURVEY §8(a)); the stable sort keeps it.
//   * reduceByKey(_ + _) -- combineValuesByKey with a Long sum: wrapping 64-bit adds, so
//     the order of additions does not change the result.
//
// Groups never span reducers: a key has one partition.  Layout: records {i64 key, i64
// value} little-endian, 16 B each, n < 2^31.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "sgx_internal.h"

namespace sgx {

namespace {

constexpr int RT = 256;        // threads per workgroup
constexpr int RI = 16;         // items per thread
constexpr int RBLK = RT * RI;  // elements per workgroup of the 64-bit scan

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    return x;
}

// exclusive scan of one value per thread over the workgroup; returns the prefix, *total
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t x, uint64_t *scratch, uint64_t *total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
    const uint64_t inc = wave_incl_scan64(x, lane);
    if (lane == 63) scratch[w] = inc;
    __syncthreads();
    uint64_t base = 0, t = 0;
    for (uint32_t v = 0; v < nw; ++v) {
        const uint64_t s = scratch[v];
        if (v < w) base += s;
        t += s;
    }
    __syncthreads();
    *total = t;
    return base + inc - x;
}

}  // namespace

// flags[i] = 1 where a new key starts
__global__ __launch_bounds__(RT) void k_group_flags(const ulonglong2 *__restrict__ rec, int64_t n,
                                                    uint32_t *__restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * RT + threadIdx.x;
    if (i >= n) return;
    flags[i] = (i == 0 || rec[i].x != rec[i - 1].x) ? 1u : 0u;
}

// gid of record i = offs[i] + flags[i] - 1 (offs: exclusive scan of flags).  A group's first
// record writes its key and start; GROUP also copies every value into `values` (same index).
__global__ __launch_bounds__(RT) void k_group_emit(const ulonglong2 *__restrict__ rec, int64_t n,
                                                   const uint32_t *__restrict__ flags,
                                                   const uint32_t *__restrict__ offs, int64_t *__restrict__ keys,
                                                   int64_t *__restrict__ starts, int64_t *__restrict__ values) {
    const int64_t i = (int64_t)blockIdx.x * RT + threadIdx.x;
    if (i >= n) return;
    const ulonglong2 r = rec[i];
    if (flags[i]) {
        const uint32_t g = offs[i];
        keys[g] = (int64_t)r.x;
        if (starts) starts[g] = i;
    }
    if (values) values[i] = (int64_t)r.y;
}

// 64-bit wrapping prefix sums of the values: per-block totals, a one-workgroup scan of the
// totals, then per-block inclusive prefixes P[i] = sum of values[0..i].
__global__ __launch_bounds__(RT) void k_sum_blocks(const ulonglong2 *__restrict__ rec, int64_t n,
                                                   uint64_t *__restrict__ bsum) {
    __shared__ uint64_t scratch[RT / 64];
    const int64_t base = (int64_t)blockIdx.x * RBLK;
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < RI; ++k) {
        const int64_t i = base + (int64_t)k * RT + threadIdx.x;
        if (i < n) s += rec[i].y;
    }
    uint64_t total;
    (void)block_excl_scan64(s, scratch, &total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_scan_bsum(uint64_t *__restrict__ bsum, int64_t nb) {
    __shared__ uint64_t scratch[1024 / 64];
    uint64_t carry = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += 1024) {
        const int64_t b = b0 + threadIdx.x;
        const uint64_t x = b < nb ? bsum[b] : 0;
        uint64_t total;
        const uint64_t ex = block_excl_scan64(x, scratch, &total);
        if (b < nb) bsum[b] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(RT) void k_prefix(const ulonglong2 *__restrict__ rec, int64_t n,
                                               const uint64_t *__restrict__ bpre, uint64_t *__restrict__ P) {
    __shared__ uint64_t scratch[RT / 64];
    const int64_t base = (int64_t)blockIdx.x * RBLK + (int64_t)threadIdx.x * RI;  // thread-contiguous
    uint64_t v[RI], s = 0;
#pragma unroll
    for (int k = 0; k < RI; ++k) {
        const int64_t i = base + k;
        v[k] = i < n ? rec[i].y : 0;
        s += v[k];
    }
    uint64_t total;
    uint64_t run = bpre[blockIdx.x] + block_excl_scan64(s, scratch, &total);
#pragma unroll
    for (int k = 0; k < RI; ++k) {
        const int64_t i = base + k;
        run += v[k];
        if (i < n) P[i] = run;
    }
}

// sums[g] = P[end_g - 1] - P[start_g - 1] (wrapping): the Long sum of the group's values
__global__ __launch_bounds__(RT) void k_group_sums(const uint64_t *__restrict__ P, const int64_t *__restrict__ starts,
                                                   int64_t ngroups, int64_t n, int64_t *__restrict__ sums) {
    const int64_t g = (int64_t)blockIdx.x * RT + threadIdx.x;
    if (g >= ngroups) return;
    const int64_t s = starts[g], e = g + 1 < ngroups ? starts[g + 1] : n;
    sums[g] = (int64_t)(P[e - 1] - (s > 0 ? P[s - 1] : 0ull));
}

// All digit histograms of the sort in one read: hist[d][b] = records whose digit d (byte
// dshift/8 of the record, the top byte of a Long key sign-flipped) is b.  A digit whose
// histogram has a single non-empty bucket is a no-op pass (keys that share that byte) and
// sgx_read_sorted skips it -- Zipf ranks or small-range ids leave most high bytes constant.
template <int RB>
__global__ __launch_bounds__(RT) void k_digit_hist(const uint8_t *__restrict__ rec, int64_t n,
                                                   uint32_t *__restrict__ hist) {
    constexpr int ND = RB == 16 ? 8 : 10;
    __shared__ uint32_t h[ND * 256];
    for (int i = threadIdx.x; i < ND * 256; i += RT) h[i] = 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * RT;
    for (int64_t i = (int64_t)blockIdx.x * RT + threadIdx.x; i < n; i += stride) {
        const uint8_t *r = rec + i * RB;
        uint32_t w[3];
        w[0] = *(const uint32_t *)r;
        w[1] = *(const uint32_t *)(r + 4);
        w[2] = ND > 8 ? *(const uint32_t *)(r + 8) : 0u;
#pragma unroll
        for (int d = 0; d < ND; ++d) {
            uint32_t b = (w[d >> 2] >> ((d & 3) * 8)) & 0xFFu;
            if (RB == 16 && d == 7) b ^= 0x80u;
            atomicAdd(&h[d * 256 + b], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < ND * 256; i += RT)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

hipError_t launch_digit_hist(const void *rec, int64_t n, int rb, uint32_t *hist, int num_cus, hipStream_t st) {
    const int nd = rb == 16 ? 8 : 10;
    hipError_t e = hipMemsetAsync(hist, 0, (size_t)nd * 256 * 4, st);
    if (e != hipSuccess || n <= 0) return e;
    const int64_t want = (n + RT * 16 - 1) / (RT * 16);
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)num_cus * 4));
    if (rb == 16)
        hipLaunchKernelGGL(k_digit_hist<16>, dim3(grid), dim3(RT), 0, st, (const uint8_t *)rec, n, hist);
    else
        hipLaunchKernelGGL(k_digit_hist<100>, dim3(grid), dim3(RT), 0, st, (const uint8_t *)rec, n, hist);
    return hipGetLastError();
}

hipError_t launch_group_flags(const void *rec, int64_t n, uint32_t *flags, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_group_flags, dim3((unsigned)((n + RT - 1) / RT)), dim3(RT), 0, st,
                       (const ulonglong2 *)rec, n, flags);
    return hipGetLastError();
}

hipError_t launch_group_emit(const void *rec, int64_t n, const uint32_t *flags, const uint32_t *offs,
                             int64_t *keys, int64_t *starts, int64_t *values, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_group_emit, dim3((unsigned)((n + RT - 1) / RT)), dim3(RT), 0, st,
                       (const ulonglong2 *)rec, n, flags, offs, keys, starts, values);
    return hipGetLastError();
}

int64_t prefix64_blocks(int64_t n) { return (n + RBLK - 1) / RBLK; }

hipError_t launch_group_sums(const void *rec, int64_t n, const int64_t *starts, int64_t ngroups,
                             uint64_t *bsum, uint64_t *P, int64_t *sums, hipStream_t st) {
    if (n <= 0 || ngroups <= 0) return hipSuccess;
    const int64_t nb = prefix64_blocks(n);
    const ulonglong2 *r = (const ulonglong2 *)rec;
    hipLaunchKernelGGL(k_sum_blocks, dim3((unsigned)nb), dim3(RT), 0, st, r, n, bsum);
    hipLaunchKernelGGL(k_scan_bsum, dim3(1), dim3(1024), 0, st, bsum, nb);
    hipLaunchKernelGGL(k_prefix, dim3((unsigned)nb), dim3(RT), 0, st, r, n, (const uint64_t *)bsum, P);
    hipLaunchKernelGGL(k_group_sums, dim3((unsigned)((ngroups + RT - 1) / RT)), dim3(RT), 0, st,
                       (const uint64_t *)P, starts, ngroups, n, sums);
    return hipGetLastError();
}

// Map-side combine (reduceByKey's mapSideCombine = true): the combiners of one map task,
// keys[g] and sums[g] of its groups, become 16 B (Long, Long) records again -- the map
// output Spark writes after ExternalSorter.insertAll with an Aggregator.
__global__ __launch_bounds__(RT) void k_pack_pairs(const int64_t *__restrict__ keys, const int64_t *__restrict__ vals,
                                                   int64_t n, longlong2 *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * RT + threadIdx.x;
    if (i < n) out[i] = make_longlong2(keys[i], vals[i]);
}

hipError_t launch_pack_pairs(const int64_t *keys, const int64_t *vals, int64_t n, void *out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_pairs, dim3((unsigned)((n + RT - 1) / RT)), dim3(RT), 0, st, keys, vals, n,
                       (longlong2 *)out);
    return hipGetLastError();
}

}  // namespace sgx
