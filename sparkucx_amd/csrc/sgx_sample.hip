// RangePartitioner.sketch on the GPU (Spark 3.0.1, spark-core; call site
// shuffle/compat/spark_3_0/UcxShuffleManager.scala:50 builds the dependency's partitioner):
//
//   sketch(rdd, k): per input partition idx, SamplingUtils.reservoirSampleAndCount(iter, k,
//   seed = byteswap32(idx ^ (rdd.id << 16))): the first k keys fill the reservoir; for the
//   l-th key (1-based, l > k) draw r = (long)(rand.nextDouble() * l) from an
//   XORShiftRandom(seed) and, if r < k, reservoir[r] = key.
//
// Sequentially that is one RNG draw per record.  Here every record's draw is computed in
// parallel: XORShiftRandom's step (s ^= s << 21; s ^= s >>> 35; s ^= s << 4) is linear over
// GF(2), so the state after m steps is M^m s0, and a thread jumps to its first draw with the
// precomputed powers M^(2^t) (64 x 64 bit matrices, column form) before stepping through a
// contiguous run of draws.  The reservoir's final content at slot r is the LAST record that
// chose r: an atomicMax of record indices per slot, then one gather of the winners' keys.
#include <hip/hip_runtime.h>

#include "sgx_internal.h"

namespace sgx {

namespace {

constexpr int ST = 256;          // threads per workgroup
constexpr int DRAWS = 1024;      // draws per thread

__device__ __forceinline__ uint64_t xs_step(uint64_t s) {
    s ^= s << 21;
    s ^= s >> 35;
    s ^= s << 4;
    return s;
}

// v -> M v for M in column form (cols[b] = M e_b)
__device__ __forceinline__ uint64_t gf2_apply(const uint64_t *__restrict__ cols, uint64_t v) {
    uint64_t r = 0;
#pragma unroll 8
    for (int b = 0; b < 64; ++b) r ^= cols[b] & (0ull - ((v >> b) & 1ull));
    return r;
}

}  // namespace

// Draw j (0-based) of record i = k + j consumes steps 2j+1 (next(26)) and 2j+2 (next(27)).
// winner[r] = max record index that chose slot r (initialised to -1 by the caller).
__global__ __launch_bounds__(ST) void k_reservoir(int64_t n, int64_t k, uint64_t s0,
                                                  const uint64_t *__restrict__ jump /*[48][64]*/,
                                                  long long *__restrict__ winner) {
    const int64_t t = (int64_t)blockIdx.x * ST + threadIdx.x;
    const int64_t ndraw = n - k;
    const int64_t j0 = t * DRAWS;
    if (j0 >= ndraw) return;
    // state before draw j0 = M^(2 j0) s0
    uint64_t s = s0;
    uint64_t m = (uint64_t)(2 * j0);
    for (int b = 0; m; ++b, m >>= 1)
        if (m & 1ull) s = gf2_apply(jump + (size_t)b * 64, s);
    const int64_t j1 = min(ndraw, j0 + DRAWS);
    for (int64_t j = j0; j < j1; ++j) {
        s = xs_step(s);
        const uint64_t a = s & ((1ull << 26) - 1);  // next(26): low 26 bits (non-negative int)
        s = xs_step(s);
        const uint64_t c = s & ((1ull << 27) - 1);  // next(27)
        const double d = (double)((a << 27) + c) * 0x1.0p-53;  // java.util.Random.nextDouble
        const int64_t l = k + j + 1;                            // 1-based count of this record
        const int64_t r = (int64_t)(d * (double)l);             // Scala .toLong: truncation
        if (r < k) atomicMax(winner + r, (long long)(k + j));
    }
}

// reservoir slot r = key of winner[r] (or of record r when no later record chose it)
__global__ __launch_bounds__(ST) void k_reservoir_gather(const char *__restrict__ recs, int rb, int key_bytes,
                                                         int64_t k, const long long *__restrict__ winner,
                                                         char *__restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * ST + threadIdx.x;
    if (r >= k) return;
    const long long w = winner[r];
    const int64_t src = w >= 0 ? (int64_t)w : r;
    for (int b = 0; b < key_bytes; ++b) out[r * key_bytes + b] = recs[src * rb + b];
}

// RangePartitioner's re-sampling of an imbalanced partition with fraction > 0.4
// (BernoulliSampler without gap sampling: one nextDouble per item, kept iff <= fraction).
// Draw i of the partition's XORShiftRandom consumes steps 2i+1 and 2i+2; flags[i] = kept.
__global__ __launch_bounds__(ST) void k_bernoulli(int64_t n, double fraction, uint64_t s0,
                                                  const uint64_t *__restrict__ jump, uint8_t *__restrict__ flags) {
    const int64_t t = (int64_t)blockIdx.x * ST + threadIdx.x;
    const int64_t i0 = t * DRAWS;
    if (i0 >= n) return;
    uint64_t s = s0;
    uint64_t m = (uint64_t)(2 * i0);
    for (int b = 0; m; ++b, m >>= 1)
        if (m & 1ull) s = gf2_apply(jump + (size_t)b * 64, s);
    const int64_t i1 = min(n, i0 + DRAWS);
    for (int64_t i = i0; i < i1; ++i) {
        s = xs_step(s);
        const uint64_t a = s & ((1ull << 26) - 1);
        s = xs_step(s);
        const uint64_t c = s & ((1ull << 27) - 1);
        const double d = (double)((a << 27) + c) * 0x1.0p-53;
        flags[i] = d <= fraction ? 1 : 0;
    }
}

// keys of the records at idx[0..m) (sorted record indices), key_bytes each, back to back
__global__ __launch_bounds__(ST) void k_gather_keys(const char *__restrict__ recs, int rb, int key_bytes,
                                                    const int64_t *__restrict__ idx, int64_t m,
                                                    char *__restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * ST + threadIdx.x;
    if (j >= m) return;
    const char *src = recs + idx[j] * rb;
    for (int b = 0; b < key_bytes; ++b) out[j * key_bytes + b] = src[b];
}

hipError_t launch_bernoulli_flags(int64_t n, double fraction, uint64_t s0, const uint64_t *jump_dev, uint8_t *flags,
                                  hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t nt = (n + DRAWS - 1) / DRAWS;
    hipLaunchKernelGGL(k_bernoulli, dim3((unsigned)((nt + ST - 1) / ST)), dim3(ST), 0, st, n, fraction, s0, jump_dev,
                       flags);
    return hipGetLastError();
}

hipError_t launch_gather_keys(const void *recs, int rb, int key_bytes, const int64_t *idx_dev, int64_t m,
                              void *out_keys, hipStream_t st) {
    if (m <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_keys, dim3((unsigned)((m + ST - 1) / ST)), dim3(ST), 0, st, (const char *)recs, rb,
                       key_bytes, idx_dev, m, (char *)out_keys);
    return hipGetLastError();
}

int64_t reservoir_threads(int64_t n, int64_t k) { return n > k ? (n - k + DRAWS - 1) / DRAWS : 0; }

hipError_t launch_reservoir(const void *recs, int64_t n, int rb, int key_bytes, int64_t k, uint64_t s0,
                            const uint64_t *jump_dev, long long *winner, void *out_keys, hipStream_t st) {
    if (k <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(winner, 0xFF, (size_t)k * 8, st);  // -1
    if (e != hipSuccess) return e;
    const int64_t nt = reservoir_threads(n, k);
    if (nt > 0)
        hipLaunchKernelGGL(k_reservoir, dim3((unsigned)((nt + ST - 1) / ST)), dim3(ST), 0, st, n, k, s0, jump_dev,
                           winner);
    const int64_t kk = n < k ? n : k;
    hipLaunchKernelGGL(k_reservoir_gather, dim3((unsigned)((kk + ST - 1) / ST)), dim3(ST), 0, st,
                       (const char *)recs, rb, key_bytes, kk, (const long long *)winner, (char *)out_keys);
    return hipGetLastError();
}

}  // namespace sgx
