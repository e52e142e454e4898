// sgx_kernels.hip — gfx950 (CDNA4, wave64) kernels of the map-side shuffle write and the
// reduce-side regroup.  Written for MI355X directly: 64-lane ballots, LDS-privatised
// counters, decoupled look-back across workgroups with agent-scope 8-byte granules.
//
//   K1+K2  k_hist      partition id (bit-exact Spark HashPartitioner / RangePartitioner)
//                       + per-chunk histogram in LDS               -> counts[R][G]
//   K3     k_scan      decoupled-look-back exclusive scan over counts (partition-major)
//                       -> per-(partition, chunk) record offsets + the index offsets
//   K4     k_scatter16 stable scatter of 16 B records, LDS-staged per 8 K-record tile so
//                       every partition run leaves the CU as one contiguous store burst
//          k_scatter_wide  same ranking, direct per-record copy for wide records (100 B)
//   K5     k_copy_items    regroup of received exchange blocks into per-reducer runs
//
// Reference semantics restated (see oracle/ for the CPU restatement used as checker):
//   HashPartitioner.getPartition = Utils.nonNegativeMod(java.lang.Long.hashCode(k), R)
//   RangePartitioner.getPartition: <=128 bounds linear "gt" scan, else JDK binarySearch
//   grouping is stable (ExternalSorter / ShuffleInMemorySorter): input order inside runs.
#include <hip/hip_runtime.h>

#include "../../include/sgx.h"
#include "sgx_internal.h"

namespace sgx {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr size_t LDS_MAX = 160 * 1024;  // per CU (gfx950)

// ------------------------------------------------------------------------------------
// Partition ids
// ------------------------------------------------------------------------------------

// u mod R for every 32-bit u, 2 <= R < 2^31 (Granlund-Montgomery round-up multiplier,
// all 32-bit VALU): q = (t + ((u - t) >> 1)) >> (l - 1), t = mulhi(m, u),
// m = floor(2^32 (2^l - R) / R) + 1, l = ceil(log2 R).  R == 1 is special-cased by callers.
__device__ __forceinline__ uint32_t mod_u32(uint32_t u, const PartParams &pp) {
    const uint32_t t = __umulhi(pp.mg_m, u);
    const uint32_t q = (t + ((u - t) >> 1)) >> pp.mg_s;
    return u - q * pp.R;
}

// nonNegativeMod((int)(k ^ (k >>> 32)), R) with k = khi:klo.
// h (signed) mod R == ((h + 2^31) mod R - 2^31 mod R) mod R, evaluated unsigned.
__device__ __forceinline__ uint32_t hash_pid(uint32_t klo, uint32_t khi, const PartParams &pp) {
    const uint32_t u = (klo ^ khi) ^ 0x80000000u;
    const uint32_t r = mod_u32(u, pp);
    const uint32_t t = r + pp.R - pp.c31;
    const uint32_t v = t >= pp.R ? t - pp.R : t;
    return pp.R == 1 ? 0u : v;
}

// KIND_HASH_POW2 (sgx_internal.h): HashPartitioner with a power-of-two R, where
// nonNegativeMod(h, R) == h & (R - 1) for two's-complement h.

// RangePartitioner.getPartition over bounds `b` (global memory, or an LDS copy).  With the
// bounds' top-bits directory (PartParams::dir, built at registration only where the answer
// is the lower bound: Spark's linear branch, or its binary search over strictly increasing
// bounds) a key searches the few bounds sharing its top RDIR_BITS bits -- ~1 at R = 1024 --
// instead of the JDK loop's ~10 dependent, lane-divergent steps.
template <typename BP, typename DP>
__device__ __forceinline__ uint32_t range_pid_i64(int64_t key, BP b, DP dir, int nb, int ascending) {
    int p = 0;
    if (dir) {
        const uint32_t j = (uint32_t)(((uint64_t)key ^ 0x8000000000000000ull) >> (64 - RDIR_BITS));
        int lo = dir[j], hi = dir[j + 1];
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (b[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        p = lo;
    } else if (nb <= 128) {
        while (p < nb && key > b[p]) ++p;
    } else {  // JDK Arrays.binarySearch0 loop, then insertion point, then clamp
        int low = 0, high = nb - 1;
        bool found = false;
        while (low <= high) {
            const int mid = (int)(((unsigned)low + (unsigned)high) >> 1);
            const int64_t mv = b[mid];
            if (mv < key) low = mid + 1;
            else if (mv > key) high = mid - 1;
            else { p = mid; found = true; break; }
        }
        if (!found) p = low;
        if (p > nb) p = nb;
    }
    return (uint32_t)(ascending ? p : nb - p);
}

__device__ __forceinline__ bool k10_lt(uint64_t ahi, uint32_t alo, uint64_t bhi, uint32_t blo) {
    return ahi < bhi || (ahi == bhi && alo < blo);
}

template <typename BP, typename DP>
__device__ __forceinline__ uint32_t range_pid_k10(uint64_t khi, uint32_t klo, BP b, DP dir, int nb, int ascending) {
    int p = 0;
    if (dir) {
        const uint32_t j = (uint32_t)(khi >> (64 - RDIR_BITS));
        int lo = dir[j], hi = dir[j + 1];
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (k10_lt(b[mid].hi, b[mid].lo, khi, klo)) lo = mid + 1;
            else hi = mid;
        }
        p = lo;
    } else if (nb <= 128) {
        while (p < nb && k10_lt(b[p].hi, b[p].lo, khi, klo)) ++p;
    } else {
        int low = 0, high = nb - 1;
        bool found = false;
        while (low <= high) {
            const int mid = (int)(((unsigned)low + (unsigned)high) >> 1);
            const uint64_t mhi = b[mid].hi;
            const uint32_t mlo = b[mid].lo;
            if (k10_lt(mhi, mlo, khi, klo)) low = mid + 1;
            else if (k10_lt(khi, klo, mhi, mlo)) high = mid - 1;
            else { p = mid; found = true; break; }
        }
        if (!found) p = low;
        if (p > nb) p = nb;
    }
    return (uint32_t)(ascending ? p : nb - p);
}

// Partition id from the first 12 bytes of a record (x, y, z little-endian dwords), range
// bounds read through `bounds` (pp.bounds in global memory, or a copy in LDS).
template <int KIND, typename BI64 = const int64_t *, typename BK10 = const Key10 *>
__device__ __forceinline__ uint32_t pid_of_b(uint32_t x, uint32_t y, uint32_t z, const PartParams &pp,
                                             BI64 bi64, BK10 bk10, const uint16_t *bdir) {
    if constexpr (KIND == SGX_PART_HASH) {
        return hash_pid(x, y, pp);
    } else if constexpr (KIND == KIND_DIGIT) {
        // 8-bit digit of the 96-bit little-endian view {x, y, z} at bit dshift (a multiple of 8)
        const uint32_t sh = pp.dshift;
        const uint32_t w = sh < 32 ? x : (sh < 64 ? y : z);
        return ((w >> (sh & 31u)) & 0xFFu) ^ pp.dflip;
    } else if constexpr (KIND == KIND_HASH_POW2) {
        return (x ^ y) & (pp.R - 1u);
    } else if constexpr (KIND == KIND_HASH_BITS) {
        return ((x ^ y) >> pp.dshift) & (pp.R - 1u);
    } else if constexpr (KIND == KIND_HOT_SPLIT) {
        return bdir[(x ^ y) & ((1u << pp.dshift) - 1u)];
    } else if constexpr (KIND == KIND_KEY_BITS) {
        const uint64_t wnd = pp.dflip ? ((((uint64_t)y << 32) | x) ^ 0x8000000000000000ull)
                                      : (((uint64_t)__builtin_bswap32(x) << 32) | __builtin_bswap32(y));
        return (uint32_t)(wnd >> pp.dshift) & (pp.R - 1u);
    } else if constexpr (KIND == SGX_PART_RANGE_I64) {
        return range_pid_i64((int64_t)(((uint64_t)y << 32) | x), bi64, bdir, pp.nb, pp.ascending);
    } else {
        const uint64_t hi = ((uint64_t)__builtin_bswap32(x) << 32) | __builtin_bswap32(y);
        const uint32_t lo = __builtin_bswap32(z) >> 16;
        return range_pid_k10(hi, lo, bk10, bdir, pp.nb, pp.ascending);
    }
}

template <int KIND, typename BI64 = const int64_t *, typename BK10 = const Key10 *>
__device__ __forceinline__ uint32_t pid_of_b(uint32_t x, uint32_t y, uint32_t z, const PartParams &pp,
                                             BI64 bi64, BK10 bk10) {
    return pid_of_b<KIND>(x, y, z, pp, bi64, bk10, pp.dir);
}

template <int KIND>
__device__ __forceinline__ uint32_t pid_of(uint32_t x, uint32_t y, uint32_t z, const PartParams &pp) {
    return pid_of_b<KIND>(x, y, z, pp, (const int64_t *)pp.bounds, (const Key10 *)pp.bounds);
}

// ------------------------------------------------------------------------------------
// Wave64 primitives
// ------------------------------------------------------------------------------------

// Lanes of `valid` whose partition id equals this lane's (no __match_any on CDNA: one
// ballot per id bit).  Must be reached by every lane of the wave.
__device__ __forceinline__ uint64_t match_peers(uint32_t p, uint64_t valid, uint32_t nbits) {
    uint64_t peers = valid;
    for (uint32_t b = 0; b < nbits; ++b) {
        const bool bit = (p >> b) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
    }
    return peers;
}

__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    return x;
}

// Exclusive scan of in[0..R) into out[0..R) by the whole block; scratch >= waves u32.
// Ends with a barrier.
template <typename E>
__device__ void block_exclusive_scan(const E *in, E *out, uint32_t R, uint32_t *scratch) {
    const uint32_t T = blockDim.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t per = (R + T - 1) / T;
    const uint32_t beg = min(tid * per, R), end = min(beg + per, R);
    uint32_t s = 0;
    for (uint32_t i = beg; i < end; ++i) s += in[i];
    const uint32_t x = wave_inclusive_scan(s, lane);
    if (lane == 63) scratch[w] = x;
    __syncthreads();
    uint32_t run = x - s;
    for (uint32_t v = 0; v < w; ++v) run += scratch[v];
    for (uint32_t i = beg; i < end; ++i) {
        const uint32_t c = in[i];
        out[i] = (E)run;
        run += c;
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------
// K1+K2: partition ids + per-chunk histogram
// ------------------------------------------------------------------------------------
constexpr int HIST_THREADS = 1024;  // 512 -> 1024: 0.730 -> 0.720 ms at C1 (profiles/r01_hist_geometry_ab*.txt)
constexpr int HIST_UNROLL = 8;

// grid = G * HIST_SPLIT: the HIST_SPLIT workgroups of chunk g walk it together, BACKWARD,
// in steps of HIST_SPLIT * T * HIST_UNROLL records (sub-block `sub` takes its T * HIST_UNROLL
// slice of each step), and add their LDS histograms into counts[p][g] (zeroed by the
// launcher's memset).  Backward, so the last bytes this pass reads -- the ones still in
// the 256 MiB Infinity Cache when K4 starts -- are the chunk heads K4 reads first.
constexpr int HIST_SPLIT = 4;

// AGG (sgx_config.hist_mode = SGX_HIST_BALLOT): wave-aggregated counting -- each lane's
// peers (same partition id) from one ballot per id bit, and only the lowest peer adds
// popcount(peers).  Measured against plain LDS atomics on uniform and Zipf(1.1) keys
// (DESIGN.md §4): plain atomics are the default.
template <int KIND, bool REC16, int UNROLL, int SPLIT, bool AGG = false, bool LB = true>
__device__ __forceinline__ void hist_body(const char *__restrict__ in, int64_t n, int rb, int64_t chunk,
                                          const PartParams &pp, uint32_t *__restrict__ counts, int G) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint32_t *hist = (uint32_t *)smem;
    const uint32_t tid = threadIdx.x, T = blockDim.x;
    for (uint32_t p = tid; p < pp.R; p += T) hist[p] = 0;
    // range partitioners: the bounds' binary search runs against an LDS copy (a dependent
    // chain of ~log2(R) loads per record: LDS latency instead of L1/L2)
    // (LB false: bounds too large for LDS, read from global memory)
    char *bl = smem + (((size_t)pp.R * 4 + 15) & ~(size_t)15);
    uint16_t *dl = (uint16_t *)(bl + (((size_t)pp.nb * (KIND == SGX_PART_RANGE_BYTES10 ? sizeof(Key10) : 8) + 15) &
                                      ~(size_t)15));
    if constexpr (LB && KIND == SGX_PART_RANGE_BYTES10) {
        for (int i = (int)tid; i < pp.nb; i += (int)T) ((Key10 *)bl)[i] = ((const Key10 *)pp.bounds)[i];
    } else if constexpr (LB && KIND == SGX_PART_RANGE_I64) {
        for (int i = (int)tid; i < pp.nb; i += (int)T) ((int64_t *)bl)[i] = ((const int64_t *)pp.bounds)[i];
    }
    if constexpr (LB && (KIND == SGX_PART_RANGE_BYTES10 || KIND == SGX_PART_RANGE_I64))
        if (pp.dir)
            for (int i = (int)tid; i < RDIR_N; i += (int)T) dl[i] = pp.dir[i];
    const int64_t *bi64 = LB ? (const int64_t *)bl : (const int64_t *)pp.bounds;
    const Key10 *bk10 = LB ? (const Key10 *)bl : (const Key10 *)pp.bounds;
    const uint16_t *bdir = (LB && pp.dir) ? (const uint16_t *)dl : pp.dir;
    __syncthreads();
    const int g = blockIdx.x / SPLIT, sub = blockIdx.x % SPLIT;
    const int64_t cbeg = (int64_t)g * chunk;
    int64_t cend = min(n, cbeg + chunk);
    if (pp.chunks) {  // a streaming map's chunk: its batch's bytes, indexed from cbeg as usual
        in += pp.chunks[2 * g] - cbeg * (REC16 ? 16 : rb);
        cend = cbeg + pp.chunks[2 * g + 1];
    }
    const int64_t slice = (int64_t)T * UNROLL, step = slice * SPLIT;
    const int64_t nsteps = cend > cbeg ? (cend - cbeg + step - 1) / step : 0;
    for (int64_t st = nsteps - 1; st >= 0; --st) {
        const int64_t base = cbeg + st * step + sub * slice;
        uint32_t x[UNROLL], y[UNROLL], z[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t i = base + (int64_t)u * T + tid;
            x[u] = y[u] = z[u] = 0;
            if (i < cend) {
                if constexpr (REC16) {
                    const uint4 r = ((const uint4 *)in)[i];
                    x[u] = r.x; y[u] = r.y; z[u] = r.z;
                } else {
                    const uint32_t *p = (const uint32_t *)(in + i * rb);
                    x[u] = p[0]; y[u] = p[1]; z[u] = p[2];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t i = base + (int64_t)u * T + tid;
            if constexpr (AGG) {
                const bool live = i < cend;
                const uint32_t p = live ? pid_of_b<KIND>(x[u], y[u], z[u], pp, bi64, bk10, bdir) : 0u;
                const uint64_t peers = match_peers(p, __ballot(live), pp.nbits);
                const uint32_t lane = tid & 63u;
                if (live && (peers & ((1ull << lane) - 1ull)) == 0) atomicAdd(&hist[p], (uint32_t)__popcll(peers));
            } else {
                if (i < cend) atomicAdd(&hist[pid_of_b<KIND>(x[u], y[u], z[u], pp, bi64, bk10, bdir)], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t p = tid; p < pp.R; p += T) {
        const uint32_t c = hist[p];
        if (c) atomicAdd(&counts[(int64_t)p * G + g], c);
    }
}

// FB: the histogram of a padded write's two-pass fallback (a no-op unless the padded K4
// flagged PAD_OVERFLOW in *pp.guard); its own instantiation, so profiles tell it apart
template <int KIND, bool REC16, bool AGG = false, bool LB = true, bool FB = false>
__global__ __launch_bounds__(HIST_THREADS) void k_hist(const char *__restrict__ in, int64_t n, int rb,
                                                       int64_t chunk, PartParams pp,
                                                       uint32_t *__restrict__ counts, int G) {
    if constexpr (FB)
        if (!(*pp.guard & PAD_OVERFLOW)) return;
    hist_body<KIND, REC16, HIST_UNROLL, HIST_SPLIT, AGG, LB>(in, n, rb, chunk, pp, counts, G);
}

hipError_t launch_hist(const void *in, int64_t n, int rb, int64_t chunk, int G,
                       const PartParams &pp, uint32_t *counts, hipStream_t stream, int mode, bool zeroed) {
    const size_t hlds = (((size_t)pp.R * 4 + 15) & ~(size_t)15);
    size_t lds = hlds;
    if (pp.kind == SGX_PART_RANGE_BYTES10) lds += (((size_t)pp.nb * sizeof(Key10) + 15) & ~(size_t)15) + RDIR_BYTES;
    else if (pp.kind == SGX_PART_RANGE_I64) lds += (((size_t)pp.nb * 8 + 15) & ~(size_t)15) + RDIR_BYTES;
    const bool lb = lds <= LDS_MAX;  // else the bounds stay in global memory
    if (!lb) lds = hlds;
    const char *p = (const char *)in;
    if (!zeroed) {
        hipError_t ze = hipMemsetAsync(counts, 0, (size_t)pp.R * G * 4, stream);
        if (ze != hipSuccess) return ze;
    }
    const bool r16 = (rb == 16);
    const dim3 grid(G * HIST_SPLIT), block(HIST_THREADS);
    if (pp.guard) {  // a padded write's fallback: hash / 16 B, or TeraSort's range / 100 B
        if (pp.kind == SGX_PART_RANGE_BYTES10 && !r16) {
            if (lb) {
                if (lds > 65536)
                    (void)hipFuncSetAttribute((const void *)k_hist<SGX_PART_RANGE_BYTES10, false, false, true, true>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                hipLaunchKernelGGL((k_hist<SGX_PART_RANGE_BYTES10, false, false, true, true>), grid, block, lds, stream,
                                   p, n, rb, chunk, pp, counts, G);
            } else {
                hipLaunchKernelGGL((k_hist<SGX_PART_RANGE_BYTES10, false, false, false, true>), grid, block, lds,
                                   stream, p, n, rb, chunk, pp, counts, G);
            }
            return hipGetLastError();
        }
        if (!r16 || pp.kind != SGX_PART_HASH) return hipErrorInvalidValue;
        if ((pp.R & (pp.R - 1)) == 0)
            hipLaunchKernelGGL((k_hist<KIND_HASH_POW2, true, false, true, true>), grid, block, lds, stream, p, n, rb,
                               chunk, pp, counts, G);
        else
            hipLaunchKernelGGL((k_hist<SGX_PART_HASH, true, false, true, true>), grid, block, lds, stream, p, n, rb,
                               chunk, pp, counts, G);
        return hipGetLastError();
    }
    if (mode == HIST_BALLOT && r16 && pp.kind == SGX_PART_HASH) {  // wave-aggregated counting
        if ((pp.R & (pp.R - 1)) == 0)
            hipLaunchKernelGGL((k_hist<KIND_HASH_POW2, true, true>), grid, block, lds, stream, p, n, rb, chunk, pp,
                               counts, G);
        else
            hipLaunchKernelGGL((k_hist<SGX_PART_HASH, true, true>), grid, block, lds, stream, p, n, rb, chunk, pp,
                               counts, G);
        return hipGetLastError();
    }
#define SGX_HIST(K, B) hipLaunchKernelGGL((k_hist<K, B>), grid, block, lds, stream, p, n, rb, chunk, pp, counts, G)
    switch (pp.kind) {
    case SGX_PART_HASH:
        if ((pp.R & (pp.R - 1)) == 0) {
            if (r16) SGX_HIST(KIND_HASH_POW2, true); else SGX_HIST(KIND_HASH_POW2, false);
        } else {
            if (r16) SGX_HIST(SGX_PART_HASH, true); else SGX_HIST(SGX_PART_HASH, false);
        }
        break;
    case KIND_DIGIT: if (r16) SGX_HIST(KIND_DIGIT, true); else SGX_HIST(KIND_DIGIT, false); break;
    case KIND_KEY_BITS: if (r16) SGX_HIST(KIND_KEY_BITS, true); else SGX_HIST(KIND_KEY_BITS, false); break;
    default: break;
    }
#undef SGX_HIST
    // range partitioners: bounds in LDS (LB) when they fit
#define SGX_HIST_R(K, B, L)                                                                                   \
    do {                                                                                                      \
        if (lds > 65536)                                                                                      \
            (void)hipFuncSetAttribute((const void *)k_hist<K, B, false, L>,                                   \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                  \
        hipLaunchKernelGGL((k_hist<K, B, false, L>), grid, block, lds, stream, p, n, rb, chunk, pp, counts, G); \
    } while (0)
    if (pp.kind == SGX_PART_RANGE_I64) {
        if (lb) { if (r16) SGX_HIST_R(SGX_PART_RANGE_I64, true, true); else SGX_HIST_R(SGX_PART_RANGE_I64, false, true); }
        else { if (r16) SGX_HIST_R(SGX_PART_RANGE_I64, true, false); else SGX_HIST_R(SGX_PART_RANGE_I64, false, false); }
    } else if (pp.kind == SGX_PART_RANGE_BYTES10) {
        if (lb) { if (r16) SGX_HIST_R(SGX_PART_RANGE_BYTES10, true, true); else SGX_HIST_R(SGX_PART_RANGE_BYTES10, false, true); }
        else { if (r16) SGX_HIST_R(SGX_PART_RANGE_BYTES10, true, false); else SGX_HIST_R(SGX_PART_RANGE_BYTES10, false, false); }
    }
#undef SGX_HIST_R
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// K3: decoupled look-back exclusive scan over counts[R*G] (partition-major), giving
// offs[p*G+g] = sum_{q<p} total[q] + sum_{g'<g} counts[p][g'].  The status of each tile
// is ONE 8-byte granule {flag:2 | value:62} written by a relaxed agent-scope atomic store
// and polled with relaxed agent-scope atomic loads (the data is the flag: no fences).
// Tiles are taken in dispatch order via an atomic ticket so a tile only ever waits on
// tiles that are already running.  Spins are bounded; a give-up sets ticket_err[1].
// ------------------------------------------------------------------------------------
constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;
constexpr uint64_t ST_AGG = 1ull << 62, ST_PRE = 2ull << 62, ST_VAL = (1ull << 62) - 1;

int64_t scan_tiles(int64_t len) { return (len + SCAN_TILE - 1) / SCAN_TILE; }

template <bool FB = false>  // FB: a padded write's fallback scan, a no-op unless *guard has PAD_OVERFLOW
__global__ __launch_bounds__(SCAN_THREADS) void k_scan(const uint32_t *__restrict__ in,
                                                       uint32_t *__restrict__ out, int64_t len,
                                                       uint64_t *status, uint32_t *ticket, uint32_t *err,
                                                       uint32_t *__restrict__ part_off, int G,
                                                       int R, const uint32_t *guard) {
    if constexpr (FB)
        if (!(*guard & PAD_OVERFLOW)) return;  // the whole workgroup, before its ticket
    __shared__ uint32_t s_tile, s_prefix_lo;
    __shared__ uint32_t s_wsum[SCAN_THREADS / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const int64_t base = (int64_t)tile * SCAN_TILE + (int64_t)tid * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const int64_t i = base + j;
        v[j] = i < len ? in[i] : 0u;
        sum += v[j];
    }
    const uint32_t incl = wave_inclusive_scan(sum, lane);
    if (lane == 63) s_wsum[w] = incl;
    __syncthreads();
    uint32_t texcl = incl - sum;
    uint64_t agg = 0;
    for (uint32_t q = 0; q < SCAN_THREADS / 64; ++q) {
        if (q < w) texcl += s_wsum[q];
        agg += s_wsum[q];
    }
    if (tid == 0) {
        uint64_t excl = 0;
        if (tile == 0) {
            __hip_atomic_store(&status[0], ST_PRE | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(&status[tile], ST_AGG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = (int64_t)tile - 1;
            uint32_t spins = 0;
            while (j >= 0) {
                const uint64_t s = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t flag = s & ~ST_VAL;
                if (flag == 0) {
                    if (++spins > (1u << 26)) { atomicOr(err, 1u); break; }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += s & ST_VAL;
                if (flag == ST_PRE) break;
                --j;
            }
            __hip_atomic_store(&status[tile], ST_PRE | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_prefix_lo = (uint32_t)excl;
    }
    __syncthreads();
    uint32_t run = s_prefix_lo + texcl;  // offsets fit 32 bits (records per map < 2^32)
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const int64_t i = base + j;
        if (i < len) {
            out[i] = run;
            if (i % G == 0) part_off[i / G] = run;
            if (i == len - 1) part_off[R] = run + v[j];
        }
        run += v[j];
    }
}

hipError_t launch_scan(const uint32_t *counts, uint32_t *offs, int64_t len, uint64_t *status,
                       uint32_t *ticket, uint32_t *err, uint32_t *part_off, int G, int R, hipStream_t stream,
                       const uint32_t *guard) {
    const int64_t tiles = scan_tiles(len);
    if (guard)
        hipLaunchKernelGGL(k_scan<true>, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, stream, counts, offs,
                           len, status, ticket, err, part_off, G, R, guard);
    else
        hipLaunchKernelGGL(k_scan<false>, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, stream, counts, offs,
                           len, status, ticket, err, part_off, G, R, guard);
    return hipGetLastError();
}

// One wave per tile of SCAN_TILE counts (64 per lane), no LDS: the ticket and the look-back
// prefix are broadcast by lane shuffles (launch_scan_wave in sgx_internal.h).
// guard (nullable): a padded write's fallback scan, a no-op unless *guard has PAD_OVERFLOW.
__global__ __launch_bounds__(64) void k_scan_wave(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                  int64_t len, uint64_t *status, uint32_t *ticket, uint32_t *err,
                                                  uint32_t *__restrict__ part_off, int G, int R,
                                                  const uint32_t *guard) {
    if (guard && !(*guard & PAD_OVERFLOW)) return;  // the whole wave, before its ticket
    constexpr int ITEMS = SCAN_TILE / 64;
    const uint32_t lane = threadIdx.x;
    uint32_t tile = lane == 0 ? atomicAdd(ticket, 1u) : 0u;
    tile = __shfl(tile, 0, 64);
    const int64_t base = (int64_t)tile * SCAN_TILE + (int64_t)lane * ITEMS;
    // the lane's counts are read twice (the second time from the cache) instead of held: few
    // VGPRs, so the waves fit beside a running K4's
    uint32_t sum = 0;
    for (int j = 0; j < ITEMS; ++j) {
        const int64_t i = base + j;
        sum += i < len ? in[i] : 0u;
    }
    const uint32_t incl = wave_inclusive_scan(sum, lane);
    const uint64_t agg = __shfl(incl, 63, 64);
    uint32_t prefix = 0;
    if (lane == 0) {
        uint64_t excl = 0;
        if (tile == 0) {
            __hip_atomic_store(&status[0], ST_PRE | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(&status[tile], ST_AGG | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = (int64_t)tile - 1;
            uint32_t spins = 0;
            while (j >= 0) {
                const uint64_t s = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t flag = s & ~ST_VAL;
                if (flag == 0) {
                    if (++spins > (1u << 26)) { atomicOr(err, 1u); break; }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += s & ST_VAL;
                if (flag == ST_PRE) break;
                --j;
            }
            __hip_atomic_store(&status[tile], ST_PRE | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        prefix = (uint32_t)excl;
    }
    uint32_t run = __shfl(prefix, 0, 64) + incl - sum;  // offsets fit 32 bits (records per map < 2^32)
    for (int j = 0; j < ITEMS; ++j) {
        const int64_t i = base + j;
        if (i < len) {
            const uint32_t v = in[i];
            out[i] = run;
            if (i % G == 0) part_off[i / G] = run;
            if (i == len - 1) part_off[R] = run + v;
            run += v;
        }
    }
}

hipError_t launch_scan_wave(const uint32_t *counts, uint32_t *offs, int64_t len, uint64_t *status, uint32_t *ticket,
                            uint32_t *err, uint32_t *part_off, int G, int R, hipStream_t stream, const uint32_t *guard) {
    const int64_t tiles = scan_tiles(len);
    hipLaunchKernelGGL(k_scan_wave, dim3((unsigned)tiles), dim3(64), 0, stream, counts, offs, len, status, ticket, err,
                       part_off, G, R, guard);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// K4: stable scatter.
//
// A workgroup owns chunk g = records [g*chunk, (g+1)*chunk) and walks it in tiles of
// TILE = WAVES*ITEMS*64 records; wave w owns the contiguous sub-tile
// [w*ITEMS*64, (w+1)*ITEMS*64) so (wave, item, lane) order == input order.
//   rank:   per-wave private u16 counters wcnt[w][p]; each item is ranked by a ballot
//           match of equal ids (leader lane bumps the counter) -> stable within the wave;
//   merge:  per partition, exclusive prefix of wcnt over waves + tile count tcnt[p];
//   stage:  (16 B records) exclusive scan of tcnt -> lstart; each record lands in LDS at
//           lstart[p] + wcnt[w][p] + rank: the tile is now partition-sorted in LDS;
//   drain:  lanes read LDS linearly and store to cursor[p] + (slot - lstart[p]), so each
//           partition run is written by consecutive lanes (coalesced), and
//           cursor[p] += tcnt[p].  cursor starts at offs[p][g] (K3).
// ------------------------------------------------------------------------------------
constexpr uint32_t SCATTER_OOB = 2u;  // error bit: a scatter destination was out of range
constexpr int WIDE_WAVES = 8;
constexpr int WIDE_THREADS = WIDE_WAVES * 64;

__host__ __device__ constexpr size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }
// Per-wave u16 counter rows are padded to an even length so each row starts on a dword:
// rank_items updates them two-per-dword with ds_add_rtn_u32.
__host__ __device__ constexpr uint32_t rowstride(uint32_t R) { return (R + 1u) & ~1u; }

// LDS of the 16 B scatter: stage[TILE] uint4 | wcnt[WAVES][R] u16 | lstart[R] u16 |
// tcnt[R] u16 | cursor[R] u32.  The block-scan scratch borrows the (idle) stage.
__host__ __device__ size_t scatter16_lds(uint32_t R, int waves, int items, int mbits) {
    const size_t tile = (size_t)waves * items * 64;
    return tile * 16 + al16((size_t)waves * rowstride(R) * 2) + 2 * al16((size_t)R * 2) + al16((size_t)R * 4) +
           (mbits ? (size_t)waves * ((size_t)8 << mbits) : 0);
}

// Largest peer-table width (<= nbits, <= 8) that still fits next to a geometry.
static int table_bits(uint32_t R, int waves, int items, uint32_t nbits, size_t budget) {
    for (int mb = (int)(nbits < 8 ? nbits : 8); mb >= 1; --mb)
        if (scatter16_lds(R, waves, items, mb) <= budget) return mb;
    return 0;
}

struct Geo16 { int waves, items; };
// every instantiated geometry (launch_scatter's switch must list the same set)
static const Geo16 kGeos16[] = {{4, 16}, {8, 16}, {12, 10}, {14, 9}, {16, 7}, {4, 12}, {8, 8}, {4, 8}, {8, 4}, {4, 4}, {4, 2}, {4, 1}};

ScatterGeom scatter_geom16(uint32_t R, int force_waves, int force_items) {
    ScatterGeom best{0, 0, 0, 0, 0};
    long best_score = -1;
    int best_occ = 0;
    for (const Geo16 &g : kGeos16) {
        if (force_waves && force_waves != g.waves) continue;
        if (force_items && force_items != g.items) continue;
        const size_t base = scatter16_lds(R, g.waves, g.items, 0);
        if (base > LDS_MAX) continue;
        const int occ = (int)(LDS_MAX / base);
        const int tile = g.waves * g.items * 64;
        // biggest tile first (longest partition runs, least per-tile O(R) overhead; one
        // chunk per CU keeps a second resident workgroup idle anyway), then occupancy
        const long score = (long)tile;
        if (score > best_score || (score == best_score && occ > best_occ)) {
            uint32_t nb = 0;
            while ((1ull << nb) < R) ++nb;
            const int mb = table_bits(R, g.waves, g.items, nb ? nb : 1, LDS_MAX / occ);
            best = ScatterGeom{g.waves, g.items, tile, scatter16_lds(R, g.waves, g.items, mb), mb};
            best_score = score;
            best_occ = occ;
        }
    }
    return best;
}

static size_t scatter_lds_wide(uint32_t R) {
    return al16((size_t)WIDE_WAVES * rowstride(R) * 2) + (size_t)2 * R * 4 + 64;
}

ScatterGeom scatter_geom_wide(uint32_t R, int /*rb*/) {
    const size_t lds = scatter_lds_wide(R);
    if (lds > LDS_MAX) return ScatterGeom{WIDE_WAVES, 0, 0, 0, 0};
    return ScatterGeom{WIDE_WAVES, 4, WIDE_WAVES * 4 * 64, lds, 0};
}

// Slot -> partition for the drain: the last p with lstart[p] <= s (empty partitions
// before p share p's start, every later partition starts after s).
template <typename T>
__device__ __forceinline__ uint32_t slot_partition(const T *lstart, uint32_t R, uint32_t s) {
    uint32_t lo = 0, hi = R - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if ((uint32_t)lstart[mid] <= s) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Stable within-wave ranking of ITEMS records per lane (input order = item, then lane).
// Equal-id lanes ("peers") are found exactly: with a per-wave LDS mask table of 2^mbits
// u64 entries, every valid lane ORs its lane bit into entry (pid & (2^mbits-1)), reads the
// entry back (candidates = lanes sharing the low mbits bits) and clears it; the remaining
// high id bits are matched with one ballot each (mbits == 0: one ballot per id bit).
// Counters: the wave's u16 counters are packed two per dword; each item's leader (lowest
// peer) does one ds_add_rtn_u32 of popc(peers) into its half, and the old value is
// broadcast to the peers with ds_bpermute.  Every phase is issued for all ITEMS items
// back to back (LDS executes a wave's ops in order, so the OR / read / clear sequence of
// item k+1 is correct without waiting for item k) and waits once: the ranking is
// throughput-bound, not LDS-latency-bound.
template <int ITEMS>
__device__ __forceinline__ void rank_items(const uint32_t (&pid)[ITEMS], const bool (&valid)[ITEMS],
                                           uint32_t (&rank)[ITEMS], uint16_t *mycnt, uint32_t nbits,
                                           uint32_t lane, uint64_t *mytab, uint32_t mbits) {
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint64_t mybit = 1ull << lane;
    uint64_t peers[ITEMS];
    if (mbits) {
        const uint32_t mmask = (1u << mbits) - 1u;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            // relaxed workgroup-scope atomics (not volatile: volatile defeats LDS address-space
            // inference and turns these into flat ops that wait on vmcnt)
            uint64_t *slot = mytab + (pid[k] & mmask);
            if (valid[k]) __hip_atomic_fetch_or(slot, mybit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            peers[k] = valid[k] ? __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0ull;
            if (valid[k]) __hip_atomic_store(slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            for (uint32_t b = mbits; b < nbits; ++b) {
                const bool bit = (pid[k] >> b) & 1u;
                const uint64_t m = __ballot(bit);
                peers[k] &= bit ? m : ~m;
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) peers[k] = match_peers(pid[k], __ballot(valid[k]), nbits);
    }
    uint32_t old[ITEMS];
    uint32_t *words = (uint32_t *)mycnt;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        old[k] = 0;
        if (valid[k] && (peers[k] & lt) == 0) {
            const uint32_t sh = (pid[k] & 1u) << 4;
            old[k] = (atomicAdd(&words[pid[k] >> 1], (uint32_t)__popcll(peers[k]) << sh) >> sh) & 0xFFFFu;
        }
    }
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const int leader = valid[k] ? (int)__ffsll((unsigned long long)peers[k]) - 1 : (int)lane;
        const uint32_t base = (uint32_t)__builtin_amdgcn_ds_bpermute(leader << 2, (int)old[k]);
        rank[k] = base + (uint32_t)__popcll(peers[k] & lt);
    }
}

// LDS-only barrier: waits for this wave's LDS ops, then s_barrier.  Unlike
// __syncthreads() it does not drain outstanding global loads/stores (vmcnt), so the next
// tile's prefetch and this tile's stores stay in flight across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Shared LDS carve-up of k_scatter16.
struct Sc16Lds {
    uint4 *stage;
    uint16_t *wcnt, *lstart, *tcnt;
    uint32_t *cursor, *scratch;
    uint64_t *mtab;  // [WAVES][2^mbits] peer masks (mbits = pp.mbits, may be 0)
    uint32_t mbits;
};

template <int WAVES, int ITEMS>
__device__ __forceinline__ Sc16Lds sc16_lds(char *smem, uint32_t R, uint32_t mbits) {
    constexpr int TILE = WAVES * ITEMS * 64;
    Sc16Lds L;
    L.stage = (uint4 *)smem;
    L.wcnt = (uint16_t *)(smem + (size_t)TILE * 16);
    L.lstart = (uint16_t *)((char *)L.wcnt + al16((size_t)WAVES * rowstride(R) * 2));
    L.tcnt = (uint16_t *)((char *)L.lstart + al16((size_t)R * 2));
    L.cursor = (uint32_t *)((char *)L.tcnt + al16((size_t)R * 2));
    L.mtab = (uint64_t *)((char *)L.cursor + al16((size_t)R * 4));
    L.scratch = (uint32_t *)smem;  // block-scan scratch: stage is idle then
    L.mbits = mbits;
    // the peer table starts (and, item by item, stays) all zero
    for (uint32_t i = threadIdx.x; i < (uint32_t)(WAVES << mbits) && mbits; i += WAVES * 64) L.mtab[i] = 0ull;
    return L;
}

// Rank + merge + scan + stage of one tile whose records/pids are in registers.
// Returns with the tile partition-sorted in L.stage (after a barrier).
template <int WAVES, int ITEMS>
__device__ __forceinline__ void sc16_rank_stage(const Sc16Lds &L, uint32_t R, const uint4 (&rec)[ITEMS],
                                                const uint32_t (&pid)[ITEMS], const bool (&valid)[ITEMS],
                                                uint32_t nbits) {
    constexpr int T = WAVES * 64;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t rank[ITEMS];
    rank_items<ITEMS>(pid, valid, rank, L.wcnt + (size_t)w * rowstride(R), nbits, lane,
                      L.mtab + ((size_t)w << L.mbits), L.mbits);
    lds_barrier();
    for (uint32_t p = tid; p < R; p += T) {
        uint32_t s = 0;
#pragma unroll
        for (int v = 0; v < WAVES; ++v) {
            const uint32_t c = L.wcnt[(size_t)v * rowstride(R) + p];
            L.wcnt[(size_t)v * rowstride(R) + p] = (uint16_t)s;
            s += c;
        }
        L.tcnt[p] = (uint16_t)s;
    }
    lds_barrier();
    block_exclusive_scan(L.tcnt, L.lstart, R, L.scratch);
    const uint16_t *mycnt = L.wcnt + (size_t)w * rowstride(R);
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        if (valid[k]) {
            const uint32_t p = pid[k];
            const uint32_t slot = (uint32_t)L.lstart[p] + mycnt[p] + rank[k];
            if (slot < (uint32_t)(WAVES * ITEMS * 64)) L.stage[slot] = rec[k];
        }
    }
    lds_barrier();
}

// Generic (guarded) tile: used for the partial tail tile and for non-hash partitioners.
template <int KIND, int WAVES, int ITEMS>
__device__ __forceinline__ void sc16_tile_generic(const Sc16Lds &L, const uint4 *__restrict__ in,
                                                  uint4 *__restrict__ out, int64_t tbase, int64_t end,
                                                  const PartParams &pp, int64_t n, uint32_t *err) {
    constexpr int T = WAVES * 64;
    constexpr int TILE = WAVES * ITEMS * 64;
    const uint32_t R = pp.R;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (uint32_t i = tid; i < (uint32_t)(WAVES * rowstride(R) / 2); i += T) ((uint32_t *)L.wcnt)[i] = 0;
    uint4 rec[ITEMS];
    uint32_t pid[ITEMS];
    bool valid[ITEMS];
    const int64_t wbase = tbase + (int64_t)w * ITEMS * 64 + lane;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const int64_t i = wbase + (int64_t)k * 64;
        valid[k] = i < end;
        rec[k] = valid[k] ? in[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) pid[k] = valid[k] ? pid_of<KIND>(rec[k].x, rec[k].y, rec[k].z, pp) : 0u;
    __syncthreads();  // wcnt zeroed
    sc16_rank_stage<WAVES, ITEMS>(L, R, rec, pid, valid, pp.nbits);
    const uint32_t tile_n = (uint32_t)min<int64_t>(TILE, end - tbase);
    for (uint32_t s = tid; s < tile_n; s += T) {
        const uint4 r = L.stage[s];
        uint32_t p;
        if constexpr (KIND == SGX_PART_HASH) p = hash_pid(r.x, r.y, pp);
        else p = slot_partition(L.lstart, R, s);
        const uint32_t d = L.cursor[p] + (s - (uint32_t)L.lstart[p]);
        if ((int64_t)d < n) out[(size_t)d] = r;
        else atomicOr(err, SCATTER_OOB);
    }
    __syncthreads();
    for (uint32_t p = tid; p < R; p += T) L.cursor[p] += L.tcnt[p];
    __syncthreads();
}

// One full tile of the pipelined staged path: rank + stage tile t (records in `rec`),
// prefetch tile tn into `rec` (issued in a pinned order, before the drain stores), drain t.
template <int KIND, int WAVES, int ITEMS>
__device__ __forceinline__ void sc16_full_tile(const Sc16Lds &L, uint4 (&rec)[ITEMS], const uint4 *src,
                                               int64_t tn, uint4 *__restrict__ out, int64_t n,
                                               const PartParams &pp, uint32_t &bad) {
    constexpr int T = WAVES * 64;
    constexpr int TILE = WAVES * ITEMS * 64;
    const uint32_t R = pp.R;
    const uint32_t tid = threadIdx.x;
    uint32_t pid[ITEMS];
    bool valid[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        valid[k] = true;
        pid[k] = pid_of<KIND>(rec[k].x, rec[k].y, rec[k].z, pp);
    }
    sc16_rank_stage<WAVES, ITEMS>(L, R, rec, pid, valid, pp.nbits);
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        rec[k] = src[tn * TILE + k * 64];
        asm volatile("" ::: "memory");  // keep the issue order identical in every copy
    }
    constexpr int BATCH = ITEMS % 4 == 0 ? 4 : (ITEMS % 2 == 0 ? 2 : 1);
#pragma unroll
    for (int k0 = 0; k0 < ITEMS; k0 += BATCH) {
        uint4 r[BATCH];
        uint32_t d[BATCH];
#pragma unroll
        for (int j = 0; j < BATCH; ++j) r[j] = L.stage[(k0 + j) * T + tid];
#pragma unroll
        for (int j = 0; j < BATCH; ++j) {
            const uint32_t s = (uint32_t)((k0 + j) * T + tid);
            uint32_t p;
            if constexpr (KIND == SGX_PART_HASH) p = hash_pid(r[j].x, r[j].y, pp);
            else p = slot_partition(L.lstart, R, s);
            d[j] = L.cursor[p] + (s - (uint32_t)L.lstart[p]);
            const bool ok = (int64_t)d[j] < n;
            bad |= ok ? 0u : 1u;
            d[j] = ok ? d[j] : (uint32_t)(n - 1);
        }
#pragma unroll
        for (int j = 0; j < BATCH; ++j) out[(size_t)d[j]] = r[j];
    }
    lds_barrier();
    for (uint32_t p = tid; p < R; p += T) L.cursor[p] += L.tcnt[p];
    for (uint32_t i = tid; i < (uint32_t)(WAVES * rowstride(R) / 2); i += T) ((uint32_t *)L.wcnt)[i] = 0;
    lds_barrier();
}

template <int KIND, int WAVES, int ITEMS>
__global__ __launch_bounds__(WAVES * 64, 2) void k_scatter16(const uint4 *__restrict__ in,
                                                             uint4 *__restrict__ out, int64_t n,
                                                             int64_t chunk, PartParams pp,
                                                             const uint32_t *__restrict__ offs,
                                                             int G, uint32_t *err) {
    constexpr int T = WAVES * 64;
    constexpr int TILE = WAVES * ITEMS * 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t R = pp.R;
    const Sc16Lds L = sc16_lds<WAVES, ITEMS>(smem, R, pp.mbits);
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int g = blockIdx.x;
    const int64_t begin = (int64_t)g * chunk;
    const int64_t end = min(n, begin + chunk);
    for (uint32_t p = tid; p < R; p += T) L.cursor[p] = offs[(int64_t)p * G + g];
    const int64_t nfull = end > begin ? (end - begin) / TILE : 0;
    int64_t tbase = begin;
    if (nfull > 0) {
        // Steady state (full tiles): tile t+1's loads are issued right after tile t is staged
        // in LDS -- before tile t's drain stores -- so the in-order vmcnt wait before ranking
        // t+1 retires exactly those loads and tile t's stores keep draining behind the next
        // tile's compute.  Tile 0 is peeled so both paths into the loop carry the same
        // outstanding (ITEMS loads, ITEMS stores) and hipcc's counted waits stay exact; loads
        // (clamped) and drain stores are branch-free; an out-of-range destination (only if
        // counts were corrupt) is clamped and reported through a register flag.
        const uint4 *src = in + begin + (int64_t)w * ITEMS * 64 + lane;
        uint4 rec[ITEMS];
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) rec[k] = src[k * 64];
        for (uint32_t i = tid; i < (uint32_t)(WAVES * rowstride(R) / 2); i += T) ((uint32_t *)L.wcnt)[i] = 0;
        __syncthreads();
        uint32_t bad = 0;
        sc16_full_tile<KIND, WAVES, ITEMS>(L, rec, src, nfull > 1 ? 1 : 0, out, n, pp, bad);
        for (int64_t t = 1; t < nfull; ++t)
            sc16_full_tile<KIND, WAVES, ITEMS>(L, rec, src, t + 1 < nfull ? t + 1 : t, out, n, pp, bad);
        if (bad) atomicOr(err, SCATTER_OOB);
        tbase = begin + nfull * TILE;
    } else {
        __syncthreads();
    }
    for (; tbase < end; tbase += TILE)
        sc16_tile_generic<KIND, WAVES, ITEMS>(L, in, out, tbase, end, pp, n, err);
}

// ------------------------------------------------------------------------------------
// K4 (default for hash partitioners): staged scatter with lane-ordered atomic ranking.
//
// Ranking is ONE ds_add_rtn_u32 per record into the wave's own packed-u16 counter row:
// the LDS atomic unit resolves the lanes of one instruction that hit the same dword in
// lane order (probed on gfx950: tools/mb_lds_atomic_order.hip, no violation in 3.4e10
// same-address lane pairs), and one wave's LDS ops execute in issue order,
// so the returned old value IS the record's stable rank among the wave's earlier records
// of its partition (item-major, then lane).  The match-based ranker (k_scatter16) remains
// selectable with SGX_RANK=match and is parity-tested the same way.
//
// Per tile (4 barriers):
//   rank      pid + atomic rank per record, counts land in row w
//   B1
//   owners    thread t owns partition pairs [t*PP, t*PP+PP): exclusive sum over the wave
//             rows (packed: both halves at once), block scan of the owned totals, then
//             row[v][p] = lstart[p] + before_v[p], dlt[p] = cursor[p] - lstart[p],
//             cursor[p] += total[p]                         (B2 inside the block scan)
//   B3
//   stage     stage[row[w][p] + rank] = record; the wave then zeroes its own row (only it
//             reads that row after B3, in LDS order), so no barrier guards the next
//             tile's atomics; the next tile's loads are issued here
//   B4
//   drain     slot s (partition-sorted) -> out[dlt[p] + s]: partition runs leave as
//             contiguous bursts
// LDS: stage[TILE] 16 B | rows[W][RS] u16 | cursor[RS] u32 | dlt[RS] u32 | scratch[64] u32
// with RS = R rounded up to 8 (pad partitions have count 0).
// ------------------------------------------------------------------------------------
__host__ __device__ constexpr uint32_t rs8(uint32_t R) { return (R + 7u) & ~7u; }

__host__ __device__ size_t scatter16_ord_lds(uint32_t R, int waves, int items) {
    return (size_t)waves * items * 64 * 16 + (size_t)waves * rs8(R) * 2 + (size_t)rs8(R) * 8 + 64 * 4;
}

template <int KIND, int WAVES, int ITEMS, int PP, bool FULL>
__device__ __forceinline__ void ord_tile(char *smem, u32x4 (&rec)[ITEMS], const bool (&valid)[ITEMS],
                                         uint32_t tile_n, const u32x4 *nsrc, u32x4 *__restrict__ out,
                                         int64_t n, const PartParams &pp, uint32_t &bad) {
    constexpr int T = WAVES * 64;
    constexpr int TILE = WAVES * ITEMS * 64;
    const uint32_t R = pp.R, RS = rs8(R), NP = RS / 2;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u32x4 *stage = (u32x4 *)smem;
    uint16_t *rows = (uint16_t *)(smem + (size_t)TILE * 16);
    uint32_t *cursor = (uint32_t *)(rows + (size_t)WAVES * RS);
    uint32_t *dlt = cursor + RS;
    uint32_t *scratch = dlt + RS;
    uint16_t *myrow = rows + (size_t)w * RS;

    // ---- rank
    uint32_t pid[ITEMS], rank[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) pid[k] = (FULL || valid[k]) ? pid_of<KIND>(rec[k].x, rec[k].y, rec[k].z, pp) : 0u;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        rank[k] = 0;
        if (FULL || valid[k]) {
            const uint32_t sh = (pid[k] & 1u) << 4;
            const uint32_t old = __hip_atomic_fetch_add((uint32_t *)myrow + (pid[k] >> 1), 1u << sh,
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            rank[k] = (old >> sh) & 0xFFFFu;
        }
        asm volatile("" ::: "memory");  // item order of the atomics is the stable order
    }
    lds_barrier();  // B1

    // ---- owners: merge the wave rows, scan, offsets
    uint32_t tot[PP], before[PP][WAVES];
    uint32_t S = 0;
#pragma unroll
    for (int i = 0; i < PP; ++i) {
        const uint32_t j = tid * PP + i;
        uint32_t run = 0;
        if (j < NP) {
#pragma unroll
            for (int v = 0; v < WAVES; ++v) {
                const uint32_t c = ((const uint32_t *)(rows + (size_t)v * RS))[j];
                before[i][v] = run;
                run += c;  // packed: the two u16 halves never carry (<= TILE each)
            }
        }
        tot[i] = run;
        S += (run & 0xFFFFu) + (run >> 16);
    }
    const uint32_t x = wave_inclusive_scan(S, lane);
    if (lane == 63) scratch[w] = x;
    lds_barrier();  // B2
    uint32_t base = x - S;
    for (uint32_t v = 0; v < w; ++v) base += scratch[v];
#pragma unroll
    for (int i = 0; i < PP; ++i) {
        const uint32_t j = tid * PP + i;
        if (j < NP) {
            const uint32_t lo = base, hi = base + (tot[i] & 0xFFFFu);
            base = hi + (tot[i] >> 16);
            const uint32_t L = lo | (hi << 16);
#pragma unroll
            for (int v = 0; v < WAVES; ++v) ((uint32_t *)(rows + (size_t)v * RS))[j] = before[i][v] + L;
            const uint2 c = ((const uint2 *)cursor)[j];
            ((uint2 *)dlt)[j] = make_uint2(c.x - lo, c.y - hi);
            ((uint2 *)cursor)[j] = make_uint2(c.x + (tot[i] & 0xFFFFu), c.y + (tot[i] >> 16));
        }
    }
    lds_barrier();  // B3

    // ---- stage, zero own row, prefetch the next tile
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        if (FULL || valid[k]) {
            const uint32_t slot = (uint32_t)myrow[pid[k]] + rank[k];
            if (FULL || slot < (uint32_t)TILE) stage[slot] = rec[k];
        }
    }
    for (uint32_t i = lane; i < RS / 8; i += 64) ((u32x4 *)myrow)[i] = u32x4{0, 0, 0, 0};
    if (nsrc) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            rec[k] = nsrc[k * 64];
            asm volatile("" ::: "memory");
        }
    }
    lds_barrier();  // B4

    // ---- drain
    constexpr int BATCH = ITEMS % 4 == 0 ? 4 : (ITEMS % 2 == 0 ? 2 : 1);
#pragma unroll
    for (int k0 = 0; k0 < ITEMS; k0 += BATCH) {
        u32x4 r[BATCH];
        uint32_t d[BATCH];
        bool live[BATCH];
#pragma unroll
        for (int j = 0; j < BATCH; ++j) {
            const uint32_t s = (uint32_t)((k0 + j) * T + tid);
            live[j] = FULL || s < tile_n;
            r[j] = live[j] ? stage[s] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < BATCH; ++j) {
            const uint32_t s = (uint32_t)((k0 + j) * T + tid);
            const uint32_t p = pid_of<KIND>(r[j].x, r[j].y, r[j].z, pp);
            d[j] = dlt[p] + s;
        }
#pragma unroll
        for (int j = 0; j < BATCH; ++j) {
            if (live[j]) {
                const bool ok = (int64_t)d[j] < n;
                bad |= ok ? 0u : 1u;
                out[(size_t)(ok ? d[j] : (uint32_t)(n - 1))] = r[j];
            }
        }
    }
}

template <int KIND, int WAVES, int ITEMS, int PP>
__global__ __launch_bounds__(WAVES * 64, 1) void k_scatter16_ord(const u32x4 *__restrict__ in,
                                                                 u32x4 *__restrict__ out, int64_t n,
                                                                 int64_t chunk, PartParams pp,
                                                                 const uint32_t *__restrict__ offs,
                                                                 int G, uint32_t *err) {
    // the two-pass fallback of a padded split write (R > 1024) runs this single pass, a no-op
    // unless the padded kernels flagged PAD_OVERFLOW
    if (pp.guard && !(*pp.guard & PAD_OVERFLOW)) return;
    constexpr int T = WAVES * 64;
    constexpr int TILE = WAVES * ITEMS * 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t R = pp.R, RS = rs8(R);
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t *rows32 = (uint32_t *)(smem + (size_t)TILE * 16);
    uint32_t *cursor = rows32 + (size_t)WAVES * RS / 2;
    const int g = blockIdx.x;
    const int64_t begin = (int64_t)g * chunk;
    const int64_t end = min(n, begin + chunk);
    for (uint32_t p = tid; p < RS; p += T) cursor[p] = p < R ? offs[(int64_t)p * G + g] : 0u;
    for (uint32_t i = tid; i < (uint32_t)WAVES * RS / 2; i += T) rows32[i] = 0u;
    const int64_t len = end > begin ? end - begin : 0;
    const int64_t nfull = len / TILE;
    const u32x4 *src = in + begin + (int64_t)w * ITEMS * 64 + lane;
    u32x4 rec[ITEMS];
    bool valid[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) valid[k] = true;
    if (nfull > 0) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) rec[k] = src[k * 64];
    }
    __syncthreads();
    uint32_t bad = 0;
    for (int64_t t = 0; t < nfull; ++t)
        ord_tile<KIND, WAVES, ITEMS, PP, true>(smem, rec, valid, (uint32_t)TILE,
                                               t + 1 < nfull ? src + (t + 1) * TILE : nullptr, out, n, pp, bad);
    const int64_t rem = len - nfull * TILE;
    if (rem > 0) {
        const u32x4 *tsrc = src + nfull * TILE;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            valid[k] = (int64_t)w * ITEMS * 64 + k * 64 + lane < rem;
            rec[k] = valid[k] ? tsrc[k * 64] : u32x4{0, 0, 0, 0};
        }
        ord_tile<KIND, WAVES, ITEMS, PP, false>(smem, rec, valid, (uint32_t)rem, nullptr, out, n, pp, bad);
    }
    if (bad) atomicOr(err, SCATTER_OOB);
}

struct OrdGeo { int waves, items, pp; };
// every instantiated lane-ordered geometry (launch_scatter's switch lists the same set)
static const OrdGeo kOrdGeos[] = {{8, 16, 1}, {12, 10, 1}, {16, 7, 1}, {8, 8, 2}, {4, 16, 8}};

ScatterGeom scatter_geom16_ord(uint32_t R, int force_waves, int force_items) {
    ScatterGeom best{0, 0, 0, 0, 0};
    for (const OrdGeo &g : kOrdGeos) {
        if (force_waves && force_waves != g.waves) continue;
        if (force_items && force_items != g.items) continue;
        const uint32_t T = (uint32_t)g.waves * 64;
        if ((rs8(R) / 2 + T - 1) / T > (uint32_t)g.pp) continue;
        const size_t lds = scatter16_ord_lds(R, g.waves, g.items);
        if (lds > LDS_MAX) continue;
        const int tile = g.waves * g.items * 64;
        if (tile > best.tile) best = ScatterGeom{ORD_GEOM_BASE + g.waves, g.items, tile, lds, g.pp};
    }
    return best;
}

// ------------------------------------------------------------------------------------
// K4 (write-combining, default for hash partitioners with R <= 1024): only whole,
// 128 B-aligned output lines leave the CU.
//
// Why: a tile of T records gives every partition a run of ~T/R records (8 at T = 8192,
// R = 1024: ONE line's worth) starting at an arbitrary record offset, so nearly every
// run straddles two 128 B lines, each completed by the NEXT tile's run tens of µs later.
// Those half-written lines leave L2 as partial-line writes that cost a full line of HBM
// time: tools/mb_scatter.hip measures the store pattern alone at 2.98 ms for unaligned
// runs vs 1.99 ms for line-aligned runs (C1, memory only, no ranking) -- and the ranked
// kernels above run at 2.9 ms, i.e. AT the unaligned floor.
//
// How: each (partition, chunk) output stream keeps its incomplete last line ON CHIP.
// Per tile, partition p's records cover output positions [a_p, e_p): the ones it kept from
// the previous tile, [a_p, c_p) (<= 7), then its new ones.  The drain writes positions
// [a_p, LE_p) with LE_p = max(e_p & ~7, a_p): every line it writes is complete (only a
// stream's first line can be partial: its head belongs to the previous stream).  Records at
// [LE_p, e_p) stay in the REGISTERS of the lane that drained them (slot k of the lane's SI
// drain items, with their output position) and are staged again next tile.  The chunk's
// last tile flushes everything; so does a tile whose kept records would not fit next to a
// full tile (sum > DCAP: rare, R <= 585 never), which only costs a few partial lines.  The
// output is byte-identical to every other K4: positions come from the same counts and the
// same stable ranks.
//
// Stage layout (round 3): the records the tile keeps, all streams' [LE_p, e_p) back to
// back, then the ones it writes, all streams' [a_p, LE_p) back to back -- so the drain's
// first ~3.5 R slots need no store instruction and the rest are stores with every lane
// active.
// (Each stream's [a_p, e_p) in one segment left every drain round with both kinds: 16
// store instructions per lane per tile, about half the lanes masked.  C1 K4 1.96 -> 1.85
// ms, bench 1612 -> 1674 GB/s; writes-first measured between the two, and slower at
// R = 4096: profiles/r03_wc_compact_ab.jsonl.)  A record at position x has s0 = x - dw_p:
// it goes to slot s0 if s0 < wend_p (x < LE_p), else to s0 + shift_p in the kept region;
// the drain inverts that per slot.
//
// Tile: NI new records per lane (TNEW = T*NI) + up to DCAP = T*SI - TNEW kept ones.
// LDS: stage[T*SI] 16 B | rows[W][RS] u16 | e[RS] u32 | LE[RS] u32 | {dw, wend | shift << 16}[RS]
// (RS = R rounded up to 8; 160 KB at R = 1024); a stream's kept count is e - LE.  The merge's
// block-scan scratch borrows the stage (free between B1 and B3: every wave has drained the
// previous tile before B1).
// ------------------------------------------------------------------------------------
#ifdef SGX_WC_STAMPS
// Diagnostic build only (tools/build_variant.sh <tag> - -DSGX_WC_STAMPS, tools/wc_stamps.py):
// per-phase s_memtime sums of the tile loop, read through sgx_diag_wc_stamps.  Never in
// libsgx.so; read the SHARES, not the build's run time (the stamps' lgkmcnt(0) forbid overlaps).
__device__ unsigned long long g_wc_stamps[16];
__device__ __forceinline__ uint64_t wc_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
extern "C" int sgx_diag_wc_stamps(unsigned long long *out16, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_wc_stamps), sizeof(g_wc_stamps)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_wc_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#define WC_STAMP(i)                                \
    do {                                           \
        const uint64_t t_ = wc_stamp();            \
        st_acc[i] += t_ - st_last;                 \
        st_last = t_;                              \
    } while (0)
#else
#define WC_STAMP(i) \
    do {            \
    } while (0)
#endif

// Drain groups (of 8 slots) whose stores are held back and issued during the next tile's
// ranking atomics, so the CU's memory queue is not idle through the LDS-only phases.  With
// each stream's records in one stage segment that bought ~1 % (profiles/r03_wc_late_stores_ab.jsonl);
// with the kept-first layout (below) the held group is nearly all stores and holding it
// back costs ~1.5 % instead (C1 K4 1.78 -> 1.75 ms without it, r03_wc_late0_ab.jsonl): off.
#ifndef SGX_WC_LATE
#define SGX_WC_LATE 0
#endif
// Records per written unit of the write-combining K4: 8 (a 128 B L2 line); an A/B probe of
// 64 B units (-DSGX_WC_LINE_RECS=4) asks whether half lines leave HBM as cheaply.
#ifndef SGX_WC_LINE_RECS
#define SGX_WC_LINE_RECS 8
#endif
// nontemporal tile loads in the 16 B write-combining K4 (A/B: -DSGX_WC_NTLOAD=0): each record
// is read once, so its lines need not displace the streams' or the next map's in the caches
// (C1 K4 1.815 -> 1.776 ms, C3 2.461 -> 2.413, 64 batches 1.814 -> 1.787; same box,
// alternating: profiles/r05yz_ntload_ab.jsonl)
#ifndef SGX_WC_NTLOAD
#define SGX_WC_NTLOAD 1
#endif
// chunk <- workgroup mapping of the 16 B write-combining K4 (A/B: -DSGX_WC_XCD_REMAP=1, one
// contiguous run of chunks per XCD)
#ifndef SGX_WC_XCD_REMAP
#define SGX_WC_XCD_REMAP 0
#endif
// nontemporal line stores in the 16 B write-combining K4's drain (A/B: -DSGX_WC_NTSTORE=0)
#ifndef SGX_WC_NTSTORE
#define SGX_WC_NTSTORE 1
#endif
__device__ __forceinline__ void wc_store(const u32x4 &v, u32x4 *p) {
    if constexpr (SGX_WC_NTSTORE) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Sub-bin capacity of a partition from its sampled count: mu = est * chunk / sampled records
// expected per chunk, cap = mu + PAD_SIGMAS * sqrt(a * mu + 16) + 8 (a = 1 + chunk / sampled:
// the chunk's Poisson spread plus the estimate's), rounded up to a whole 128 B line.
__device__ __forceinline__ uint32_t pad_cap_of(uint32_t est, double scale, double a) {
    const double mu = (double)est * scale;
    const double c = mu + PAD_SIGMAS * sqrt(a * mu + 16.0) + 8.0;
    return ((uint32_t)ceil(c) + 7u) & ~7u;
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t x, int d) {
    const uint32_t lo = __shfl_up((uint32_t)x, d, 64), hi = __shfl_up((uint32_t)(x >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}

#ifndef SGX_PAD_CHUNK_MAJOR  // (A/B builds: 0 lays a padded write's sub-bins out partition-major)
#define SGX_PAD_CHUNK_MAJOR 1
#endif
// A padded write's sub-bin layout, computed by each workgroup of its K4 from the sampled counts
// (PartParams.pad_est; the same numbers k_pad_caps computes for the split): stream (p, g) of
// this workgroup's chunk g starts at min(pbase[p] + g cap[p], olim) -> pe[p], ple[p] (p < RS,
// 0 past R).  Workgroup 0 publishes {cap[R], pbase[R]} (pp.pad_layout) for the write's tail
// and flags a layout larger than olim.  RS <= 2 T.  scratch: T / 64 u64 of LDS.  Ends with a
// barrier.
template <int T>
__device__ void pad_layout_starts(const PartParams &pp, uint32_t R, uint32_t RS, int g, int G, uint32_t *pe,
                                  uint32_t *ple, uint64_t *scratch, uint32_t *err) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t cap[2];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t p = 2 * tid + k;
        cap[k] = p < R ? pad_cap_of(pp.pad_est[p], pp.pad_scale, pp.pad_a) : 0u;
        sum += SGX_PAD_CHUNK_MAJOR ? (uint64_t)cap[k] : (uint64_t)cap[k] * (uint64_t)G;
    }
    uint64_t x = sum;  // inclusive scan over the wave, then over the waves' totals
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = shfl_up64(x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) scratch[w] = x;
    __syncthreads();
    uint64_t run = x - sum, total = 0;
#pragma unroll
    for (int v = 0; v < T / 64; ++v) {
        const uint64_t y = scratch[v];
        if (v < (int)w) run += y;
        total += y;
    }
    // chunk-major (SGX_PAD_CHUNK_MAJOR): chunk g's sub-bins are one region, [g total, (g + 1)
    // total), partition p's at run_p inside it -- a workgroup's 1024 streams span ~olim / G
    // records instead of the whole output; partition-major: stream (p, g) at run_p + g cap_p
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t p = 2 * tid + k;
        if (p < RS) {
            const uint64_t at = SGX_PAD_CHUNK_MAJOR ? (uint64_t)g * total + run : run + (uint64_t)g * cap[k];
            const uint32_t c0 = p < R ? (uint32_t)min<uint64_t>(at, (uint64_t)pp.olim) : 0u;
            pe[p] = c0;
            ple[p] = c0;
            if (g == 0 && p < R) {
                pp.pad_layout[p] = cap[k];
                pp.pad_layout[R + p] = (uint32_t)min<uint64_t>(run, (uint64_t)pp.olim);
            }
        }
        run += SGX_PAD_CHUNK_MAJOR ? (uint64_t)cap[k] : (uint64_t)cap[k] * (uint64_t)G;
    }
    const uint64_t whole = SGX_PAD_CHUNK_MAJOR ? total * (uint64_t)G : total;
    if (g == 0 && tid == 0 && whole > (uint64_t)pp.olim) atomicOr(err, PAD_OVERFLOW);
    __syncthreads();
}

__host__ __device__ size_t scatter16_wc_lds(uint32_t R, int waves, int si) {
    return (size_t)waves * 64 * si * 16 + (size_t)waves * rs8(R) * 2 + (size_t)rs8(R) * 16;  // e, LE, {dw, dt}
}

// SEG (level 2 of the two-level split, launch_scatter16_seg): the workgroup's records are
// piece desc[blockIdx.x] = {begin, -, super s, chunk g}, up to the next piece's begin,
// instead of chunk blockIdx.x, and its R streams start at offs[(s * R + p) * G + g].
// MODE (single-pass padded write): 0 the two-pass K4; WC_PADDED the padded K4
// (streams start at their sub-bins, output capacity pp.olim, final counts to pp.pad_cnt
// checked against pp.pad_cap); WC_FALLBACK the fallback's K4, a no-op unless *pp.guard holds
// PAD_OVERFLOW.  Three instantiations, so profiles tell them apart.
constexpr int WC_PADDED = 1, WC_FALLBACK = 2;
template <int KIND, int WAVES, int NI, int SI, bool SEG = false, int MODE = 0>
__global__ __launch_bounds__(WAVES * 64, 1) void k_scatter16_wc(const u32x4 *__restrict__ in,
                                                                u32x4 *__restrict__ out, int64_t n,
                                                                int64_t chunk, PartParams pp,
                                                                const uint32_t *__restrict__ offs,
                                                                int G, uint32_t *err,
                                                                const int64_t *__restrict__ desc = nullptr,
                                                                const uint32_t *__restrict__ ndesc = nullptr,
                                                                u32x4 *__restrict__ out2 = nullptr,
                                                                uint32_t hot_cap = 0,
                                                                const uint32_t *__restrict__ seg_end = nullptr) {
    constexpr int T = WAVES * 64;
    constexpr int TNEW = T * NI;
    constexpr int STAGE = T * SI;
    constexpr uint32_t DCAP = (uint32_t)(STAGE - TNEW);
    static_assert(SI > NI && SI <= 32 && SI % 8 == 0, "kept slots: 32-bit mask, drained 8 at a time");
    // drain slots [LATE_K, SI) store during the next tile's ranking (SGX_WC_LATE groups of 8,
    // never the only group)
    constexpr int LATE_K = SI - 8 * (SGX_WC_LATE < SI / 8 - 1 ? SGX_WC_LATE : SI / 8 - 1);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t R = pp.R, RS = rs8(R), NP = RS / 2;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u32x4 *stage = (u32x4 *)smem;
    uint16_t *rows = (uint16_t *)(smem + (size_t)STAGE * 16);
    // per stream p: pe = end of its records so far, ple = LE (written up to), pdw = {dw, wend |
    // shift << 16}: a record at position x has s0 = x - dw; it is written from slot s0 if
    // s0 < wend (x < LE), else kept in slot s0 + shift (shift: signed 16 bits)
    uint32_t *pe = (uint32_t *)(rows + (size_t)WAVES * RS);
    uint32_t *ple = pe + RS;
    uint2 *pdw = (uint2 *)(ple + RS);
    uint32_t *scratch = (uint32_t *)smem;  // merge only (B1..B3)
    // KIND_HOT_SPLIT: the map's partition -> stream table, staged after pdw
    uint16_t *tbl = (uint16_t *)(pdw + RS);
    // a record's stream: the partition id, or (hybrid split) its partition's stream
    auto pidf = [&](const u32x4 &r) __attribute__((always_inline)) -> uint32_t {
        if constexpr (KIND == KIND_HOT_SPLIT) return tbl[(r.x ^ r.y) & ((1u << pp.dshift) - 1u)];
        else return pid_of<KIND>(r.x, r.y, r.z, pp);
    };
    uint16_t *myrow = rows + (size_t)w * RS;
    uint32_t *myrow32 = (uint32_t *)myrow;
    // output capacity in records: n, or the padded output's (every position stays below it)
    const uint32_t n32 = MODE == WC_PADDED ? pp.olim : (uint32_t)n;  // n < 2^32 (sgx_write_map)
    if constexpr (MODE == WC_FALLBACK)
        if (!(*pp.guard & PAD_OVERFLOW)) return;  // the whole workgroup, before any barrier
    uint32_t bad = 0;

    // FRAGS (level 2 of the padded split): workgroup k G + g reads the level-1 fragments (s,
    // g) of supers s = k pack + f, f < pack, back to back as one sequence -- item i of it is
    // record i + fdl[f] of the scratch for the last f with fpre[f] <= i -- into the R = 64 pack
    // streams of partitions k R + p.  (One 64-stream fragment per workgroup pass left each
    // pass under a third of a tile: 0.71 ms for C3's 2.9 GB.)  Otherwise one chunk / piece.
    // The fragment table lives in lane f of two registers of every wave (fpre: prefix, or ~0
    // past the group; fdl: scratch start - prefix): a 4-step search by lane shuffles per item
    // (16 compares, or the table in scalar registers, spilled)
    constexpr bool FRAGS = SEG && MODE == WC_PADDED;
    uint32_t fpre = 0xFFFFFFFFu, fdl = 0;
    {
    int g = blockIdx.x;
#if SGX_WC_XCD_REMAP
    // workgroup b runs on XCD b % 8: give each XCD a contiguous run of chunks (and, chunk-major,
    // of output regions)
    if constexpr (!SEG)
        if ((G & 7) == 0 && (int)gridDim.x == G) g = (int)(blockIdx.x & 7u) * (G >> 3) + (int)(blockIdx.x >> 3);
#endif
    int64_t begin = (int64_t)g * chunk, end = min(n, begin + chunk), obase = 0;
    if constexpr (FRAGS) {
        const int kg = (int)blockIdx.x / G;
        g = (int)blockIdx.x - kg * G;
        obase = (int64_t)kg * R;
        const bool on = lane < pp.pack;
        const int64_t i1 = ((int64_t)kg * pp.pack + lane) * G + g;
        const uint32_t b = on ? pp.frag_start[i1] : 0u, c = on ? pp.frag_cnt[i1] : 0u;
        const uint32_t incl = wave_inclusive_scan(c, lane);
        if (on) {
            fpre = incl - c;
            fdl = b - fpre;
        }
        begin = 0;
        end = (uint32_t)__shfl((int)incl, 63, 64);
    } else if constexpr (SEG) {
        if (blockIdx.x >= *ndesc) return;  // the whole workgroup, before any barrier
        const int64_t *d = desc + 4 * (int64_t)blockIdx.x;
        begin = d[0];
        // the next piece's begin; the last piece ends with the level-1 records (the cold ones)
        end = blockIdx.x + 1 < *ndesc ? d[4] : (int64_t)*seg_end;
        obase = d[2] * (int64_t)R;
        g = (int)d[3];
    }
    // the chunk's records (a streaming map's chunk: its batch's bytes, chunk table)
    const u32x4 *cin = in + begin;
    if constexpr (!SEG)
        if (pp.chunks) {
            cin = (const u32x4 *)((const char *)in + pp.chunks[2 * g]);
            end = begin + pp.chunks[2 * g + 1];
        }
    const int64_t len = end > begin ? end - begin : 0;
    const int64_t ntiles = (len + TNEW - 1) / TNEW;
    if (MODE == WC_PADDED && !SEG && pp.pad_est) {
        pad_layout_starts<T>(pp, R, RS, g, G, pe, ple, (uint64_t *)smem, err);  // scratch: the stage
    } else {
        for (uint32_t p = tid; p < RS; p += T) {
            const uint32_t c0 = p < R ? offs[(obase + p) * G + g] : 0u;
            pe[p] = c0;
            ple[p] = c0;  // nothing kept
        }
    }
    for (uint32_t i = tid; i < (uint32_t)WAVES * RS / 2; i += T) ((uint32_t *)rows)[i] = 0u;
    if constexpr (KIND == KIND_HOT_SPLIT)
        for (uint32_t i = tid; i < (1u << pp.dshift); i += T) tbl[i] = pp.dir[i];

    const u32x4 *src = cin + (int64_t)w * NI * 64 + lane;
    // FRAGS: the scratch record behind item i of the workgroup's sequence
    auto fidx = [&](uint32_t i) __attribute__((always_inline)) -> uint32_t {
        uint32_t f = 0;  // the last fragment whose prefix is <= i (fragment 0's is 0)
#pragma unroll
        for (uint32_t st = SPLIT_PACK_MAX / 2; st >= 1; st >>= 1)
            f = i >= (uint32_t)__shfl((int)fpre, (int)(f + st), 64) ? f + st : f;
        return i + (uint32_t)__shfl((int)fdl, (int)f, 64);
    };
    u32x4 rec[NI];
    bool valid[NI];
    u32x4 dk[SI];
    uint32_t dpos[SI];
    uint32_t dmask = 0;  // drained records this lane keeps for the next tile
    uint32_t wmask = 0;  // drained records whose store waits for the next tile's rank (SGX_WC_LATE)
#pragma unroll
    for (int k = 0; k < SI; ++k) { dk[k] = u32x4{0, 0, 0, 0}; dpos[k] = 0; }
    if (ntiles > 0) {
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            valid[k] = (int64_t)w * NI * 64 + k * 64 + lane < len;
            const u32x4 *a = FRAGS ? cin + fidx((uint32_t)(w * NI * 64 + k * 64 + lane)) : src + k * 64;
            rec[k] = valid[k] ? (SGX_WC_NTLOAD ? __builtin_nontemporal_load(a) : *a) : u32x4{0, 0, 0, 0};
        }
    }
    __syncthreads();
#ifdef SGX_WC_STAMPS
    uint64_t st_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t st_last = wc_stamp();
#endif
    // ---- drain: the stage's kept region [0, nkeep) into this lane's registers (dk/dpos), the
    //      written region [nkeep, ntot) out as whole lines.
    //      (Draining tile t after tile t+1's ranking, so the wait for t+1's loads does not
    //      also wait for t's stores, measured slightly slower: 1.90-1.97 vs 1.86-1.95 ms.)
    auto drain = [&](const uint32_t ntot, const uint32_t nkeep) __attribute__((always_inline)) {
        dmask = 0;
#pragma unroll
        for (int k0 = 0; k0 < SI; k0 += 8) {
            uint2 dm[8];
            uint32_t pq[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t s = (uint32_t)((k0 + q) * T + tid);
                dk[k0 + q] = stage[s];  // slots past `ntot` hold stale records: never used
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                pq[q] = pidf(dk[k0 + q]);
                dm[q] = pdw[pq[q]];
            }
            WC_STAMP(9);  // drain: stage + dw reads
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t s = (uint32_t)((k0 + q) * T + tid);
                const bool live = s < ntot;
                const bool keep = s < nkeep;
                const uint32_t pos = s + dm[q].x - (keep ? (uint32_t)((int32_t)dm[q].y >> 16) : 0u);
                // every written position is below n by construction; a corrupt count (flagged
                // in the merge) drops the record here instead of storing outside the output
                const bool wr = live && !keep && pos < n32;
                dpos[k0 + q] = pos;
                // nontemporal: the map output is read back much later (exchange / fetch);
                // streaming it past the caches keeps the input's lines in the Infinity
                // Cache for the next histogram (C1: map side 2.65 -> 2.63 ms,
                // profiles/r01_wc_nt_ab.txt).  (Branch-free stores with masked lanes into a
                // junk line, so the next tile could wait for its loads only, measured slower:
                // 2.01-2.04 vs 1.92-1.96 ms.)
                uint64_t ob = (uint64_t)out;
                if constexpr (KIND == KIND_HOT_SPLIT) {
                    const bool o2 = pq[q] >= hot_cap;
                    ob = o2 ? (uint64_t)out2 : ob;
                }
                if (k0 >= LATE_K) wmask |= wr ? 1u << (k0 + q) : 0u;
                else if (wr) wc_store(dk[k0 + q], (u32x4 *)ob + pos);
                dmask |= (live && keep) ? 1u << (k0 + q) : 0u;
            }
            WC_STAMP(10);  // drain: global stores issued
        }
    };
    // the previous drain's held-back stores, issued while this tile's ranking atomics run
    auto late_stores = [&]() __attribute__((always_inline)) {
        if constexpr (LATE_K < SI) {
#pragma unroll
            for (int k = LATE_K; k < SI; ++k) {
                // (a held record's buffer is looked up again: keeping a per-slot mask of it made
                // hipcc move dk[] to scratch memory)
                uint64_t ob = (uint64_t)out;
                if constexpr (KIND == KIND_HOT_SPLIT) ob = pidf(dk[k]) >= hot_cap ? (uint64_t)out2 : ob;
                if ((wmask >> k) & 1u) wc_store(dk[k], (u32x4 *)ob + dpos[k]);
            }
            wmask = 0;
        }
    };
    for (int64_t t = 0; t < ntiles; ++t) {
        const bool last = t == ntiles - 1;
#ifdef SGX_WC_STAMPS
        WC_STAMP(5);  // loop overhead
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the wait hipcc places here anyway
        WC_STAMP(0);  // waiting for this tile's loads (and the last drain's stores)
#endif
        // ---- rank the new records: one LDS atomic each, issued back to back in item order
        //      (a wave's LDS ops execute in issue order; lanes of one op in lane order), one
        //      wait at the end.  An invalid item adds 0 (branch-free issue).
        uint32_t pid[NI], old[NI];
#pragma unroll
        for (int k = 0; k < NI; ++k) pid[k] = valid[k] ? pidf(rec[k]) : 0u;
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const uint32_t inc = valid[k] ? 1u << ((pid[k] & 1u) << 4) : 0u;
            old[k] = __hip_atomic_fetch_add(myrow32 + (pid[k] >> 1), inc, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        late_stores();
        lds_barrier();  // B1
        WC_STAMP(1);  // rank

        // ---- merge: per partition pair (one pair per thread).  Stream p's records this tile
        //      cover positions [a, e): a = LE of the last tile (its kept records, dl = c - a of
        //      them, then the new ones from c on); it writes [a, LE) and keeps [LE, e),
        //      LE = max(e & ~7, a) -- everything when the tile flushes.
        const uint32_t j = tid;
        uint32_t before[WAVES], tot = 0, S = 0, D = 0;
        uint2 c = make_uint2(0, 0), a = make_uint2(0, 0), e = make_uint2(0, 0), kf = make_uint2(0, 0);
        if (j < NP) {
#pragma unroll
            for (int v = 0; v < WAVES; ++v) {
                const uint32_t x = ((const uint32_t *)(rows + (size_t)v * RS))[j];
                before[v] = tot;
                tot += x;  // <= TNEW per half: no carry between halves
            }
            c = ((const uint2 *)pe)[j];
            a = ((const uint2 *)ple)[j];
            e = make_uint2(c.x + (tot & 0xFFFFu), c.y + (tot >> 16));
            kf = make_uint2(e.x - max(e.x & ~(SGX_WC_LINE_RECS - 1u), a.x),
                            e.y - max(e.y & ~(SGX_WC_LINE_RECS - 1u), a.y));  // kept if no flush
            S = (e.x - a.x) + (e.y - a.y);
            D = kf.x + kf.y;
        }
        const uint32_t sd = S | (D << 16);  // S <= STAGE, D <= 7R
        const uint32_t xs = wave_inclusive_scan(sd, lane);
        if (lane == 63) scratch[w] = xs;
        lds_barrier();  // B2
        uint32_t base = (xs - sd) & 0xFFFFu, based = (xs - sd) >> 16, total = 0, dsum = 0;
#pragma unroll
        for (int v = 0; v < WAVES; ++v) {
            const uint32_t y = scratch[v];
            if (v < (int)w) {
                base += y & 0xFFFFu;
                based += y >> 16;
            }
            total += y & 0xFFFFu;
            dsum += y >> 16;
        }
        const bool flush = last || dsum > DCAP;
        const uint32_t nkeep = flush ? 0u : dsum;
        if (j < NP) {
            if (flush) kf = make_uint2(0, 0), based = 0;
            // stream 2j: written slots from wb0, kept slots from kb0; stream 2j+1 follows it
            const uint32_t seg0 = e.x - a.x;
            const uint32_t wb0 = nkeep + base - based, kb0 = based;
            const uint32_t wb1 = wb0 + seg0 - kf.x, kb1 = kb0 + kf.x;
            const uint32_t le0 = e.x - kf.x, le1 = e.y - kf.y;
            const uint32_t dw0 = a.x - wb0, dw1 = a.y - wb1;
            // a kept record's slot: kb + (x - LE) = (x - dw) + shift, shift = kb - wb - (LE - a)
            const uint32_t sh0 = kb0 - wb0 - (le0 - a.x), sh1 = kb1 - wb1 - (le1 - a.y);
            const uint32_t we0 = wb0 + (le0 - a.x), we1 = wb1 + (le1 - a.y);
            // new records start after the kept ones in the written region (their slot is
            // corrected into the kept region in the stage phase when past LE)
            const uint32_t L = (wb0 + (c.x - a.x)) | ((wb1 + (c.y - a.y)) << 16);
#pragma unroll
            for (int v = 0; v < WAVES; ++v) ((uint32_t *)(rows + (size_t)v * RS))[j] = before[v] + L;
            // every position this tile writes is below e <= n by construction; a corrupt count
            // is reported here and its records are dropped at the store (pos < n)
            bad |= (e.x > n32 || e.y > n32) ? 1u : 0u;
            ((uint2 *)pe)[j] = e;
            ((uint2 *)ple)[j] = make_uint2(le0, le1);
            ((u32x4 *)pdw)[j] = u32x4{dw0, we0 | (sh0 << 16), dw1, we1 | (sh1 << 16)};
        }
        lds_barrier();  // B3
        WC_STAMP(2);  // merge

        // ---- stage: a record at position x of stream p goes to s0 = x - dw if x < LE (a
        //      written slot), else to s0 + shift (a kept slot).  LDS reads of a phase are
        //      issued together, one wait each (kept records in groups of 8: registers).
        auto slot_of = [](uint32_t s0, uint32_t ws) __attribute__((always_inline)) -> uint32_t {
            return s0 < (ws & 0xFFFFu) ? s0 : s0 + (uint32_t)((int32_t)ws >> 16);
        };
#pragma unroll
        for (int k0 = 0; k0 < SI; k0 += 8) {
            uint2 kd[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) kd[q] = pdw[pidf(dk[k0 + q])];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if ((dmask >> (k0 + q)) & 1u) stage[slot_of(dpos[k0 + q] - kd[q].x, kd[q].y)] = dk[k0 + q];
        }
        WC_STAMP(7);  // stage: kept-record reads + writes
        {
            uint32_t rb[NI], nw[NI];
#pragma unroll
            for (int k = 0; k < NI; ++k) {
                rb[k] = myrow[pid[k]];
                nw[k] = ((const uint32_t *)pdw)[2 * pid[k] + 1];
            }
            WC_STAMP(6);  // stage: row + slot-map reads
#pragma unroll
            for (int k = 0; k < NI; ++k) {
                const uint32_t sh = (pid[k] & 1u) << 4;
                if (valid[k]) stage[slot_of(rb[k] + ((old[k] >> sh) & 0xFFFFu), nw[k])] = rec[k];
            }
            WC_STAMP(8);  // stage: new writes
        }
        for (uint32_t i = lane; i < RS / 8; i += 64) ((u32x4 *)myrow)[i] = u32x4{0, 0, 0, 0};
        if (!last) {
            const int64_t nb = (t + 1) * TNEW;
            const u32x4 *cb = cin;
#pragma unroll
            for (int k = 0; k < NI; ++k) {
                const int64_t i = nb + (int64_t)w * NI * 64 + k * 64 + lane;
                valid[k] = i < len;
                // branch-free: an invalid item re-reads the chunk head
                const int64_t ia = FRAGS ? (int64_t)fidx(valid[k] ? (uint32_t)i : 0u) : (valid[k] ? i : 0);
                rec[k] = SGX_WC_NTLOAD ? __builtin_nontemporal_load(cb + ia) : cb[ia];
            }
        }
        lds_barrier();  // B4
        WC_STAMP(3);  // stage: zero rows, next loads, B4
        drain(total, nkeep);
    }
    late_stores();
#ifdef SGX_WC_STAMPS
    if (lane == 0) {
        for (int i = 0; i < 12; ++i) atomicAdd(&g_wc_stamps[i], (unsigned long long)st_acc[i]);
        atomicAdd(&g_wc_stamps[14], (unsigned long long)ntiles);
        atomicAdd(&g_wc_stamps[15], 1ull);
    }
#endif
    // padded output: every stream's final count, and whether it stayed inside its sub-bin
    // (pe is final: every thread passed the last tile's B4, or the prologue's barrier)
    if constexpr (MODE == WC_PADDED) {
        if (!SEG && pp.pad_est) {  // the end positions: k_pad_finish makes them counts
            for (uint32_t p = tid; p < R; p += T) pp.pad_cnt[(int64_t)p * G + g] = pe[p];
        } else {
            bool ovf = false;
            for (uint32_t p = tid; p < R; p += T) {
                const int64_t i = (obase + p) * G + g;
                const uint32_t cnt = pe[p] - offs[i];
                pp.pad_cnt[i] = cnt;
                ovf |= cnt > pp.pad_cap[obase + p];
            }
            if (ovf) atomicOr(err, PAD_OVERFLOW);
        }
    }
    }
    if (bad) atomicOr(err, SCATTER_OOB);
}


// geometry: waves = WC_GEOM_BASE + 8, items = NI (new records per lane), mbits = SI (16)
ScatterGeom scatter_geom16_wc(uint32_t R) {
    constexpr int W = 8;
    const uint32_t T = W * 64;
    // (two 6-wave workgroups per CU with 8 drain slots per lane measured slower at small R:
    // R = 200 1.82 -> 2.45 ms, the split's R = 64 levels 3.6 -> 4.0 ms;
    // profiles/r03_wc_two_per_cu_rejected.jsonl)
    constexpr int SI = 16;
    if (rs8(R) / 2 > T) return ScatterGeom{0, 0, 0, 0, 0};
    const size_t lds = scatter16_wc_lds(R, W, SI);
    if (lds > LDS_MAX) return ScatterGeom{0, 0, 0, 0, 0};
    // biggest new-record share whose deferred cap (T*SI - T*NI) still holds 7 per partition
    const int ni = 7u * rs8(R) <= T * (SI - 12) ? 12 : 8;
    return ScatterGeom{WC_GEOM_BASE + W, ni, (int)T * ni, lds, SI};
}

// Wide records (record_bytes multiple of 4, e.g. TeraSort's 100 B): same ranking, each
// lane then copies its record straight to its destination.
template <int KIND, int ITEMS>
__global__ __launch_bounds__(WIDE_THREADS, 1) void k_scatter_wide(const char *__restrict__ in,
                                                                char *__restrict__ out, int64_t n,
                                                                int rb, int64_t chunk,
                                                                PartParams pp,
                                                                const uint32_t *__restrict__ offs,
                                                                int G, uint32_t *err) {
    constexpr int TILE = WIDE_WAVES * ITEMS * 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t R = pp.R;
    uint16_t *wcnt = (uint16_t *)smem;
    uint32_t *cursor = (uint32_t *)(smem + al16((size_t)WIDE_WAVES * rowstride(R) * 2));
    uint32_t *tcnt = cursor + R;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int g = blockIdx.x;
    const int64_t begin = (int64_t)g * chunk;
    const int64_t end = min(n, begin + chunk);
    const int dw = rb >> 2;
    for (uint32_t p = tid; p < R; p += WIDE_THREADS) cursor[p] = offs[(int64_t)p * G + g];

    for (int64_t tbase = begin; tbase < end; tbase += TILE) {
        for (uint32_t i = tid; i < WIDE_WAVES * rowstride(R) / 2; i += WIDE_THREADS) ((uint32_t *)wcnt)[i] = 0;
        uint32_t pid[ITEMS], rank[ITEMS];
        bool valid[ITEMS];
        const int64_t wbase = tbase + (int64_t)w * ITEMS * 64 + lane;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const int64_t i = wbase + (int64_t)k * 64;
            valid[k] = i < end;
            pid[k] = 0;
            if (valid[k]) {
                const uint32_t *p = (const uint32_t *)(in + i * rb);
                pid[k] = pid_of<KIND>(p[0], p[1], p[2], pp);
            }
        }
        __syncthreads();
        rank_items<ITEMS>(pid, valid, rank, wcnt + (size_t)w * rowstride(R), pp.nbits, lane, nullptr, 0u);
        __syncthreads();
        for (uint32_t p = tid; p < R; p += WIDE_THREADS) {
            uint32_t s = 0;
#pragma unroll
            for (int v = 0; v < WIDE_WAVES; ++v) {
                const uint32_t c = wcnt[(size_t)v * rowstride(R) + p];
                wcnt[(size_t)v * rowstride(R) + p] = (uint16_t)s;
                s += c;
            }
            tcnt[p] = s;
        }
        __syncthreads();
        const uint16_t *mycnt = wcnt + (size_t)w * rowstride(R);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            if (valid[k]) {
                const int64_t i = wbase + (int64_t)k * 64;
                const uint32_t p = pid[k];
                const uint64_t dst = (uint64_t)cursor[p] + mycnt[p] + rank[k];
                if ((int64_t)dst >= n) { atomicOr(err, SCATTER_OOB); continue; }
                const uint32_t *s = (const uint32_t *)(in + i * rb);
                uint32_t *d = (uint32_t *)(out + dst * (uint64_t)rb);
                for (int q = 0; q < dw; ++q) d[q] = s[q];
            }
        }
        __syncthreads();
        for (uint32_t p = tid; p < R; p += WIDE_THREADS) cursor[p] += tcnt[p];
    }
}

// ------------------------------------------------------------------------------------
// K4 for wide records (TeraSort 100 B): the tile's bytes are staged in LDS by coalesced
// 16 B loads (issued one tile ahead into registers, so they fly during the whole previous
// tile), the records are ranked exactly like the 16 B kernels (one LDS atomic per record,
// lane-ordered, per-wave rows merged in wave order), a partition-sorted index of the tile
// is built in LDS, and the drain streams the tile out as DWORDS in sorted order: thread t
// moves dword d = t, t + T, ... of the sorted tile, so every partition run leaves the CU
// as consecutive lanes.  Range bounds (RangePartitioner) are copied to LDS once.
// LDS: stage[TR * RB] | bounds[nb] | rows[W][RS] u16 | cur[RS] u32 | dlt[RS] u32 | idx[TR] u32
// ------------------------------------------------------------------------------------
constexpr int WIDE2_TR = 1024;
// A/B probe: nontemporal drain stores (tools/build_variant.sh <tag> - -DSGX_WIDE_NT=1)
#ifndef SGX_WIDE_NT
#define SGX_WIDE_NT 0
#endif
// A/B probe: nontemporal tile loads, so the input stream does not evict the streams' open
// output lines from L2 (-DSGX_WIDE_NTLOAD=1)
#ifndef SGX_WIDE_NTLOAD
#define SGX_WIDE_NTLOAD 0
#endif

__host__ __device__ size_t scatter_wide2_lds(uint32_t R, int rb, int kind, int nb) {
    const size_t bsz = kind == SGX_PART_RANGE_BYTES10 ? sizeof(Key10) : 8;
    return al16((size_t)WIDE2_TR * rb) + (kind == SGX_PART_HASH ? 0 : al16((size_t)nb * bsz) + RDIR_BYTES) +
           (size_t)8 * rs8(R) * 2 + (size_t)rs8(R) * 8 + (size_t)WIDE2_TR * 4 + 64 * 4;
}

// MODE: as k_scatter16_wc's (0, WC_PADDED: streams start at their sub-bins, final counts to
// pp.pad_cnt checked against pp.pad_cap; WC_FALLBACK: a no-op unless *pp.guard has
// PAD_OVERFLOW), so TeraSort maps are written in one pass too.
template <int KIND, int RB, int MODE = 0>
__global__ __launch_bounds__(512, 1) void k_scatter_wide2(const u32x4 *__restrict__ in, uint32_t *__restrict__ out,
                                                          int64_t n, int64_t chunk, PartParams pp,
                                                          const uint32_t *__restrict__ offs, int G,
                                                          uint32_t *err) {
    if constexpr (MODE == WC_FALLBACK)
        if (!(*pp.guard & PAD_OVERFLOW)) return;  // the whole workgroup, before any barrier
    // output capacity in records: n, or the padded output's
    const uint32_t olim = MODE == WC_PADDED ? pp.olim : (uint32_t)n;
    constexpr int T = 512, W = 8, TR = WIDE2_TR, ITEMS = TR / T;  // 2 records per lane
    constexpr int DW = RB / 4;                                     // dwords per record
    constexpr int NCH = TR * RB / 16;                              // 16 B chunks per full tile
    constexpr int LD = (NCH + T - 1) / T;
    constexpr int PC = (RB + 15) / 16;                             // drain pieces per record
    // every piece is 16 B: the last one of a record whose size is not a multiple of 16 ends
    // at the record's end and overlaps the one before it (the same bytes written twice), so
    // the drain's stores are one dwordx4 per lane with every lane active
    auto piece_dw = [](uint32_t pc) -> uint32_t { return pc + 1 < (uint32_t)PC ? 4 * pc : (uint32_t)DW - 4; };
    constexpr int DRB = 7;                                         // pieces per lane per batch
    static_assert(RB % 16 == 4 || RB % 16 == 8 || RB % 16 == 12 || RB % 16 == 0, "RB multiple of 4");
    static_assert((TR * RB) % 16 == 0, "tiles start 16 B aligned");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t R = pp.R, RS = rs8(R), NP = RS / 2;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    char *sp = smem;
    uint32_t *stage = (uint32_t *)sp;
    sp += al16((size_t)TR * RB);
    const Key10 *bk10 = (const Key10 *)sp;
    const int64_t *bi64 = (const int64_t *)sp;
    const uint16_t *bdir = nullptr;
    if constexpr (KIND == SGX_PART_RANGE_BYTES10) {
        for (int i = tid; i < pp.nb; i += T) ((Key10 *)sp)[i] = ((const Key10 *)pp.bounds)[i];
        sp += al16((size_t)pp.nb * sizeof(Key10));
    } else if constexpr (KIND == SGX_PART_RANGE_I64) {
        for (int i = tid; i < pp.nb; i += T) ((int64_t *)sp)[i] = ((const int64_t *)pp.bounds)[i];
        sp += al16((size_t)pp.nb * 8);
    }
    if constexpr (KIND == SGX_PART_RANGE_BYTES10 || KIND == SGX_PART_RANGE_I64) {
        if (pp.dir) {
            for (int i = tid; i < RDIR_N; i += T) ((uint16_t *)sp)[i] = pp.dir[i];
            bdir = (const uint16_t *)sp;
        }
        sp += RDIR_BYTES;
    }
    uint16_t *rows = (uint16_t *)sp;
    uint32_t *cur = (uint32_t *)(rows + (size_t)W * RS);
    uint32_t *dlt = cur + RS;
    uint32_t *idx = dlt + RS;
    uint32_t *scratch = idx + TR;
    uint16_t *myrow = rows + (size_t)w * RS;
    uint32_t *myrow32 = (uint32_t *)myrow;

    const int g = blockIdx.x;
    const int64_t begin = (int64_t)g * chunk;
    const int64_t end = min(n, begin + chunk);
    // the chunk's bytes (a streaming map's chunk: its batch's, chunk table)
    const char *cin = pp.chunks ? (const char *)in + pp.chunks[2 * g] : (const char *)in + begin * RB;
    const int64_t len = pp.chunks ? pp.chunks[2 * g + 1] : end > begin ? end - begin : 0;
    // tile counts in 32 bits, the last tile's size computed once: a 64-bit min() of the
    // per-tile remainder was mis-selected by the compiler (s_cselect on a stale SCC)
    const int ntiles = (int)((len + TR - 1) / TR);
    const int lastn = ntiles > 0 ? (int)(len - (int64_t)(ntiles - 1) * TR) : 0;
    for (uint32_t p = tid; p < RS; p += T) cur[p] = p < R ? offs[(int64_t)p * G + g] : 0u;
    for (uint32_t i = tid; i < (uint32_t)W * RS / 2; i += T) ((uint32_t *)rows)[i] = 0u;

    // tile loads: 16 B chunks of a full tile; the input's last (partial) tile goes dword-wise
    u32x4 ld[LD];
    auto issue = [&](int t) {
        const u32x4 *tb = (const u32x4 *)(cin + (int64_t)t * TR * RB);
        const int nrec = t + 1 < ntiles ? TR : lastn;
        const int nch = nrec == TR ? NCH : 0;  // partial tiles are loaded dword-wise below
#pragma unroll
        for (int i = 0; i < LD; ++i) {
            const int c = i * T + tid;
#if SGX_WIDE_NTLOAD
            ld[i] = c < nch ? __builtin_nontemporal_load(tb + c) : u32x4{0, 0, 0, 0};
#else
            ld[i] = c < nch ? tb[c] : u32x4{0, 0, 0, 0};
#endif
        }
    };
    if (ntiles > 0) issue(0);
    uint32_t bad = 0;
#ifdef SGX_WC_STAMPS
    uint64_t st_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t st_last = wc_stamp();
#endif
    auto store_piece = [&](const u32x4 &v, uint32_t dst, uint32_t pc) {
#if SGX_WIDE_NT
        __builtin_nontemporal_store(v, (u32x4 *)(out + (uint64_t)dst * DW + piece_dw(pc)));
#else
        *(u32x4 *)(out + (uint64_t)dst * DW + piece_dw(pc)) = v;
#endif
    };
    for (int t = 0; t < ntiles; ++t) {
        const int nrec = t + 1 < ntiles ? TR : lastn;
        WC_STAMP(0);  // loop top (previous drain's barrier)
        // ---- land the tile in LDS (the previous drain finished at the last barrier)
        if (nrec == TR) {
#pragma unroll
            for (int i = 0; i < LD; ++i) {
                const int c = i * T + tid;
                if (c < NCH) ((u32x4 *)stage)[c] = ld[i];
            }
        } else {
            const uint32_t *tb = (const uint32_t *)(cin + (int64_t)t * TR * RB);
            for (int d = tid; d < nrec * DW; d += T) stage[d] = tb[d];
        }
        __syncthreads();
        WC_STAMP(1);  // land: wait for the tile's loads, LDS stage writes, barrier
        if (t + 1 < ntiles) issue(t + 1);  // in flight during this whole tile
        WC_STAMP(2);  // issue the next tile's loads
        // ---- partition ids + rank (records w*128 + k*64 + lane: input order = (wave, item, lane))
        uint32_t pid[ITEMS], old[ITEMS];
        bool valid[ITEMS];
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t r = w * (TR / W) + k * 64 + lane;
            valid[k] = r < (uint32_t)nrec;
            const uint32_t *rp = stage + (valid[k] ? r : 0) * DW;
            pid[k] = valid[k] ? pid_of_b<KIND>(rp[0], rp[1], rp[2], pp, bi64, bk10, bdir) : 0u;
        }
        WC_STAMP(3);  // partition ids (range search in LDS)
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t inc = valid[k] ? 1u << ((pid[k] & 1u) << 4) : 0u;
            old[k] = __hip_atomic_fetch_add(myrow32 + (pid[k] >> 1), inc, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        lds_barrier();
        WC_STAMP(4);  // rank atomics + barrier
        // ---- merge: per partition pair, prefix over the wave rows, block scan
        constexpr int PPM = 2;  // pairs per thread (R <= 2048)
        uint32_t before[PPM][W], tot[PPM], S = 0;
#pragma unroll
        for (int i = 0; i < PPM; ++i) {
            const uint32_t j = tid * PPM + i;
            tot[i] = 0;
            if (j < NP) {
#pragma unroll
                for (int v = 0; v < W; ++v) {
                    before[i][v] = tot[i];
                    tot[i] += ((const uint32_t *)(rows + (size_t)v * RS))[j];
                }
            }
            S += (tot[i] & 0xFFFFu) + (tot[i] >> 16);
        }
        const uint32_t xs = wave_inclusive_scan(S, lane);
        if (lane == 63) scratch[w] = xs;
        lds_barrier();
        uint32_t base = xs - S;
        for (uint32_t v = 0; v < w; ++v) base += scratch[v];
#pragma unroll
        for (int i = 0; i < PPM; ++i) {
            const uint32_t j = tid * PPM + i;
            if (j < NP) {
                const uint32_t lo = base, hi = base + (tot[i] & 0xFFFFu);
                base = hi + (tot[i] >> 16);
                const uint32_t L = lo | (hi << 16);
#pragma unroll
                for (int v = 0; v < W; ++v) ((uint32_t *)(rows + (size_t)v * RS))[j] = before[i][v] + L;
                const uint2 c = ((const uint2 *)cur)[j];
                ((uint2 *)dlt)[j] = make_uint2(c.x - lo, c.y - hi);
                ((uint2 *)cur)[j] = make_uint2(c.x + (tot[i] & 0xFFFFu), c.y + (tot[i] >> 16));
                bad |= (c.x + (tot[i] & 0xFFFFu) > olim || c.y + (tot[i] >> 16) > olim) ? 1u : 0u;
            }
        }
        lds_barrier();
        WC_STAMP(5);  // merge (two barriers)
        // ---- sorted index of the tile: idx[slot] = source record | partition << 16
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t sh = (pid[k] & 1u) << 4;
            const uint32_t rb16 = myrow[pid[k]];
            if (valid[k]) idx[rb16 + ((old[k] >> sh) & 0xFFFFu)] = (w * (TR / W) + k * 64 + lane) | (pid[k] << 16);
        }
        for (uint32_t i = lane; i < RS / 8; i += 64) ((u32x4 *)myrow)[i] = u32x4{0, 0, 0, 0};
        lds_barrier();
        WC_STAMP(6);  // sorted index + barrier
        // ---- drain: the sorted tile in 16 B pieces, PC per record (RB = 100: bytes 0-95 in six
        //      and 84-99 in the seventh, piece_dw), consecutive lanes -> consecutive pieces, so a
        //      partition run still
        //      leaves the CU as consecutive lanes, with a quarter of the store instructions and
        //      LDS lookups of a dword stream.  Records are 4 B-aligned in the stage and in the
        //      output: the pieces are read as dwords (ds_read2_b32 pairs) and stored as one
        //      dwordx4 at a 4 B-aligned address (global memory needs only dword alignment).
        const int units = (int)nrec * PC;
        for (int u0 = 0; u0 < units; u0 += DRB * T) {
            u32x4 v[DRB];
            uint32_t dst[DRB], pc[DRB];
            bool live[DRB];
#pragma unroll
            for (int q = 0; q < DRB; ++q) {
                const int u = u0 + q * T + (int)tid;
                live[q] = u < units;
                const uint32_t uu = live[q] ? (uint32_t)u : 0u;
                const uint32_t s = uu / PC;
                pc[q] = uu - s * PC;
                const uint32_t e = idx[s];
                const uint32_t *sp = stage + (e & 0xFFFFu) * DW + piece_dw(pc[q]);
                v[q] = u32x4{sp[0], sp[1], sp[2], sp[3]};
                dst[q] = dlt[e >> 16] + s;
            }
            WC_STAMP(7);  // drain: LDS reads
            // (holding the last batch's pieces back for the next tile's ranking, as the 16 B
            // kernel does, measured slower here: DESIGN.md §6.3)
#pragma unroll
            for (int q = 0; q < DRB; ++q)
                if (live[q] && dst[q] < olim) store_piece(v[q], dst[q], pc[q]);
            WC_STAMP(8);  // drain: global stores
        }
        __syncthreads();  // stage / idx reused by the next tile
        WC_STAMP(9);  // final barrier
    }
#ifdef SGX_WC_STAMPS
    if (lane == 0) {
        for (int i = 0; i < 12; ++i) atomicAdd(&g_wc_stamps[i], (unsigned long long)st_acc[i]);
        atomicAdd(&g_wc_stamps[14], (unsigned long long)ntiles);
        atomicAdd(&g_wc_stamps[15], 1ull);
    }
#endif
    if constexpr (MODE == WC_PADDED) {  // every stream's final count against its sub-bin
        bool ovf = false;
        for (uint32_t p = tid; p < R; p += T) {
            const int64_t i = (int64_t)p * G + g;
            const uint32_t cnt = cur[p] - offs[i];  // cur[p]: written by this thread or before a barrier
            pp.pad_cnt[i] = cnt;
            ovf |= cnt > pp.pad_cap[p];
        }
        if (ovf) atomicOr(err, PAD_OVERFLOW);
    }
    if (bad) atomicOr(err, SCATTER_OOB);
}

ScatterGeom scatter_geom_wide2(uint32_t R, int rb, int kind, int nb) {
    if (rb != 100 || rs8(R) / 2 > 2u * 512u) return ScatterGeom{0, 0, 0, 0, 0};
    const size_t lds = scatter_wide2_lds(R, rb, kind, nb);
    if (lds > LDS_MAX) return ScatterGeom{0, 0, 0, 0, 0};
    return ScatterGeom{WIDE2_GEOM_TAG, 2, WIDE2_TR, lds, 0};
}

// ------------------------------------------------------------------------------------
// Write-combining K4 for 100 B records (TeraSort under its RangePartitioner, R <= 1024;
// DESIGN.md §6.3).  k_scatter_wide2 writes each record as it comes; at R = 1024 a tile holds
// ~1 record per stream, so every record leaves as partial 128 B lines that the L2 merges only
// while the line stays resident (1.18x the record bytes written).  Here every stream keeps
// its incomplete 64 B unit on chip (a carry of <= 60 bytes in LDS, 64 KB at R = 1024) and
// the drain stores whole units only: 4 lanes x 16 B, 64 B-aligned in the output.  A unit's
// bytes come from the stream's carry (its head) and from the tile's records (staged in LDS,
// found through the partition-sorted index).  The stream's first unit (bytes before the
// stream's start belong to its neighbour) and its last (the chunk's end) are written dword by
// dword.  Tiles of 512 records (51 KB staged) leave room for the carries, the ranking rows
// and the bounds (12 B each).
// LDS: stage[TR*100] | bounds (12 B) | rdir | carry[RS][16] u32 (15 data dwords + the stream's
// first record) | rows[W][RS] u16 (ranking; then ps[RS+1] u32 + umap u16 for the drain) |
// cur[RS] u32 | idx[TR] u16 | scratch
// ------------------------------------------------------------------------------------
#ifndef SGX_WIDE_WC
#define SGX_WIDE_WC 1
#endif
#ifndef SGX_WWC_LAND_SYNC
#define SGX_WWC_LAND_SYNC 1
#endif
// the two-pass TeraSort K4 (streams start at the scan's offsets) on the write-combining kernel
// ... and the reduce side's digit / key-window passes
#ifndef SGX_WIDE_WC_REDUCE
#define SGX_WIDE_WC_REDUCE 0
#endif
#ifndef SGX_WIDE_WC_TWOPASS
#define SGX_WIDE_WC_TWOPASS 1
#endif
// XOR-swizzled carry rows (A/B: -DSGX_WWC_SWIZZLE=0)
#ifndef SGX_WWC_SWIZZLE
#define SGX_WWC_SWIZZLE 1
#endif
// nontemporal unit stores in the drain, as the 16 B kernel's (A/B: -DSGX_WWC_NT=0): whole 64 B
// units need no L2 merging, and the output streamed past the caches leaves the next map's
// sample and scan their lines (K4 1.826 -> 1.775 ms, sample 0.038 -> 0.030 ms,
// profiles/r05w_terasort_nt_ab.jsonl)
#ifndef SGX_WWC_NT
#define SGX_WWC_NT 1
#endif
// nontemporal tile loads in the TeraSort K4 (A/B: -DSGX_WWC_NTLOAD=0): K4 1.782 -> 1.775 ms
// (profiles/r05yz_ntload_ab.jsonl)
#ifndef SGX_WWC_NTLOAD
#define SGX_WWC_NTLOAD 1
#endif
// diagnostic probe only (tools/build_variant.sh <tag> - -DSGX_WWC_NOSTORE=1): the drain computes
// its stores but does not issue them -- the kernel's time without its writes
#ifndef SGX_WWC_NOSTORE
#define SGX_WWC_NOSTORE 0
#endif
constexpr int WWC_TR = 512;
// whole units per tile: a stream with k new records closes <= (63 + 100 k) / 64 units, and at
// most WWC_TR streams have records in a tile
constexpr int WWC_UMAX = (WWC_TR * 100 + WWC_TR * 63) / 64 + 1;

// range bounds packed 12 B each in LDS: {hi lo32, hi hi32, lo}
struct Bounds12 {
    const uint32_t *w;
    __device__ __forceinline__ Key10 operator[](int i) const {
        Key10 k;
        k.hi = (uint64_t)w[3 * i] | ((uint64_t)w[3 * i + 1] << 32);
        k.lo = w[3 * i + 2];
        k.pad = 0;
        return k;
    }
};

__host__ __device__ size_t scatter_wide_wc_lds(uint32_t R, int nb);
bool wide_wc_padded_ok(uint32_t R, int nb, int64_t chunk) {
    return SGX_WIDE_WC && R <= 1024 && scatter_wide_wc_lds(R, nb) <= LDS_MAX && chunk % WWC_TR == 0;
}

__host__ __device__ size_t scatter_wide_wc_lds(uint32_t R, int nb) {
    return al16((size_t)WWC_TR * 100) + al16((size_t)nb * 12) + RDIR_BYTES + (size_t)rs8(R) * 64 +
           (size_t)8 * rs8(R) * 2 + al16((size_t)WWC_UMAX * 4) + (size_t)rs8(R) * 4 + al16((size_t)WWC_TR * 2) +
           al16((size_t)(WWC_TR + 1) * 4) + 64 * 4;
}

template <int KIND, int MODE>
__global__ __launch_bounds__(512, 1) void k_scatter_wide_wc(const u32x4 *__restrict__ in, uint32_t *__restrict__ out,
                                                            int64_t n, int64_t chunk, PartParams pp,
                                                            const uint32_t *__restrict__ offs, int G,
                                                            uint32_t *err) {
    constexpr int T = 512, W = 8, TR = WWC_TR, RB = 100, DW = RB / 4;
    constexpr int NCH = TR * RB / 16;  // 16 B chunks per full tile
    constexpr int LD = (NCH + T - 1) / T;
    static_assert((TR * RB) % 16 == 0 && TR == T, "one record per thread, tiles 16 B aligned");
    const uint32_t olim = MODE == WC_PADDED ? pp.olim : (uint32_t)n;
    const uint64_t capB = (uint64_t)olim * RB;  // output bytes
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t R = pp.R, RS = rs8(R), NP = RS / 2;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    char *sp = smem;
    uint32_t *stage = (uint32_t *)sp;
    sp += al16((size_t)TR * RB);
    uint32_t *b12 = (uint32_t *)sp;
    if constexpr (KIND == SGX_PART_RANGE_BYTES10) {
        const Key10 *gb = (const Key10 *)pp.bounds;
        for (int i = tid; i < pp.nb; i += T) {
            const Key10 k = gb[i];
            b12[3 * i] = (uint32_t)k.hi;
            b12[3 * i + 1] = (uint32_t)(k.hi >> 32);
            b12[3 * i + 2] = k.lo;
        }
    } else if constexpr (KIND == SGX_PART_RANGE_I64) {
        for (int i = tid; i < pp.nb; i += T) ((int64_t *)sp)[i] = ((const int64_t *)pp.bounds)[i];
    }
    sp += al16((size_t)pp.nb * 12);
    const uint16_t *bdir = nullptr;
    if (pp.dir) {
        for (int i = tid; i < RDIR_N; i += T) ((uint16_t *)sp)[i] = pp.dir[i];
        bdir = (const uint16_t *)sp;
    }
    sp += RDIR_BYTES;
    uint32_t *carry = (uint32_t *)sp;  // [p][0..14] the open unit's bytes, [p][15] the stream's first record
    sp += (size_t)RS * 64;
    uint16_t *rows = (uint16_t *)sp;
    sp += (size_t)8 * RS * 2;
    uint32_t *desc = (uint32_t *)sp;  // whole units of the tile: p | slot base << 10 | unit of p << 20
    sp += al16((size_t)WWC_UMAX * 4);
    uint32_t *cur = (uint32_t *)sp;
    sp += (size_t)RS * 4;
    uint16_t *idx = (uint16_t *)sp;
    sp += al16((size_t)TR * 2);
    // the tile's active streams (those with records), in stream order: p | first slot << 10 |
    // first unit << 20, then a sentinel {records, units} -- the per-stream work of the tile runs
    // one active stream per thread instead of two streams of every pair per thread
    uint32_t *act = (uint32_t *)sp;
    sp += al16((size_t)(TR + 1) * 4);
    uint32_t *scratch = (uint32_t *)sp;
    uint16_t *myrow = rows + (size_t)w * RS;
    uint32_t *myrow32 = (uint32_t *)myrow;
    const Bounds12 bk{b12};
    const int64_t *bi64 = (const int64_t *)b12;
    // dword i of stream p's carry row, XOR-swizzled by the stream's p / 4: a row is 16 dwords,
    // so unswizzled the rows of streams p, p + 4, ... share their banks -- the owners' carry
    // writes (lanes j -> streams 2j + h) were 32-way bank conflicts (SQ counters,
    // profiles/r05a_terasort_k4_sq_counters.txt: conflicts 56 % of the LDS cycles)
    auto cx = [](uint32_t p, uint32_t i) __attribute__((always_inline)) -> uint32_t {
        return 16u * p + (i ^ (SGX_WWC_SWIZZLE ? (p >> 2) & 15u : 0u));
    };

    const int g = blockIdx.x;
    const int64_t begin = (int64_t)g * chunk;
    const int64_t end = min(n, begin + chunk);
    // the chunk's bytes (a streaming map's chunk: its batch's, chunk table)
    const char *cin = pp.chunks ? (const char *)in + pp.chunks[2 * g] : (const char *)in + begin * RB;
    const int64_t len = pp.chunks ? pp.chunks[2 * g + 1] : end > begin ? end - begin : 0;
    const int ntiles = (int)((len + TR - 1) / TR);
    const int lastn = ntiles > 0 ? (int)(len - (int64_t)(ntiles - 1) * TR) : 0;
    if (MODE == WC_PADDED && pp.pad_est) {  // the sub-bins laid out here (PartParams.pad_est)
        pad_layout_starts<T>(pp, R, RS, g, G, cur, cur, (uint64_t *)scratch, err);
        for (uint32_t p = tid; p < RS; p += T) carry[cx(p, 15)] = cur[p];
    } else {
        for (uint32_t p = tid; p < RS; p += T) {
            const uint32_t c0 = p < R ? offs[(int64_t)p * G + g] : 0u;
            cur[p] = c0;
            carry[cx(p, 15)] = c0;  // the stream's first record: bytes before it are not ours
        }
    }

    // the next tile's loads in registers, two named buffers taking turns (the tile loop is
    // unrolled by two; a second tile in flight made hipcc wait vmcnt(0) at every landing, behind
    // the drain's stores, and bought nothing)
    u32x4 ld0[LD], ld1[LD];
    auto issue = [&](int t, u32x4(&ld)[LD]) __attribute__((always_inline)) {
        const u32x4 *tb = (const u32x4 *)(cin + (int64_t)t * TR * RB);
        const int nch = (t + 1 < ntiles ? TR : lastn) == TR ? NCH : 0;  // partial tiles: dword-wise
#pragma unroll
        for (int i = 0; i < LD; ++i) {
            const int c = i * T + tid;
            ld[i] = c < nch ? (SGX_WWC_NTLOAD ? __builtin_nontemporal_load(tb + c) : tb[c]) : u32x4{0, 0, 0, 0};
        }
    };
    if (ntiles > 0) issue(0, ld0);
    uint32_t bad = 0;
#ifdef SGX_WC_STAMPS
    uint64_t st_acc[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t st_last = wc_stamp();
#endif
    // the thread's active stream of the last tile (act[tid]): its next cursor and carry, taken
    // from the tile's last record of the stream after the drain, stored at the next tile's
    // start (after the barrier that ends every drain's reads of the old ones)
    uint32_t ap = 0, ak = 0, acc = 0, asb = 0, ncur = 0, ncnt = 0, creg[15];
    bool upd = false;
    auto writeback = [&]() __attribute__((always_inline)) {
        if (!upd) return;
#pragma unroll
        for (int i = 0; i < 15; ++i)
            if ((uint32_t)i < ncnt) carry[cx(ap, i)] = creg[i];
        cur[ap] = ncur;
        upd = false;
    };
    auto tile = [&](const int t, u32x4(&ld)[LD], u32x4(&ldn)[LD]) __attribute__((always_inline)) {
        const int nrec = t + 1 < ntiles ? TR : lastn;
        WC_STAMP(0);  // loop top
        writeback();
        WC_STAMP(1);  // owners' carry writeback
        // ---- land the tile; clear the ranking rows
        if (nrec == TR) {
#pragma unroll
            for (int i = 0; i < LD; ++i) {
                const int c = i * T + tid;
                if (c < NCH) ((u32x4 *)stage)[c] = ld[i];
            }
        } else {
            const uint32_t *tb = (const uint32_t *)(cin + (int64_t)t * TR * RB);
            for (int d = tid; d < nrec * DW; d += T) stage[d] = tb[d];
        }
        for (uint32_t i = tid; i < (uint32_t)W * RS / 8; i += T) ((u32x4 *)rows)[i] = u32x4{0, 0, 0, 0};
        // SGX_WWC_LAND_SYNC=0: an LDS-only barrier, so the last drain's global stores stay in
        // flight through this tile's ranking (the tile's loads are waited for where their
        // registers are used)
#if SGX_WWC_LAND_SYNC
        __syncthreads();
#else
        lds_barrier();
#endif
        WC_STAMP(2);  // land the tile (its loads' wait) + barrier
        if (t + 1 < ntiles) issue(t + 1, ldn);
        WC_STAMP(3);  // issue the next tile's loads
        // ---- partition id + rank (record tid: input order = thread order)
        const bool valid = tid < (uint32_t)nrec;
        uint32_t pid = 0, old;
        if (valid) {
            const uint32_t *rp = stage + tid * DW;
            pid = pid_of_b<KIND>(rp[0], rp[1], rp[2], pp, bi64, bk, bdir);
        }
        old = __hip_atomic_fetch_add(myrow32 + (pid >> 1), valid ? 1u << ((pid & 1u) << 4) : 0u, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
        lds_barrier();
        WC_STAMP(4);  // partition ids + ranking atomics + barrier
        // ---- merge: per partition pair j = tid, prefix over the wave rows; block scan of
        //      {records, whole units, active streams} packed 10 | 11 | 11 (<= 512, 1304, 512)
        const uint32_t j = tid;
        uint32_t before[W], tot = 0, val = 0, k[2] = {0, 0}, nu[2] = {0, 0}, cc[2] = {0, 0};
        if (j < NP) {
#pragma unroll
            for (int v = 0; v < W; ++v) {
                before[v] = tot;
                tot += ((const uint32_t *)(rows + (size_t)v * RS))[j];
            }
            k[0] = tot & 0xFFFFu;
            k[1] = tot >> 16;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                cc[h] = cur[2 * j + h];  // the cursors (cur[] becomes the drain's view below)
                nu[h] = ((uint32_t)(((uint64_t)cc[h] * RB) & 63u) + RB * k[h]) >> 6;
            }
            val = (k[0] + k[1]) | ((nu[0] + nu[1]) << 10) | (((k[0] ? 1u : 0u) + (k[1] ? 1u : 0u)) << 21);
        }
        WC_STAMP(5);  // merge: rank rows read
        const uint32_t xs = wave_inclusive_scan(val, lane);
        if (lane == 63) scratch[w] = xs;
        lds_barrier();
        WC_STAMP(10);  // merge: scan + barrier
        uint32_t base = xs - val, total = 0;
#pragma unroll
        for (int v = 0; v < W; ++v) {
            const uint32_t y = scratch[v];
            if (v < (int)w) base += y;
            total += y;
        }
        WC_STAMP(11);  // merge: wave totals read
        const uint32_t sb[2] = {base & 1023u, (base & 1023u) + k[0]};
        const uint32_t ubs[2] = {(base >> 10) & 2047u, ((base >> 10) & 2047u) + nu[0]};
        if (j < NP) {
            const uint32_t L = sb[0] | (sb[1] << 16);
#pragma unroll
            for (int v = 0; v < W; ++v) ((uint32_t *)(rows + (size_t)v * RS))[j] = before[v] + L;
            // the pair's active streams into the list; cur[p] becomes the drain's view cur - sb
            // (the unit's output dword = 25 (view + slot) + w - cneg); the next writeback
            // restores it (a stream without records keeps its cursor)
            uint32_t a = base >> 21;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (k[h] == 0) continue;
                act[a++] = (2 * j + h) | (sb[h] << 10) | (ubs[h] << 20);
                cur[2 * j + h] = cc[h] - sb[h];
            }
        }
        if (tid == 0) act[total >> 21] = ((total & 1023u) << 10) | (((total >> 10) & 2047u) << 20);  // sentinel
        WC_STAMP(12);  // merge: rows + active list written
        lds_barrier();
        WC_STAMP(13);  // merge: barrier
        // ---- partition-sorted index of the tile; the unit words, one active stream per thread:
        //      unit i of stream p starts at dword 16 i - cbD of the stream's new records: below 0
        //      (unit 0 only) its first cneg dwords are the carry's, else record slot sb + r, dword
        //      w.  desc = p | slot << 10 | w << 19 | cneg << 24 | slow << 28, slow: the unit holds
        //      dwords before the stream's first record or past the output's end
        if (valid) idx[myrow[pid] + ((old >> ((pid & 1u) << 4)) & 0xFFFFu)] = (uint16_t)tid;
        const uint32_t nact = total >> 21;
        if (tid < nact) {
            const uint32_t e0 = act[tid], e1 = act[tid + 1];
            ap = e0 & 1023u;
            asb = (e0 >> 10) & 1023u;
            ak = ((e1 >> 10) & 1023u) - asb;
            const uint32_t ub = e0 >> 20, nun = (e1 >> 20) - ub;
            acc = cur[ap] + asb;  // the cursor (cur[] holds the drain's view)
            const uint64_t cD = (uint64_t)acc * DW, u0D = cD & ~(uint64_t)15;
            const uint64_t startD = (uint64_t)carry[cx(ap, 15)] * DW, capD = (uint64_t)olim * DW;
            const uint64_t room = capD > u0D ? (capD - u0D) >> 4 : 0;  // whole units before the end
            const uint32_t ncap = room > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)room;
            const uint32_t cb = (uint32_t)(cD - u0D), w0 = ap | (asb << 10);
            // unit 0: its first cb dwords are the carry's; units 1.. start in the records
            desc[ub] = w0 | (cb << 24) | ((u0D < startD || ncap == 0 ? 1u : 0u) << 28);
            uint32_t r = 0, wv = 16u - cb;
            for (uint32_t i = 1; i < nun; ++i) {
                desc[ub + i] = (w0 + (r << 10)) | (wv << 19) | ((i >= ncap ? 1u : 0u) << 28);
                wv += 16u;
                if (wv >= (uint32_t)DW) wv -= DW, ++r;
            }
        }
        lds_barrier();
        WC_STAMP(6);  // sorted index + unit words + barrier
        // ---- drain: whole 64 B units, 16 B per lane, 4 lanes per unit.  Unit byte x of
        //      stream p: its carry below cb (the open unit's bytes), else byte x - cb of the
        //      stream's records in sorted order
        const uint32_t npieces = ((total >> 10) & 2047u) * 4u;
        // two pieces per step, each phase issued for both before its results are used: the
        // unit word; then the two index slots (and carry dwords); then the 4 data dwords
        const uint32_t coff = (uint32_t)(carry - stage);
        for (uint32_t q0 = tid; q0 < npieces; q0 += 2 * T) {
            uint32_t Dw[2], o4[2], s0[2], s1[2], vw[2][4];
            bool live[2];
            // both words at once (one ds_read2: the second is T / 4 words on, inside the LDS
            // block even past the desc array; a dead piece's word is zeroed)
            Dw[0] = desc[q0 >> 2];
            Dw[1] = desc[(q0 >> 2) + T / 4];
            live[0] = true;
            live[1] = q0 + T < npieces;
            Dw[1] = live[1] ? Dw[1] : 0u;
            uint32_t vx[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint32_t D = Dw[u], p = D & 1023u, slot = (D >> 10) & 511u;
                o4[u] = ((D >> 19) & 31u) + ((q0 + (uint32_t)u * T) & 3u) * 4u;  // + cneg
                s0[u] = idx[slot];
                s1[u] = idx[min(slot + 1u, (uint32_t)TR - 1u)];
                vx[u] = cur[p];
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint32_t D = Dw[u], p = D & 1023u, cneg = (D >> 24) & 15u;
                const uint32_t b0 = s0[u] * DW, b1 = s1[u] * DW - DW;
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    // dword od = o4 + d - cneg of the unit's records: the carry's below 0 (its
                    // dword o4 + d), else record slot (slot + 1 from dword 25; od < 50).  The
                    // choices as masks, so the four reads issue back to back without branches
                    // (the carry rows addressed from the stage's base)
                    const uint32_t e = o4[u] + d;
                    const uint32_t w = e - cneg;
                    const uint32_t m1 = 0u - (uint32_t)(w >= (uint32_t)DW);
                    const uint32_t sa = w + (b0 ^ ((b0 ^ b1) & m1));
                    const uint32_t ca = coff + cx(p, e & 15u);
                    const uint32_t m2 = 0u - (uint32_t)(e < cneg);
                    vw[u][d] = stage[sa ^ ((sa ^ ca) & m2)];
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (!live[u]) continue;
                const uint32_t D = Dw[u], p = D & 1023u, slot = (D >> 10) & 511u, cneg = (D >> 24) & 15u;
                const uint64_t bD = (uint64_t)(vx[u] + slot) * DW + o4[u] - cneg;
                if (SGX_WWC_NOSTORE && bD != ~0ull) {
                } else if (!(D >> 28)) {
#if SGX_WWC_NT
                    __builtin_nontemporal_store(u32x4{vw[u][0], vw[u][1], vw[u][2], vw[u][3]}, (u32x4 *)(out + bD));
#else
                    *(u32x4 *)(out + bD) = u32x4{vw[u][0], vw[u][1], vw[u][2], vw[u][3]};
#endif
                } else {  // the stream's first unit, or the output's end: only the dwords that are ours
                    const uint64_t startD = (uint64_t)carry[cx(p, 15)] * DW, capD = (uint64_t)olim * DW;
#pragma unroll
                    for (int d = 0; d < 4; ++d)
                        if (bD + d >= startD && bD + d < capD) out[bD + d] = vw[u][d];
                }
            }
        }
        WC_STAMP(7);  // drain
        // the thread's active stream: next cursor, and the new open unit = the tail of the
        // tile's last record of the stream (a record is longer than a unit, so it always closes
        // the old one)
        if (tid < nact) {
            const uint64_t cB = (uint64_t)acc * RB, cnB = cB + (uint64_t)RB * ak;
            const uint64_t u1B = cnB & ~(uint64_t)63;
            const uint32_t o = (uint32_t)(u1B - cB) - RB * (ak - 1);  // byte of the last record
            const uint32_t s0 = (uint32_t)idx[asb + ak - 1] * DW + (o >> 2);
            ncnt = (uint32_t)(cnB - u1B) >> 2;
#pragma unroll
            for (int i = 0; i < 15; ++i) creg[i] = stage[min(s0 + i, (uint32_t)(TR * DW - 1))];
            ncur = acc + ak;
            upd = true;
            bad |= ncur > olim ? 1u : 0u;
        }
        WC_STAMP(8);  // owners' next carries
        lds_barrier();
        WC_STAMP(9);  // final barrier
    };
    for (int t = 0; t < ntiles; t += 2) {
        tile(t, ld0, ld1);
        if (t + 1 < ntiles) tile(t + 1, ld1, ld0);
    }
#ifdef SGX_WC_STAMPS
    if (lane == 0) {
        for (int i = 0; i < 14; ++i) atomicAdd(&g_wc_stamps[i], (unsigned long long)st_acc[i]);
        atomicAdd(&g_wc_stamps[14], (unsigned long long)ntiles);
        atomicAdd(&g_wc_stamps[15], 1ull);
    }
#endif
    writeback();
    __syncthreads();
    // ---- the chunk's end: every stream's open unit (its own dwords)
    for (uint32_t p = tid; p < R; p += T) {
        const uint64_t cB = (uint64_t)cur[p] * RB, u0B = cB & ~(uint64_t)63;
        const uint64_t startB = (uint64_t)carry[cx(p, 15)] * RB;
        for (uint64_t b = u0B > startB ? u0B : startB; b < cB; b += 4)
            if (b + 4 <= capB) *(uint32_t *)((char *)out + b) = carry[cx(p, (uint32_t)((b - u0B) >> 2))];
    }
    if constexpr (MODE == WC_PADDED) {
        if (pp.pad_est) {  // the end positions: k_pad_finish makes them counts
            for (uint32_t p = tid; p < R; p += T) pp.pad_cnt[(int64_t)p * G + g] = cur[p];
        } else {
            bool ovf = false;
            for (uint32_t p = tid; p < R; p += T) {
                const int64_t i = (int64_t)p * G + g;
                const uint32_t cnt = cur[p] - offs[i];
                pp.pad_cnt[i] = cnt;
                ovf |= cnt > pp.pad_cap[p];
            }
            if (ovf) atomicOr(err, PAD_OVERFLOW);
        }
    }
    if (bad) atomicOr(err, SCATTER_OOB);
}

// ------------------------------------------------------------------------------------
// Two-level split scatter for R > 1024 (hash partitioner, power-of-two R, 16 B records).
//
// A single pass at R = 4096 (k_scatter16_ord) gives every partition ~1 record per 4 K-record
// tile: its runs start at arbitrary offsets and leave L2 as partial lines -- 7.0 GB written
// per 4.3 GB of records (profiles/r02a_u4096_summary.md) -- and the write-combining kernel
// cannot keep 4096 streams' incomplete lines on chip.  So the split runs two
// write-combining passes of R <= 1024 each, both writing whole lines only:
//   level 1: partition by the top log2(S) bits of the id (S super-partitions) into a scratch
//            buffer, cursors from a scan of the per-chunk super counts -- the hybrid below
//            (KIND_HOT_SPLIT) sends the largest partitions straight to the output instead;
//   level 2: inside every super-partition, partition by the low log2(Q) bits (R = Q = 64),
//            over pieces of whole (super, chunk) blocks: the level-1 output holds super s's
//            records chunk after chunk in input order, so a piece starting at block (s, g)
//            continues every sub-partition stream at exactly the single-level offset
//            offs[(s*Q + q)][g] -- no second histogram, and the result is byte-identical to
//            the single-pass scatter (both stable, same offsets).
// ------------------------------------------------------------------------------------
// Level-2 pieces.  Block i = s*G + g (s-major, the level-1 layout) starts a piece when g == 0
// or when it crosses a multiple of `target` records (k_seg_flags); an exclusive scan of the
// flags (K3) numbers the pieces, and k_seg_desc writes piece k = {begin, -, super, chunk}.
// A piece ends where the next begins (the supers are contiguous), the last one at n: the
// level-2 kernel reads its end from its successor's begin.
// pieces: about `pieces` of them over the level-1 records (*total, on the device: the hybrid's
// cold records), cut every `target` records
__global__ __launch_bounds__(256) void k_seg_flags(const uint32_t *__restrict__ offs1, int S, int G, int64_t pieces,
                                                   const uint32_t *__restrict__ total, uint32_t *__restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)S * G) return;
    const int64_t target = max((int64_t)1, ((int64_t)*total + pieces - 1) / pieces);
    const bool f = i % G == 0 || (int64_t)offs1[i] / target != (int64_t)offs1[i - 1] / target;
    flags[i] = f ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_seg_desc(const uint32_t *__restrict__ offs1, const uint32_t *__restrict__ flags,
                                                  const uint32_t *__restrict__ idx, int S, int G,
                                                  int64_t *__restrict__ desc) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)S * G || !flags[i]) return;
    int64_t *d = desc + 4 * (int64_t)idx[i];
    d[0] = offs1[i];
    d[2] = i / G;
    d[3] = i % G;
}

hipError_t launch_seg_desc(const uint32_t *offs1, int S, int G, const uint32_t *total, int64_t pieces, int64_t *desc,
                           uint32_t *flags, uint32_t *idx, uint64_t *status, uint32_t *ticket, uint32_t *err,
                           uint32_t *npieces, hipStream_t stream) {
    const int64_t nb = (int64_t)S * G;
    const unsigned grid = (unsigned)((nb + 255) / 256);
    hipLaunchKernelGGL(k_seg_flags, dim3(grid), dim3(256), 0, stream, offs1, S, G, pieces, total, flags);
    // one "partition" over all blocks: idx = exclusive prefix of the flags, npieces[1] = total
    hipLaunchKernelGGL(k_scan<false>, dim3((unsigned)scan_tiles(nb)), dim3(SCAN_THREADS), 0, stream, (const uint32_t *)flags,
                       idx, nb, status, ticket, err, npieces, (int)nb, 1, nullptr);
    hipLaunchKernelGGL(k_seg_desc, dim3(grid), dim3(256), 0, stream, offs1, (const uint32_t *)flags,
                       (const uint32_t *)idx, S, G, desc);
    return hipGetLastError();
}

// Hybrid split.  Moving a hot partition's records twice is what made the
// plain split lose on skewed keys, so level 1 writes about the SPLIT_HOT_CAP largest
// partitions straight to the final output through streams of their own (write-combined like
// every stream: a write-combining pass costs about the same at 768 streams as at 64), and
// only the others go through their super-partition to level 2 -- fewer records for level 2
// on any keys.  Any choice of hot set gives the same bytes: a hot stream's cursors are the
// single-pass offsets, and level 2 sees every cold partition's records of a chunk in input
// order.  The cut: a 256-bin log-scale histogram of the counts; every partition of the bins
// above bmin -- the highest bin whose suffix holds >= SPLIT_HOT_CAP partitions -- then bin
// bmin's in id order up to SPLIT_HOT_CAP.
// One workgroup; R <= 4 * 1024.
constexpr int HS_THREADS = 1024, HS_PER = 4;
// counts: per-partition counts (the padded split's sampled estimate), or null to take them from
// the partition offsets
__global__ __launch_bounds__(HS_THREADS) void k_hot_select(const uint32_t *__restrict__ part_off,
                                                           const uint32_t *__restrict__ counts, int R, int Q,
                                                           uint16_t *__restrict__ stream_of,
                                                           int32_t *__restrict__ hot_part) {
    __shared__ uint32_t s_w[HS_THREADS / 64], s_w2[HS_THREADS / 64];
    __shared__ uint32_t s_hist[256];
    __shared__ uint32_t s_bin;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // bins on a log scale, 8 per octave (a bin's counts within 9% of each other): linear bins
    // over [0, max] put every partition but a few under a Zipf head in bin 0, and the cut then
    // took the first partitions by id
    auto hbin = [](uint32_t c) -> uint32_t {
        const uint32_t l = 31u - (uint32_t)__clz(c | 1u);
        const uint32_t m = (l >= 3 ? c >> (l - 3) : c << (3 - l)) & 7u;
        return l * 8u + m;
    };
    uint32_t cnt[HS_PER];
#pragma unroll
    for (int i = 0; i < HS_PER; ++i) {
        const int p = (int)tid * HS_PER + i;
        cnt[i] = p < R ? (counts ? counts[p] : part_off[p + 1] - part_off[p]) : 0u;
    }
    if (tid < 256) s_hist[tid] = 0;
    __syncthreads();
    // one LDS atomic per distinct bin of a wave (the lanes of a bin counted by a ballot): equal
    // counts -- most partitions of a skewed map -- made every lane's atomic hit one address
#pragma unroll
    for (int i = 0; i < HS_PER; ++i) {
        const uint32_t b = hbin(cnt[i]);
        bool todo = cnt[i] != 0;
        while (__ballot(todo)) {
            const uint32_t lead = (uint32_t)__ffsll((unsigned long long)__ballot(todo)) - 1u;
            const uint32_t lb = (uint32_t)__shfl((int)b, (int)lead, 64);
            const bool mine = todo && b == lb;
            const uint32_t k = (uint32_t)__popcll(__ballot(mine));
            if (lane == lead) atomicAdd(&s_hist[lb], k);
            todo = todo && !mine;
        }
    }
    __syncthreads();
    // the lowest bin whose bins above hold >= SPLIT_HOT_CAP partitions: the highest bin b whose
    // suffix sum (bins b..255) reaches the cap, else 0 -- a suffix scan over the 256 bins by the
    // first four waves (a serial walk of the bins by one thread was most of this kernel)
    if (tid == 0) s_bin = 0;
    __syncthreads();
    if (tid < 256) {
        const uint32_t hb = s_hist[255 - tid];  // reversed: an inclusive prefix = a suffix sum
        const uint32_t incl = wave_inclusive_scan(hb, lane);
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        uint32_t suf = incl;
        for (uint32_t v = 0; v < w; ++v) suf += s_w[v];
        if (suf >= (uint32_t)SPLIT_HOT_CAP) atomicMax(&s_bin, 255u - tid);
    } else {
        __syncthreads();
    }
    __syncthreads();
    // hot: every partition of a bin above bmin (fewer than the cap), then bin bmin's in id
    // order up to the cap
    const uint32_t bmin = s_bin;
    uint32_t hot[HS_PER], eq = 0, ca = 0, ce = 0;
#pragma unroll
    for (int i = 0; i < HS_PER; ++i) {
        const uint32_t hb = hbin(cnt[i]);
        hot[i] = (cnt[i] > 0 && hb > bmin) ? 1u : 0u;
        eq |= (cnt[i] > 0 && hb == bmin) ? 1u << i : 0u;
        ca += hot[i];
        ce += (eq >> i) & 1u;
    }
    {
        const uint32_t x = ca | (ce << 16);  // both <= R <= 4096
        const uint32_t xi = wave_inclusive_scan(x, lane);
        if (lane == 63) s_w2[w] = xi;
        __syncthreads();
        uint32_t eb = (xi - x) >> 16, above = 0;
        for (uint32_t v = 0; v < HS_THREADS / 64; ++v) {
            if (v < w) eb += s_w2[v] >> 16;
            above += s_w2[v] & 0xFFFFu;
        }
        const uint32_t room = (uint32_t)SPLIT_HOT_CAP - min(above, (uint32_t)SPLIT_HOT_CAP);
#pragma unroll
        for (int i = 0; i < HS_PER; ++i) {
            if ((eq >> i) & 1u) {
                hot[i] = eb < room ? 1u : 0u;
                ++eb;
            }
        }
    }
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < HS_PER; ++i) c += hot[i];
    const uint32_t incl = wave_inclusive_scan(c, lane);
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    uint32_t base = incl - c, total = 0;
    for (uint32_t v = 0; v < HS_THREADS / 64; ++v) {
        if (v < w) base += s_w[v];
        total += s_w[v];
    }
#pragma unroll
    for (int i = 0; i < HS_PER; ++i) {
        const int p = (int)tid * HS_PER + i;
        if (p >= R) break;
        if (hot[i] && base < (uint32_t)SPLIT_HOT_CAP) {
            stream_of[p] = (uint16_t)base;
            hot_part[base] = p;
        } else {
            stream_of[p] = (uint16_t)(SPLIT_HOT_CAP + p / Q);
        }
        base += hot[i];
    }
    if (tid < (uint32_t)SPLIT_HOT_CAP && tid >= total) hot_part[tid] = -1;
}

hipError_t launch_hot_select(const uint32_t *part_off, int R, int Q, uint16_t *stream_of, int32_t *hot_part,
                             hipStream_t stream, const uint32_t *counts) {
    if (R > HS_THREADS * HS_PER) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_hot_select, dim3(1), dim3(HS_THREADS), 0, stream, part_off, counts, R, Q, stream_of,
                       hot_part);
    return hipGetLastError();
}

// ---- the padded split: level 1 into sub-bins (hot partitions: their final
// sub-bins; cold super-partitions: sub-bins of a scratch buffer), level 2 one (super, chunk)
// fragment at a time into the cold partitions' final sub-bins.
// est1[s] = the cold partitions' sampled counts summed per super-partition.
__global__ __launch_bounds__(64) void k_cold_super_est(const uint32_t *__restrict__ est,
                                                       const uint16_t *__restrict__ stream_of, int S, int Q,
                                                       uint32_t *__restrict__ est1) {
    // one wave per super, its Q partitions across the lanes (a serial walk of them per thread
    // was a chain of dependent loads)
    const int sidx = (int)blockIdx.x;
    const uint32_t lane = threadIdx.x;
    uint32_t acc = 0;
    for (int q = (int)lane; q < Q; q += 64)
        if (stream_of[(int64_t)sidx * Q + q] >= SPLIT_HOT_CAP) acc += est[(int64_t)sidx * Q + q];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d, 64);
    if (lane == 0) est1[sidx] = acc;
}

hipError_t launch_cold_super_est(const uint32_t *est, const uint16_t *stream_of, int S, int Q, uint32_t *est1,
                                 hipStream_t stream) {
    if (S <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_cold_super_est, dim3((unsigned)S), dim3(64), 0, stream, est, stream_of, S, Q, est1);
    return hipGetLastError();
}

// The hot partitions' final counts, from their level-1 streams (level 2 wrote 0 for them).
__global__ __launch_bounds__(256) void k_hot_counts(const uint32_t *__restrict__ cnt1,
                                                    const int32_t *__restrict__ hot_part, int G,
                                                    uint32_t *__restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)SPLIT_HOT_CAP * G) return;
    const int64_t h = i / G, g = i - h * G;
    const int32_t p = hot_part[h];
    if (p >= 0) cnt[(int64_t)p * G + g] = cnt1[i];
}

hipError_t launch_hot_counts(const uint32_t *cnt1, const int32_t *hot_part, int G, uint32_t *cnt, hipStream_t stream) {
    const int64_t n = (int64_t)SPLIT_HOT_CAP * G;
    hipLaunchKernelGGL(k_hot_counts, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, cnt1, hot_part, G, cnt);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_super_counts_cold(const uint32_t *__restrict__ counts,
                                                           const uint16_t *__restrict__ stream_of,
                                                           uint32_t *__restrict__ csum, int S, int Q, int G) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)S * G) return;
    const int64_t sidx = i / G, g = i - sidx * G;
    uint32_t acc = 0;
    for (int q = 0; q < Q; ++q)
        if (stream_of[sidx * Q + q] >= SPLIT_HOT_CAP) acc += counts[(sidx * Q + q) * G + g];
    csum[i] = acc;
}

hipError_t launch_super_counts_cold(const uint32_t *counts, const uint16_t *stream_of, uint32_t *csum, int S, int Q,
                                    int G, hipStream_t stream) {
    const int64_t n = (int64_t)S * G;
    hipLaunchKernelGGL(k_super_counts_cold, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, counts,
                       stream_of, csum, S, Q, G);
    return hipGetLastError();
}

// pcap / cap1 / capS (the padded split only): capS[stream] = its sub-bin capacity, a hot
// stream's partition's (pcap) or a cold super's (cap1)
__global__ __launch_bounds__(256) void k_hot_cursors(const uint32_t *__restrict__ offs,
                                                     const int32_t *__restrict__ hot_part,
                                                     const uint32_t *__restrict__ offs1, uint32_t *__restrict__ cur1,
                                                     int S, int G, const uint32_t *__restrict__ pcap,
                                                     const uint32_t *__restrict__ cap1, uint32_t *__restrict__ capS) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)(SPLIT_HOT_CAP + S) * G) return;
    const int64_t st = i / G, g = i - st * G;
    if (st < SPLIT_HOT_CAP) {
        const int32_t p = hot_part[st];
        cur1[i] = p >= 0 ? offs[(int64_t)p * G + g] : 0u;
        if (capS && g == 0) capS[st] = p >= 0 ? pcap[p] : 0u;
    } else {
        cur1[i] = offs1[(st - SPLIT_HOT_CAP) * G + g];
        if (capS && g == 0) capS[st] = cap1[st - SPLIT_HOT_CAP];
    }
}

hipError_t launch_hot_cursors(const uint32_t *offs, const int32_t *hot_part, const uint32_t *offs1, uint32_t *cur1,
                              int S, int G, hipStream_t stream, const uint32_t *pcap, const uint32_t *cap1,
                              uint32_t *capS) {
    const int64_t n = (int64_t)(SPLIT_HOT_CAP + S) * G;
    hipLaunchKernelGGL(k_hot_cursors, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, offs, hot_part, offs1,
                       cur1, S, G, pcap, cap1, capS);
    return hipGetLastError();
}

hipError_t launch_scatter16_seg(const void *in, void *out, int64_t n, const PartParams &pp, const uint32_t *offs,
                                int G, const int64_t *desc, const uint32_t *ndesc, const uint32_t *seg_end, int grid,
                                const ScatterGeom &geo, uint32_t *err, hipStream_t stream) {
    if ((pp.R & (pp.R - 1)) != 0) return hipErrorInvalidValue;
    if (pp.pad_cnt && (!pp.pad_cap || !pp.olim)) return hipErrorInvalidValue;
    // the padded split's level 2: packed fragments, a workgroup per (super group, chunk)
    if (pp.pad_cnt && (!pp.frag_start || !pp.frag_cnt || pp.pack < 1 || pp.pack > SPLIT_PACK_MAX ||
                       pp.R != 64u * pp.pack || grid % G != 0))
        return hipErrorInvalidValue;
    // the map side's split level 2 (hash bits), or the sorted read's segmented window pass
    // (key bits, never padded)
    const bool key_bits = pp.kind == KIND_KEY_BITS, digit = pp.kind == KIND_DIGIT;
    if ((key_bits || digit) && pp.pad_cnt) return hipErrorInvalidValue;
#define SGX_WCS_K(K, W, NI, SI, M)                                                                           \
    do {                                                                                                     \
        (void)hipFuncSetAttribute((const void *)k_scatter16_wc<K, W, NI, SI, true, M>,                      \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)geo.lds_bytes);           \
        hipLaunchKernelGGL((k_scatter16_wc<K, W, NI, SI, true, M>), dim3(grid), dim3(W * 64),                \
                           geo.lds_bytes, stream, (const u32x4 *)in, (u32x4 *)out, n, (int64_t)0, pp, offs, G, \
                           err, desc, ndesc, nullptr, 0u, seg_end);                                         \
    } while (0)
#define SGX_WCS(W, NI, SI, M)                                         \
    do {                                                              \
        if (key_bits) SGX_WCS_K(KIND_KEY_BITS, W, NI, SI, 0);         \
        else if (digit) SGX_WCS_K(KIND_DIGIT, W, NI, SI, 0);          \
        else SGX_WCS_K(KIND_HASH_POW2, W, NI, SI, M);                 \
    } while (0)
    const int W = geo.waves - WC_GEOM_BASE;
    const bool pad = pp.pad_cnt != nullptr;
    if (W == 8 && geo.mbits == 16 && geo.items == 12) {
        if (pad) SGX_WCS(8, 12, 16, WC_PADDED); else SGX_WCS(8, 12, 16, 0);
    } else if (W == 8 && geo.mbits == 16 && geo.items == 8) {
        if (pad) SGX_WCS(8, 8, 16, WC_PADDED); else SGX_WCS(8, 8, 16, 0);
    } else {
        return hipErrorInvalidValue;
    }
#undef SGX_WCS
#undef SGX_WCS_K
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// The sorted read's segmented window pass.  After the gather the records of
// each partition are contiguous (canonical reducer-major order), so sorting by (partition,
// window bits) needs no pass by the partitioner: one stable write-combining pass by the
// window bits inside every partition's segment -- K4's SEG mode over pieces of the segments,
// each piece's streams starting at offsets from a per-piece histogram -- replaces the
// window pass + partitioner pass (two histograms, two scatters) of the LSD form.
// ------------------------------------------------------------------------------------
constexpr int PH_THREADS = 1024;
template <int KIND>
__global__ __launch_bounds__(PH_THREADS) void k_piece_hist(const u32x4 *__restrict__ in, int64_t n,
                                                           const int64_t *__restrict__ desc, int64_t npieces,
                                                           PartParams pp, uint32_t *__restrict__ cnt) {
    __shared__ uint32_t h[1024];
    const uint32_t Q = pp.R, tid = threadIdx.x;
    for (uint32_t i = tid; i < Q; i += PH_THREADS) h[i] = 0;
    __syncthreads();
    const int64_t k = blockIdx.x;
    const int64_t b = desc[4 * k], e = k + 1 < npieces ? desc[4 * (k + 1)] : n;
    constexpr int U = 4;  // loads in flight per thread
    int64_t i = b + tid;
    for (; i + (U - 1) * PH_THREADS < e; i += U * PH_THREADS) {
        u32x4 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = in[i + u * PH_THREADS];
#pragma unroll
        for (int u = 0; u < U; ++u) atomicAdd(&h[pid_of<KIND>(r[u].x, r[u].y, r[u].z, pp)], 1u);
    }
    for (; i < e; i += PH_THREADS) {
        const u32x4 r = in[i];
        atomicAdd(&h[pid_of<KIND>(r.x, r.y, r.z, pp)], 1u);
    }
    __syncthreads();
    for (uint32_t q = tid; q < Q; q += PH_THREADS) cnt[k * Q + q] = h[q];
}

// A sorted read's first look at its keys in ONE pass (round 5): every piece's window histogram
// for the window the bucket path takes when the keys' top byte varies (the common case: the
// caller checks that guess against the digit histograms and recounts if it was wrong) plus the
// eight digit histograms the skip / window decisions need (k_digit_hist's, with its
// wave-uniform shortcut).  16 B records, KIND_KEY_BITS.
__global__ __launch_bounds__(PH_THREADS) void k_piece_digit_hist(const u32x4 *__restrict__ in, int64_t n,
                                                                 const int64_t *__restrict__ desc, int64_t npieces,
                                                                 PartParams pp, uint32_t *__restrict__ cnt,
                                                                 uint32_t *__restrict__ dhist) {
    __shared__ uint32_t h[1024];
    __shared__ uint32_t dh[8 * 256];
    const uint32_t Q = pp.R, tid = threadIdx.x, lane = tid & 63u;
    for (uint32_t i = tid; i < Q; i += PH_THREADS) h[i] = 0;
    for (uint32_t i = tid; i < 8 * 256; i += PH_THREADS) dh[i] = 0;
    __syncthreads();
    const int64_t k = blockIdx.x;
    const int64_t b = desc[4 * k], e = k + 1 < npieces ? desc[4 * (k + 1)] : n;
    auto count = [&](const u32x4 &r) __attribute__((always_inline)) {
        const uint64_t act = __ballot(1);
        const uint32_t first = (uint32_t)__ffsll((unsigned long long)act) - 1u;
        // (the guessed window of skewed keys -- small keys share their top bits -- is one bin
        // for the whole wave: one atomic, as for the constant digits below)
        const uint32_t q = pid_of<KIND_KEY_BITS>(r.x, r.y, r.z, pp);
        const uint32_t q0 = __builtin_amdgcn_readfirstlane(q);
        if (__ballot(q == q0) == act) {
            if (lane == first) atomicAdd(&h[q0], (uint32_t)__popcll(act));
        } else {
            atomicAdd(&h[q], 1u);
        }
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            uint32_t v = ((d < 4 ? r.x : r.y) >> ((d & 3) * 8)) & 0xFFu;
            if (d == 7) v ^= 0x80u;
            const uint32_t v0 = __builtin_amdgcn_readfirstlane(v);
            if (__ballot(v == v0) == act) {
                if (lane == first) atomicAdd(&dh[d * 256 + v0], (uint32_t)__popcll(act));
            } else {
                atomicAdd(&dh[d * 256 + v], 1u);
            }
        }
    };
    constexpr int U = 4;  // loads in flight per thread
    int64_t i = b + tid;
    for (; i + (U - 1) * PH_THREADS < e; i += U * PH_THREADS) {
        u32x4 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = in[i + u * PH_THREADS];
#pragma unroll
        for (int u = 0; u < U; ++u) count(r[u]);
    }
    for (; i < e; i += PH_THREADS) count(in[i]);
    __syncthreads();
    for (uint32_t q = tid; q < Q; q += PH_THREADS) cnt[k * Q + q] = h[q];
    for (uint32_t j = tid; j < 8 * 256; j += PH_THREADS)
        if (dh[j]) atomicAdd(&dhist[j], dh[j]);
}

hipError_t launch_piece_digit_hist(const void *in, int64_t n, const int64_t *desc, int64_t npieces,
                                   const PartParams &pp, uint32_t *cnt, uint32_t *dhist, hipStream_t st) {
    hipError_t err = hipMemsetAsync(dhist, 0, 8 * 256 * 4, st);
    if (err != hipSuccess || npieces <= 0) return err;
    if (pp.R > 1024 || pp.kind != KIND_KEY_BITS) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_piece_digit_hist, dim3((unsigned)npieces), dim3(PH_THREADS), 0, st, (const u32x4 *)in, n, desc,
                       npieces, pp, cnt, dhist);
    return hipGetLastError();
}

hipError_t launch_piece_hist(const void *in, int64_t n, const int64_t *desc, int64_t npieces, const PartParams &pp,
                             uint32_t *cnt, hipStream_t st) {
    if (npieces <= 0) return hipSuccess;
    if (pp.R > 1024) return hipErrorInvalidValue;
    if (pp.kind == KIND_KEY_BITS)
        hipLaunchKernelGGL(k_piece_hist<KIND_KEY_BITS>, dim3((unsigned)npieces), dim3(PH_THREADS), 0, st,
                           (const u32x4 *)in, n, desc, npieces, pp, cnt);
    else if (pp.kind == KIND_DIGIT)
        hipLaunchKernelGGL(k_piece_hist<KIND_DIGIT>, dim3((unsigned)npieces), dim3(PH_THREADS), 0, st,
                           (const u32x4 *)in, n, desc, npieces, pp, cnt);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// one workgroup per segment s, whose pieces are [pk[s], pk[s+1]): offs[k * Q + q] = the first
// record of segment s + every count before (q, k) in bucket-major, piece-minor order
constexpr int SO_THREADS = 256;
__global__ __launch_bounds__(SO_THREADS) void k_seg_offsets(const uint32_t *__restrict__ cnt,
                                                            const int64_t *__restrict__ seg_base,
                                                            const int32_t *__restrict__ pk, uint32_t Q,
                                                            uint32_t *__restrict__ offs) {
    __shared__ uint32_t s_w[SO_THREADS / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t sg = blockIdx.x;
    const uint32_t k0 = (uint32_t)pk[sg], np = (uint32_t)pk[sg + 1] - k0;
    const uint32_t m = Q * np;  // entries of the segment: j = q * np + (k - k0)
    const uint32_t per = (m + SO_THREADS - 1) / SO_THREADS, j0 = min(m, tid * per), j1 = min(m, j0 + per);
    auto at = [&](uint32_t j) -> int64_t { return (int64_t)(k0 + j % np) * Q + j / np; };
    uint32_t sum = 0;
    for (uint32_t j = j0; j < j1; ++j) sum += cnt[at(j)];
    const uint32_t x = wave_inclusive_scan(sum, lane);
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t base = (uint32_t)seg_base[sg] + x - sum;
    for (uint32_t v = 0; v < w; ++v) base += s_w[v];
    for (uint32_t j = j0; j < j1; ++j) {
        const int64_t a = at(j);
        offs[a] = base;
        base += cnt[a];
    }
}

hipError_t launch_seg_offsets(const uint32_t *cnt, const int64_t *seg_base, const int32_t *pk, int64_t nseg, uint32_t Q,
                              uint32_t *offs, hipStream_t st) {
    if (nseg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_seg_offsets, dim3((unsigned)nseg), dim3(SO_THREADS), 0, st, cnt, seg_base, pk, Q, offs);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// The sorted read's bucket sort.  After the key-window passes (KIND_KEY_BITS) and the pass by
// the shuffle's partitioner, the records are ordered by bucket = (P << kbits) | window bits;
// each bucket (a few dozen records when the window is sized to the data) is sorted stably by
// its full key ON CHIP: a workgroup owns the buckets that START in its TILE of positions
// (plus a HALO to reach the last one's end), stages the records in LDS, finds every
// record's bucket bounds by two block scans of the boundary flags, ranks each record among
// its bucket by comparison (key, then position: stable) and writes the bucket region out
// through the inverse permutation, coalesced.  One read + one write of every record instead
// of the 7-9 LSD digit passes that remain below the window.
// ------------------------------------------------------------------------------------
constexpr int BS_THREADS = 512;
// sub-bins inside each bucket before the rank (A/B: -DSGX_BS_SUBBIN=0, the whole-bucket rank)
#ifndef SGX_BS_SUBBIN
#define SGX_BS_SUBBIN 1
#endif
// the bucket region stored nontemporal (A/B: -DSGX_BS_NT=0)
#ifndef SGX_BS_NT
#define SGX_BS_NT 1
#endif
// 16 B records per bucket-sort tile (A/B builds: -DSGX_BS_TILE16=1280, three workgroups per CU)
#ifndef SGX_BS_TILE16
#define SGX_BS_TILE16 2048
#endif
#ifndef BS_UNROLL
#define BS_UNROLL 8  // keys compared per step of the rank loop (independent LDS loads; 8 vs 4: sorted 1 GiB 3.67 -> 3.62 ms, profiles/r03_bucket_unroll_ab.jsonl)
#endif

// the order key of a staged record: 16 B -> the signed Long sign-flipped (hi), lo = 0;
// 100 B -> the first 8 key bytes big-endian (hi) and the last 2 (lo)
template <int RB>
__device__ __forceinline__ void bucket_key(const uint32_t *r, uint64_t &hi, uint32_t &lo) {
    if constexpr (RB == 16) {
        hi = (((uint64_t)r[1] << 32) | r[0]) ^ 0x8000000000000000ull;
        lo = 0;
    } else {
        hi = ((uint64_t)__builtin_bswap32(r[0]) << 32) | __builtin_bswap32(r[1]);
        lo = __builtin_bswap32(r[2]) >> 16;
    }
}

template <int RB, int TILE, int HALO>
__global__ __launch_bounds__(BS_THREADS) void k_bucket_sort(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                            int64_t n, PartParams pp, int use_p, uint32_t kshift,
                                                            uint32_t kbits, uint32_t *err) {
    constexpr int DW = RB / 4;
    constexpr int CAP = TILE + HALO + 1;
    constexpr bool LO = RB != 16;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint32_t *rec = (uint32_t *)smem;                             // CAP records
    uint64_t *khi = (uint64_t *)(rec + (size_t)CAP * DW);         // order keys (8-aligned: CAP*DW*4 % 8 == 0 below)
    uint32_t *klo = (uint32_t *)(khi + CAP);                      // 100 B: the key's last 2 bytes
    uint16_t *bs = (uint16_t *)(klo + (LO ? CAP : 0));            // bucket start of each local position
    uint16_t *be = bs + CAP;                                      // bucket end
    uint16_t *inv = be + CAP;                                     // output slot -> local position
    uint16_t *cnt = inv + CAP;                                    // sub-bin counts (SGX_BS_SUBBIN)
    uint8_t *flag = (uint8_t *)(cnt + (SGX_BS_SUBBIN ? CAP : 0)); // a bucket starts here
    __shared__ uint32_t s_a, s_b, s_scr[BS_THREADS / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t t0 = (int64_t)blockIdx.x * TILE;
    if (t0 >= n) return;
    const int64_t t1 = min(n, t0 + TILE);
    const int64_t L0 = t0 > 0 ? t0 - 1 : 0, L1 = min(n, t1 + HALO);
    const int m = (int)(L1 - L0);
    const uint64_t wmask = kbits >= 64 ? ~0ull : ((1ull << kbits) - 1ull);
    for (int u = (int)tid; u < m * DW; u += BS_THREADS) rec[u] = in[L0 * DW + u];
    if constexpr (SGX_BS_SUBBIN)
        for (int j = (int)tid; j < m; j += BS_THREADS) cnt[j] = 0;
    if (tid == 0) {
        s_a = 0xFFFFFFFFu;
        s_b = 0xFFFFFFFFu;
    }
    __syncthreads();
    auto comp = [&](int j) -> uint64_t {
        const uint32_t *r = rec + (size_t)j * DW;
        uint64_t hi;
        uint32_t lo;
        bucket_key<RB>(r, hi, lo);
        const uint64_t p = use_p ? (uint64_t)hash_pid(r[0], r[1], pp) : 0ull;
        return (p << kbits) | ((hi >> kshift) & wmask);
    };
    // order keys, boundary flags; the first nominal boundary (a), the first one at or past t1 (b)
    for (int j = (int)tid; j < m; j += BS_THREADS) {
        uint64_t hi;
        uint32_t lo;
        bucket_key<RB>(rec + (size_t)j * DW, hi, lo);
        khi[j] = hi;
        if constexpr (LO) klo[j] = lo;
        const int64_t pos = L0 + j;
        const bool f = pos == 0 || (j > 0 && comp(j) != comp(j - 1));
        flag[j] = f ? 1 : 0;
        if (f && pos >= t0 && pos < t1) atomicMin(&s_a, (uint32_t)j);
        if (f && pos >= t1) atomicMin(&s_b, (uint32_t)j);
    }
    __syncthreads();
    const uint32_t a = s_a;
    uint32_t b = s_b;
    if (b == 0xFFFFFFFFu) {
        if (L1 == n) b = (uint32_t)m;  // the array's end closes the last bucket
        else {
            if (tid == 0 && a != 0xFFFFFFFFu) atomicOr(err, 4u);  // a bucket longer than the halo
            return;
        }
    }
    if (a == 0xFFFFFFFFu) return;  // no bucket starts in this tile
    // bucket bounds of every position in [a, b): start = last flag <= j (prefix max), end =
    // next flag > j (suffix min); one contiguous run of positions per thread
    const int len = (int)(b - a);
    const int per = (len + BS_THREADS - 1) / BS_THREADS;
    const int j0 = (int)a + min(len, (int)tid * per), j1 = (int)a + min(len, ((int)tid + 1) * per);
    {
        int run = -1;
        for (int j = j0; j < j1; ++j) if (flag[j]) run = j;
        int x = run;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(x, d, 64);
            if (lane >= (uint32_t)d) x = max(x, y);
        }
        if (lane == 63) s_scr[w] = (uint32_t)(x + 1);
        __syncthreads();
        int prev = __shfl_up(x, 1, 64);
        if (lane == 0) prev = -1;
        for (uint32_t v = 0; v < w; ++v) prev = max(prev, (int)s_scr[v] - 1);
        int cur = prev;
        for (int j = j0; j < j1; ++j) {
            if (flag[j]) cur = j;
            bs[j] = (uint16_t)cur;
        }
        __syncthreads();
        int nxt = 0x7FFFFFFF;
        for (int j = j1 - 1; j >= j0; --j) if (flag[j]) nxt = j;
        int y2 = nxt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int z = __shfl_down(y2, d, 64);
            if (lane + d < 64) y2 = min(y2, z);
        }
        if (lane == 0) s_scr[w] = (uint32_t)y2;
        __syncthreads();
        int after = __shfl_down(y2, 1, 64);
        if (lane == 63) after = 0x7FFFFFFF;
        for (uint32_t v = w + 1; v < BS_THREADS / 64; ++v) after = min(after, (int)s_scr[v]);
        int e = min(after, (int)b);
        for (int j = j1 - 1; j >= j0; --j) {
            be[j] = (uint16_t)e;
            if (flag[j]) e = j;
        }
    }
    __syncthreads();
#if SGX_BS_SUBBIN
    // Sub-bins (round 5): a bucket [s0, e0) of m records owns the m positions s0 .. e0 - 1 as
    // bins, and record j goes to bin s0 + floor(x_j * m / 2^32), x_j = the 32 key bits right
    // below the window -- monotone in the key, so equal keys share a bin and every key of a
    // lower bin is smaller.  Bins are counted, scanned over [a, b) into output slots, their
    // members listed, and a record is ranked among its bin's members only (about two on
    // uniform keys) instead of among its whole bucket (~64): the rank loop was the kernel's
    // VALU time.  Stable: equal keys rank by position.
    {
        constexpr int PER = (CAP + BS_THREADS - 1) / BS_THREADS;
        const uint32_t kl_sh = kshift;  // the window's low bit
        // S1: bins (kept in be[j] from here on), counts
        for (int j = (int)a + (int)tid; j < (int)b; j += BS_THREADS) {
            const uint32_t s0 = bs[j], mm = (uint32_t)be[j] - s0;
            const uint64_t kh = khi[j];
            const uint64_t below = kl_sh == 0 ? 0ull : (kl_sh >= 32 ? (kh >> (kl_sh - 32)) : (kh << (32 - kl_sh)));
            const uint32_t x = (uint32_t)below;
            const uint32_t bin = s0 + (uint32_t)(((uint64_t)x * mm) >> 32);
            be[j] = (uint16_t)bin;
            atomicAdd((uint32_t *)((uintptr_t)(cnt + (bin & ~1u))), 1u << ((bin & 1u) << 4));
        }
        __syncthreads();
        // S2: exclusive scan of the counts over [a, b) -> bs[bin] = the bin's first output slot
        // (relative to a); one contiguous run of positions per thread
        {
            const int lenb = (int)(b - a);
            const int per = (lenb + BS_THREADS - 1) / BS_THREADS;
            const int q0 = (int)a + min(lenb, (int)tid * per), q1 = (int)a + min(lenb, ((int)tid + 1) * per);
            uint32_t sum = 0;
            for (int q = q0; q < q1; ++q) sum += cnt[q];
            const uint32_t x = wave_inclusive_scan(sum, lane);
            if (lane == 63) s_scr[w] = x;
            __syncthreads();
            uint32_t base = x - sum;
            for (uint32_t v = 0; v < w; ++v) base += s_scr[v];
            for (int q = q0; q < q1; ++q) {
                bs[q] = (uint16_t)base;
                base += cnt[q];
            }
        }
        __syncthreads();
        // S3: list every bin's members in its slots (inv[a + slot], any order: the count runs
        // down)
        for (int j = (int)a + (int)tid; j < (int)b; j += BS_THREADS) {
            const uint32_t bin = be[j];
            const uint32_t sh = (bin & 1u) << 4;
            const uint32_t old = atomicSub((uint32_t *)((uintptr_t)(cnt + (bin & ~1u))), 1u << sh);
            const uint32_t k = ((old >> sh) & 0xFFFFu) - 1u;
            inv[a + bs[bin] + k] = (uint16_t)j;
        }
        __syncthreads();
        // S4: rank among the bin's members (key, then position), slot kept in registers until
        // every member list has been read, then written over be[] as the output permutation
        int myslot[PER], myj[PER];
#pragma unroll
        for (int t = 0; t < PER; ++t) {
            const int j = (int)a + (int)tid + t * BS_THREADS;
            myj[t] = -1;
            if (j >= (int)b) continue;
            const uint32_t bin = be[j];
            const uint32_t st0 = bs[bin], st1 = bin + 1 < b ? bs[bin + 1] : (uint32_t)(b - a);
            const uint64_t kh = khi[j];
            const uint32_t kl = LO ? klo[j] : 0u;
            uint32_t rank = 0;
            for (uint32_t u = st0; u < st1; ++u) {
                const int i = inv[a + u];
                const uint64_t h = khi[i];
                const uint32_t l = LO ? klo[i] : 0u;
                const bool lt = LO ? (h < kh || (h == kh && l < kl)) : h < kh;
                const bool eq = LO ? (h == kh && l == kl) : h == kh;
                rank += (lt || (i < j && eq)) ? 1u : 0u;
            }
            myslot[t] = (int)(a + st0 + rank);
            myj[t] = j;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < PER; ++t)
            if (myj[t] >= 0) be[myslot[t]] = (uint16_t)myj[t];
        __syncthreads();
    }
    const uint16_t *perm = be;
#else
    // stable rank inside the bucket: keys below, plus equal keys at earlier positions.  Keys
    // come from the compact key array four at a time (independent LDS loads, one wait).
    for (int j = (int)a + (int)tid; j < (int)b; j += BS_THREADS) {
        const int s0 = bs[j], e0 = be[j];
        const uint64_t kh = khi[j];
        const uint32_t kl = LO ? klo[j] : 0u;
        int rank = 0, i = s0;
        for (; i + BS_UNROLL <= e0; i += BS_UNROLL) {
            uint64_t h[BS_UNROLL];
            uint32_t l[BS_UNROLL];
#pragma unroll
            for (int q = 0; q < BS_UNROLL; ++q) {
                h[q] = khi[i + q];
                l[q] = LO ? klo[i + q] : 0u;
            }
#pragma unroll
            for (int q = 0; q < BS_UNROLL; ++q) {
                const bool lt = LO ? (h[q] < kh || (h[q] == kh && l[q] < kl)) : h[q] < kh;
                const bool eq = LO ? (h[q] == kh && l[q] == kl) : h[q] == kh;
                rank += (lt || (i + q < j && eq)) ? 1 : 0;
            }
        }
        for (; i < e0; ++i) {
            const uint64_t h = khi[i];
            const uint32_t l = LO ? klo[i] : 0u;
            const bool lt = LO ? (h < kh || (h == kh && l < kl)) : h < kh;
            const bool eq = LO ? (h == kh && l == kl) : h == kh;
            rank += (lt || (i < j && eq)) ? 1 : 0;
        }
        inv[s0 + rank] = (uint16_t)j;
    }
    __syncthreads();
    const uint16_t *perm = inv;
#endif
    // the bucket region, coalesced: output position L0 + p takes local record perm[p]
    if constexpr (RB == 16) {
        for (int p = (int)a + (int)tid; p < (int)b; p += BS_THREADS) {
            if (SGX_BS_NT) __builtin_nontemporal_store(((const u32x4 *)rec)[perm[p]], (u32x4 *)out + L0 + p);
            else ((u32x4 *)out)[L0 + p] = ((const u32x4 *)rec)[perm[p]];
        }
    } else {
        for (int u = (int)tid; u < len * DW; u += BS_THREADS) {
            const int p = (int)a + u / DW, q = u % DW;
            out[(L0 + p) * DW + q] = rec[(size_t)perm[p] * DW + q];
        }
    }
}

template <int RB, int TILE, int HALO>
static size_t bucket_sort_lds() {
    constexpr int CAP = TILE + HALO + 1;
    return (size_t)CAP * RB + (size_t)CAP * 8 + (RB != 16 ? (size_t)CAP * 4 : 0) + (size_t)CAP * (SGX_BS_SUBBIN ? 8 : 6) +
           (size_t)CAP + 16;
}

hipError_t launch_bucket_sort(const void *in, void *out, int64_t n, int rb, const PartParams &pp, int use_p,
                              uint32_t kshift, uint32_t kbits, uint32_t *err, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    if (rb == 16) {
        // CAP = 2560 (sub-bins: 2304, two workgroups per CU): the key array stays 8-byte aligned
        constexpr int T = SGX_BS_TILE16, H = SGX_BS_SUBBIN ? 255 : 511;
        const size_t lds = bucket_sort_lds<16, T, H>();
        (void)hipFuncSetAttribute((const void *)k_bucket_sort<16, T, H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL((k_bucket_sort<16, T, H>), dim3((unsigned)((n + T - 1) / T)), dim3(BS_THREADS), lds, stream,
                           (const uint32_t *)in, (uint32_t *)out, n, pp, use_p, kshift, kbits, err);
    } else if (rb == 100) {
        // CAP = 640 (even: 100 B records keep the key array 8-aligned); with sub-bins a halo of 127
        // (buckets average ~64 records) reads 1.25x the tile instead of 1.66x
        constexpr int T = SGX_BS_SUBBIN ? 512 : 384, H = SGX_BS_SUBBIN ? 127 : 253;
        const size_t lds = bucket_sort_lds<100, T, H>();
        (void)hipFuncSetAttribute((const void *)k_bucket_sort<100, T, H>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds);
        hipLaunchKernelGGL((k_bucket_sort<100, T, H>), dim3((unsigned)((n + T - 1) / T)), dim3(BS_THREADS), lds,
                           stream, (const uint32_t *)in, (uint32_t *)out, n, pp, use_p, kshift, kbits, err);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// Engine-start self-check of the ordering the lane-ordered ranking rests on (K4's
// k_scatter16_wc / _ord / _wide2 and the reduce side's digit and key-window passes): NI
// same-address LDS atomics issued back to back by one wave return their old values in
// (issue order, then lane order).  Probed once per engine with the ranking's exact
// instruction pattern (packed u16 counters, relaxed workgroup-scope fetch-add, one wait):
// every (item k, lane l) must receive exactly the number of earlier (k' < k, or k' == k and
// l' < l) increments of its counter.  A violation sets *bad.
// ------------------------------------------------------------------------------------
constexpr int PROBE_NI = 8, PROBE_ROUNDS = 96;
__global__ __launch_bounds__(512) void k_lds_order_probe(uint32_t *bad) {
    __shared__ uint32_t rows[8][64];  // per wave: 128 packed u16 counters
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t viol = 0;
    for (int r = 0; r < PROBE_ROUNDS; ++r) {
        rows[w][lane] = 0u;  // each wave zeroes its own row (a wave's LDS ops run in order)
        const int K = 1 + (int)((blockIdx.x * 7u + (uint32_t)r * 13u + w) % 48u);  // 1..48 counters
        uint32_t p[PROBE_NI], old[PROBE_NI];
#pragma unroll
        for (int k = 0; k < PROBE_NI; ++k) {
            uint32_t h = (blockIdx.x * 2654435761u) ^ ((uint32_t)r * 40503u) ^ (w * 97u + (uint32_t)k * 1031u) ^
                         (lane * 0x9E3779B9u);
            h ^= h >> 15;
            h *= 0x2C1B3C6Du;
            h ^= h >> 12;
            p[k] = h % (uint32_t)K;
        }
#pragma unroll
        for (int k = 0; k < PROBE_NI; ++k)
            old[k] = __hip_atomic_fetch_add(&rows[w][p[k] >> 1], 1u << ((p[k] & 1u) << 4), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
        for (int k = 0; k < PROBE_NI; ++k) {
            const uint32_t got = (old[k] >> ((p[k] & 1u) << 4)) & 0xFFFFu;
            uint32_t want = 0;
            for (int k2 = 0; k2 <= k; ++k2) {
                // lanes whose item k2 hit the same counter as my item k
                uint64_t same = 0;
                for (uint32_t v = 0; v < (uint32_t)K; ++v) {
                    const uint64_t m = __ballot(p[k2] == v);
                    if (v == p[k]) same = m;
                }
                want += (uint32_t)__popcll(k2 < k ? same : (same & ((1ull << lane) - 1ull)));
            }
            viol |= got != want ? 1u : 0u;
        }
    }
    if (viol) atomicOr(bad, 1u);
}

hipError_t launch_lds_order_probe(uint32_t *bad, hipStream_t stream) {
    hipLaunchKernelGGL(k_lds_order_probe, dim3(512), dim3(512), 0, stream, bad);
    return hipGetLastError();
}

hipError_t launch_scatter(const void *in, void *out, int64_t n, int rb, int64_t chunk, int G,
                          const PartParams &pp, const uint32_t *offs, const ScatterGeom &geo,
                          uint32_t *err, hipStream_t stream, void *out2, uint32_t hot_cap) {
    const bool pow2 = (pp.R & (pp.R - 1)) == 0;
    if (rb == 16 && geo.waves >= WC_GEOM_BASE) {
        if ((pp.kind != SGX_PART_HASH && pp.kind != KIND_DIGIT && pp.kind != KIND_HASH_BITS &&
             pp.kind != KIND_KEY_BITS && pp.kind != KIND_HOT_SPLIT) ||
            geo.waves < WC_GEOM_BASE)
            return hipErrorInvalidValue;
#define SGX_WC_SIM(K, W, NI, SI, M)                                                              \
    do {                                                                                         \
        (void)hipFuncSetAttribute((const void *)k_scatter16_wc<K, W, NI, SI, false, M>,         \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)geo.lds_bytes); \
        hipLaunchKernelGGL((k_scatter16_wc<K, W, NI, SI, false, M>), dim3(G), dim3(W * 64),      \
                           geo.lds_bytes, stream, (const u32x4 *)in, (u32x4 *)out, n, chunk, pp, \
                           offs, G, err, nullptr, nullptr, (u32x4 *)out2, hot_cap);              \
    } while (0)
#define SGX_WC_SI(K, W, NI, SI) SGX_WC_SIM(K, W, NI, SI, 0)
        // geometries: 8 waves, NI 12 | 8, SI 16, one workgroup per CU
        const int W = geo.waves - WC_GEOM_BASE;
#define SGX_WC(K)                                                                                \
    do {                                                                                         \
        if (W == 8 && geo.mbits == 16 && geo.items == 12) SGX_WC_SI(K, 8, 12, 16);               \
        else if (W == 8 && geo.mbits == 16 && geo.items == 8) SGX_WC_SI(K, 8, 8, 16);            \
        else return hipErrorInvalidValue;                                                        \
    } while (0)
        // a padded write's K4 and its fallback's (hash partitioner only)
        const int mode = pp.pad_cnt ? WC_PADDED : pp.guard ? WC_FALLBACK : 0;
        const bool hot_split = pp.kind == KIND_HOT_SPLIT;  // level 1 of the padded split
        if (mode && ((pp.kind != SGX_PART_HASH && !(hot_split && mode == WC_PADDED)) ||
                     !(W == 8 && geo.mbits == 16 && (geo.items == 12 || geo.items == 8)) ||
                     (mode == WC_PADDED && ((!pp.pad_cap && !(pp.pad_est && pp.pad_layout)) || !pp.olim)) ||
                     (hot_split && (!pp.dir || !out2 || pp.dshift > 13))))
            return hipErrorInvalidValue;
#define SGX_WC_PAD(K)                                                                            \
    do {                                                                                         \
        if (mode == WC_PADDED) {                                                                 \
            if (geo.items == 12) SGX_WC_SIM(K, 8, 12, 16, WC_PADDED);                           \
            else SGX_WC_SIM(K, 8, 8, 16, WC_PADDED);                                            \
        } else {                                                                                 \
            if (geo.items == 12) SGX_WC_SIM(K, 8, 12, 16, WC_FALLBACK);                         \
            else SGX_WC_SIM(K, 8, 8, 16, WC_FALLBACK);                                          \
        }                                                                                        \
    } while (0)
        if (mode) {
            if (hot_split) {
                if (geo.items == 12) SGX_WC_SIM(KIND_HOT_SPLIT, 8, 12, 16, WC_PADDED);
                else SGX_WC_SIM(KIND_HOT_SPLIT, 8, 8, 16, WC_PADDED);
            } else if (pow2) {
                SGX_WC_PAD(KIND_HASH_POW2);
            } else {
                SGX_WC_PAD(SGX_PART_HASH);
            }
#undef SGX_WC_PAD
        } else if (pp.kind == KIND_DIGIT) {
            if (pp.R != DIGIT_R) return hipErrorInvalidValue;
            SGX_WC(KIND_DIGIT);
        } else if (pp.kind == KIND_KEY_BITS) {
            if (!pow2) return hipErrorInvalidValue;
            SGX_WC(KIND_KEY_BITS);
        } else if (pp.kind == KIND_HASH_BITS) {
            if (!pow2) return hipErrorInvalidValue;
            SGX_WC(KIND_HASH_BITS);
        } else if (pp.kind == KIND_HOT_SPLIT) {
            if (!pp.dir || !out2 || pp.dshift > 13) return hipErrorInvalidValue;
            SGX_WC(KIND_HOT_SPLIT);
        } else if (pow2) {
            SGX_WC(KIND_HASH_POW2);
        } else {
            SGX_WC(SGX_PART_HASH);
        }
#undef SGX_WC
#undef SGX_WC_SI
#undef SGX_WC_SIM
        return hipGetLastError();
    }
    if (rb == 16 && geo.waves >= ORD_GEOM_BASE) {
        const int W = geo.waves - ORD_GEOM_BASE;
#define SGX_ORD(K, WV, I, P)                                                                     \
    do {                                                                                         \
        (void)hipFuncSetAttribute((const void *)k_scatter16_ord<K, WV, I, P>,                   \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)geo.lds_bytes); \
        hipLaunchKernelGGL((k_scatter16_ord<K, WV, I, P>), dim3(G), dim3(WV * 64), geo.lds_bytes, \
                           stream, (const u32x4 *)in, (u32x4 *)out, n, chunk, pp, offs, G, err); \
    } while (0)
#define SGX_ORD_K(K)                                                      \
    do {                                                                  \
        switch (W * 10000 + geo.items * 100 + geo.mbits) {                \
        case 81601: SGX_ORD(K, 8, 16, 1); break;                          \
        case 121001: SGX_ORD(K, 12, 10, 1); break;                        \
        case 160701: SGX_ORD(K, 16, 7, 1); break;                         \
        case 80802: SGX_ORD(K, 8, 8, 2); break;                           \
        case 41608: SGX_ORD(K, 4, 16, 8); break;                          \
        default: return hipErrorInvalidValue;                             \
        }                                                                 \
    } while (0)
        if (pp.kind != SGX_PART_HASH) return hipErrorInvalidValue;
        if (pow2) SGX_ORD_K(KIND_HASH_POW2);
        else SGX_ORD_K(SGX_PART_HASH);
#undef SGX_ORD_K
#undef SGX_ORD
        return hipGetLastError();
    }
    // (16 B digit / key-window passes reach the per-lane kernel below only when the engine-start
    // LDS ordering check failed)
    if (rb == 16 && pp.kind != KIND_DIGIT && pp.kind != KIND_KEY_BITS) {
        if (geo.items == 0) return hipErrorInvalidValue;
        const uint4 *i4 = (const uint4 *)in;
        uint4 *o4 = (uint4 *)out;
#define SGX_SC16(K, W, I)                                                                       \
    do {                                                                                        \
        (void)hipFuncSetAttribute((const void *)k_scatter16<K, W, I>,                          \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)geo.lds_bytes); \
        hipLaunchKernelGGL((k_scatter16<K, W, I>), dim3(G), dim3(W * 64), geo.lds_bytes, stream, \
                           i4, o4, n, chunk, pp, offs, G, err);                                \
    } while (0)
#define SGX_SC16_K(K)                                                        \
    do {                                                                     \
        switch (geo.waves * 100 + geo.items) {                               \
        case 416: SGX_SC16(K, 4, 16); break;                                 \
        case 816: SGX_SC16(K, 8, 16); break;                                 \
        case 1210: SGX_SC16(K, 12, 10); break;                               \
        case 1409: SGX_SC16(K, 14, 9); break;                                \
        case 1607: SGX_SC16(K, 16, 7); break;                                \
        case 412: SGX_SC16(K, 4, 12); break;                                 \
        case 808: SGX_SC16(K, 8, 8); break;                                  \
        case 408: SGX_SC16(K, 4, 8); break;                                  \
        case 804: SGX_SC16(K, 8, 4); break;                                  \
        case 404: SGX_SC16(K, 4, 4); break;                                  \
        case 402: SGX_SC16(K, 4, 2); break;                                  \
        case 401: SGX_SC16(K, 4, 1); break;                                  \
        default: return hipErrorInvalidValue;                                \
        }                                                                    \
    } while (0)
        switch (pp.kind) {
        case SGX_PART_HASH: SGX_SC16_K(SGX_PART_HASH); break;
        case SGX_PART_RANGE_I64: SGX_SC16_K(SGX_PART_RANGE_I64); break;
        case SGX_PART_RANGE_BYTES10: SGX_SC16_K(SGX_PART_RANGE_BYTES10); break;
        default: return hipErrorInvalidValue;
        }
#undef SGX_SC16_K
#undef SGX_SC16
    } else if (rb == 100 && geo.waves == WIDE2_GEOM_TAG) {
        if (((uintptr_t)in & 15) != 0) return hipErrorInvalidValue;
#define SGX_W2M(K, M)                                                                            \
    do {                                                                                         \
        (void)hipFuncSetAttribute((const void *)k_scatter_wide2<K, 100, M>,                     \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)geo.lds_bytes); \
        hipLaunchKernelGGL((k_scatter_wide2<K, 100, M>), dim3(G), dim3(512), geo.lds_bytes, stream, \
                           (const u32x4 *)in, (uint32_t *)out, n, chunk, pp, offs, G, err);     \
    } while (0)
#define SGX_W2(K) SGX_W2M(K, 0)
        // a padded write's K4 and its fallback's (RangePartitioner over 10-byte keys)
        const int mode = pp.pad_cnt ? WC_PADDED : pp.guard ? WC_FALLBACK : 0;
        if (mode) {
            if (pp.kind != SGX_PART_RANGE_BYTES10 ||
                (mode == WC_PADDED && ((!pp.pad_cap && !(pp.pad_est && pp.pad_layout)) || !pp.olim)))
                return hipErrorInvalidValue;
            // the padded K4 write-combines whole 64 B units when its LDS fits (R <= 1024); only
            // that kernel lays its sub-bins out itself
            const bool wwc = wide_wc_padded_ok(pp.R, pp.nb, chunk);
            if (mode == WC_PADDED && pp.pad_est && !wwc) return hipErrorInvalidValue;
            if (mode == WC_PADDED && wwc) {
                const size_t wlds = scatter_wide_wc_lds(pp.R, pp.nb);
                (void)hipFuncSetAttribute((const void *)k_scatter_wide_wc<SGX_PART_RANGE_BYTES10, WC_PADDED>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)wlds);
                hipLaunchKernelGGL((k_scatter_wide_wc<SGX_PART_RANGE_BYTES10, WC_PADDED>), dim3(G), dim3(512), wlds,
                                   stream, (const u32x4 *)in, (uint32_t *)out, n, chunk, pp, offs, G, err);
                return hipGetLastError();
            }
            if (mode == WC_PADDED) SGX_W2M(SGX_PART_RANGE_BYTES10, WC_PADDED);
            else SGX_W2M(SGX_PART_RANGE_BYTES10, WC_FALLBACK);
            return hipGetLastError();
        }
        switch (pp.kind) {
        case SGX_PART_HASH:
            if (pow2) SGX_W2(KIND_HASH_POW2); else SGX_W2(SGX_PART_HASH);
            break;
#define SGX_WWC_OR_W2(K)                                                                                      \
    do {                                                                                                      \
        const size_t wlds = scatter_wide_wc_lds(pp.R, pp.nb);                                                 \
        if (SGX_WIDE_WC && SGX_WIDE_WC_REDUCE && pp.R <= 1024 && wlds <= LDS_MAX && chunk % WWC_TR == 0) {    \
            (void)hipFuncSetAttribute((const void *)k_scatter_wide_wc<K, 0>,                                  \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)wlds);                 \
            hipLaunchKernelGGL((k_scatter_wide_wc<K, 0>), dim3(G), dim3(512), wlds, stream, (const u32x4 *)in, \
                               (uint32_t *)out, n, chunk, pp, offs, G, err);                                  \
        } else {                                                                                              \
            SGX_W2(K);                                                                                        \
        }                                                                                                     \
    } while (0)
        // the reduce side's digit / key-window passes over 100 B records
        case KIND_DIGIT: SGX_WWC_OR_W2(KIND_DIGIT); break;
        case KIND_KEY_BITS: SGX_WWC_OR_W2(KIND_KEY_BITS); break;
#undef SGX_WWC_OR_W2
        case SGX_PART_RANGE_I64: SGX_W2(SGX_PART_RANGE_I64); break;
        case SGX_PART_RANGE_BYTES10: {
            // the two-pass TeraSort K4 write-combines too (streams start at their offsets)
            const size_t wlds = scatter_wide_wc_lds(pp.R, pp.nb);
            if (SGX_WIDE_WC && SGX_WIDE_WC_TWOPASS && pp.R <= 1024 && wlds <= LDS_MAX && chunk % WWC_TR == 0) {
                (void)hipFuncSetAttribute((const void *)k_scatter_wide_wc<SGX_PART_RANGE_BYTES10, 0>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)wlds);
                hipLaunchKernelGGL((k_scatter_wide_wc<SGX_PART_RANGE_BYTES10, 0>), dim3(G), dim3(512), wlds, stream,
                                   (const u32x4 *)in, (uint32_t *)out, n, chunk, pp, offs, G, err);
            } else {
                SGX_W2(SGX_PART_RANGE_BYTES10);
            }
            break;
        }
        default: return hipErrorInvalidValue;
        }
#undef SGX_W2
#undef SGX_W2M
    } else {
        if (geo.items == 0 || (rb & 3) != 0 || rb < 12) return hipErrorInvalidValue;
        const char *ic = (const char *)in;
        char *oc = (char *)out;
#define SGX_SCW(K)                                                                              \
    do {                                                                                        \
        (void)hipFuncSetAttribute((const void *)k_scatter_wide<K, 4>,                          \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)geo.lds_bytes); \
        hipLaunchKernelGGL((k_scatter_wide<K, 4>), dim3(G), dim3(WIDE_THREADS), geo.lds_bytes,   \
                           stream, ic, oc, n, rb, chunk, pp, offs, G, err);                    \
    } while (0)
        switch (pp.kind) {
        case SGX_PART_HASH: SGX_SCW(SGX_PART_HASH); break;
        case KIND_DIGIT: SGX_SCW(KIND_DIGIT); break;        // lds_order_ok == false
        case KIND_KEY_BITS: SGX_SCW(KIND_KEY_BITS); break;  // lds_order_ok == false
        case SGX_PART_RANGE_I64: SGX_SCW(SGX_PART_RANGE_I64); break;
        case SGX_PART_RANGE_BYTES10: SGX_SCW(SGX_PART_RANGE_BYTES10); break;
        default: return hipErrorInvalidValue;
        }
#undef SGX_SCW
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// K5: copy items {src_off, dst_off, bytes} (regroup of the exchange's receive buffer into
// per-reducer runs ordered by source rank).  One workgroup per item, coalesced.
// ------------------------------------------------------------------------------------
template <int ALIGN>
__global__ __launch_bounds__(256) void k_copy_items(const char *__restrict__ src,
                                                    char *__restrict__ dst,
                                                    const int64_t *__restrict__ items) {
    const int64_t *it = items + 3 * (int64_t)blockIdx.x;
    const int64_t so = it[0], d0 = it[1], bytes = it[2];
    if constexpr (ALIGN == 16) {
        const uint4 *s = (const uint4 *)(src + so);
        uint4 *d = (uint4 *)(dst + d0);
        const int64_t m = bytes >> 4;
        for (int64_t i = threadIdx.x; i < m; i += 256) d[i] = s[i];
    } else {
        const uint32_t *s = (const uint32_t *)(src + so);
        uint32_t *d = (uint32_t *)(dst + d0);
        const int64_t m = bytes >> 2;
        for (int64_t i = threadIdx.x; i < m; i += 256) d[i] = s[i];
    }
}

hipError_t launch_copy_items(const void *src, void *dst, const int64_t *items, int64_t n_items,
                             int align, hipStream_t stream) {
    if (n_items <= 0) return hipSuccess;
    if (align == 16)
        hipLaunchKernelGGL(k_copy_items<16>, dim3((unsigned)n_items), dim3(256), 0, stream,
                           (const char *)src, (char *)dst, items);
    else
        hipLaunchKernelGGL(k_copy_items<4>, dim3((unsigned)n_items), dim3(256), 0, stream,
                           (const char *)src, (char *)dst, items);
    return hipGetLastError();
}

// Gather (fetchBlocksByBlockIds): items {src address, dst address, bytes}, one workgroup
// per <= 64 KiB piece; ALIGN 16 when every address and size is 16-byte aligned, else 4
// (blocks are whole records: 16 B or 100 B).
template <int ALIGN>
__global__ __launch_bounds__(256) void k_gather_items(const int64_t *__restrict__ items) {
    const int64_t *it = items + 3 * (int64_t)blockIdx.x;
    const int64_t bytes = it[2];
    if constexpr (ALIGN == 16) {
        const uint4 *s = (const uint4 *)(uintptr_t)it[0];
        uint4 *d = (uint4 *)(uintptr_t)it[1];
        for (int64_t i = threadIdx.x; i < (bytes >> 4); i += 256) d[i] = s[i];
    } else if constexpr (ALIGN == 4) {
        const uint32_t *s = (const uint32_t *)(uintptr_t)it[0];
        uint32_t *d = (uint32_t *)(uintptr_t)it[1];
        for (int64_t i = threadIdx.x; i < (bytes >> 2); i += 256) d[i] = s[i];
    } else {
        // byte-granular blocks (Kryo-framed shuffles): the destination's whole dwords are
        // built from two aligned source dwords (a dword that holds a valid source byte lies
        // inside the allocation), the head / tail bytes are copied one by one
        const uint8_t *s = (const uint8_t *)(uintptr_t)it[0];
        uint8_t *d = (uint8_t *)(uintptr_t)it[1];
        const int64_t hb = min<int64_t>(bytes, (int64_t)((4u - ((uintptr_t)d & 3u)) & 3u));
        const int64_t nw = (bytes - hb) >> 2;
        const int64_t tb = hb + 4 * nw;
        if ((int64_t)threadIdx.x < hb) d[threadIdx.x] = s[threadIdx.x];
        if ((int64_t)threadIdx.x < bytes - tb) d[tb + threadIdx.x] = s[tb + threadIdx.x];
        const uint8_t *sb = s + hb;
        const uint32_t sh = 8u * (uint32_t)((uintptr_t)sb & 3u);
        const uint32_t *sw = (const uint32_t *)((uintptr_t)sb & ~(uintptr_t)3);
        uint32_t *dw = (uint32_t *)(d + hb);
        for (int64_t i = threadIdx.x; i < nw; i += 256) {
            const uint32_t lo = sw[i];
            dw[i] = sh ? (lo >> sh) | (sw[i + 1] << (32u - sh)) : lo;
        }
    }
}

hipError_t launch_gather_items(const int64_t *items, int64_t n_items, int align, hipStream_t stream) {
    if (n_items <= 0) return hipSuccess;
    if (align == 16)
        hipLaunchKernelGGL(k_gather_items<16>, dim3((unsigned)n_items), dim3(256), 0, stream, items);
    else if (align == 4)
        hipLaunchKernelGGL(k_gather_items<4>, dim3((unsigned)n_items), dim3(256), 0, stream, items);
    else
        hipLaunchKernelGGL(k_gather_items<1>, dim3((unsigned)n_items), dim3(256), 0, stream, items);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// Single-pass padded map output.  The two-pass map side reads every record
// twice (K1+K2's histogram, then K4): 48 B of HBM per 16 B record instead of 32.  The
// padded write skips the full histogram.  A sampled histogram (one line in `stride`) sizes
// a sub-bin per (partition, chunk) stream with a Poisson margin; K4 writes every stream from
// the start of its sub-bin (line-aligned) and reports the streams' true counts; K3 then
// scans those counts into the index offsets and each stream's place in the contiguous
// layout.  The output keeps every partition's streams in chunk order, i.e. in input order,
// with unwritten gaps between them, and is read through the fragment tables
// (k_gather_frags).  A stream longer than its sub-bin sets PAD_OVERFLOW and the map is
// redone by the two-pass kernels guarded on that bit, on the same stream.
// ------------------------------------------------------------------------------------
// 128 workgroups of 1024 threads, 8 loads in flight per lane: 13 µs at C1 against 23-25 µs for
// 512 x 256 (fewer workgroups end with fewer global atomics into est; profiles/r06e_*.log)
#ifndef SGX_PAD_SAMPLE_THREADS  // (A/B builds: -DSGX_PAD_SAMPLE_THREADS / _GRID / _UNROLL)
#define SGX_PAD_SAMPLE_THREADS 1024
#endif
#ifndef SGX_PAD_SAMPLE_GRID
#define SGX_PAD_SAMPLE_GRID 128
#endif
#ifndef SGX_PAD_SAMPLE_UNROLL
#define SGX_PAD_SAMPLE_UNROLL 8
#endif
constexpr int PAD_SAMPLE_THREADS = SGX_PAD_SAMPLE_THREADS;
constexpr int PAD_SAMPLE_UNROLL = SGX_PAD_SAMPLE_UNROLL;
// few workgroups, many loads each: every workgroup ends with up to R global atomics into the
// same R counters (2048 workgroups of 4 loads per lane measured 63 µs at C1, mostly that)
constexpr int PAD_SAMPLE_GRID = SGX_PAD_SAMPLE_GRID;
constexpr int PAD_SAMPLE_MAX_R = 4096;

int64_t pad_sampled_records(int64_t n, int stride) {
    if (n <= 0) return 0;
    const int64_t nlines = (n + 7) / 8, ns = (nlines + stride - 1) / stride;
    const int64_t last = (ns - 1) * stride * 8;  // the last sampled line's first record
    return (ns - 1) * 8 + (n - last < 8 ? n - last : 8);
}

// sample slots per chunk of a streaming map (chunk table): every chunk is sampled on its own,
// one group of 8 records in `stride`, like a whole map
__host__ __device__ inline int64_t pad_chunk_slots(int64_t chunk, int stride) {
    return ((chunk + 7) / 8 + stride - 1) / stride * 8;
}

template <int KIND, int RB>
__global__ __launch_bounds__(PAD_SAMPLE_THREADS) void k_pad_sample(const char *__restrict__ in, int64_t n,
                                                                   int stride, PartParams pp,
                                                                   uint32_t *__restrict__ est, int64_t chunk,
                                                                   int G) {
    __shared__ uint32_t h[PAD_SAMPLE_MAX_R];
    const uint32_t tid = threadIdx.x;
    for (uint32_t p = tid; p < pp.R; p += PAD_SAMPLE_THREADS) h[p] = 0;
    __syncthreads();
    const int64_t nlines = (n + 7) / 8, ns = (nlines + stride - 1) / stride;
    const int64_t per = pp.chunks ? pad_chunk_slots(chunk, stride) : 0;
    const int64_t nt = pp.chunks ? per * G : ns * 8;
    const int64_t step = (int64_t)gridDim.x * PAD_SAMPLE_THREADS;
    // sampled slot t = record t & 7 of group (t >> 3) * stride of 8 records: 8 lanes read one
    // 128 B line (16 B records) or 800 B (100 B records); a streaming map's slot t is slot
    // t % per of chunk t / per
    for (int64_t t0 = (int64_t)blockIdx.x * PAD_SAMPLE_THREADS + tid; t0 < nt; t0 += step * PAD_SAMPLE_UNROLL) {
        uint32_t x[PAD_SAMPLE_UNROLL], y[PAD_SAMPLE_UNROLL], z[PAD_SAMPLE_UNROLL];
        bool ok[PAD_SAMPLE_UNROLL];
#pragma unroll
        for (int u = 0; u < PAD_SAMPLE_UNROLL; ++u) {
            int64_t t = t0 + u * step, lim = n;
            const char *base = in;
            if (pp.chunks && t < nt) {
                const int64_t g = t / per;
                t -= g * per;
                base = in + pp.chunks[2 * g];
                lim = pp.chunks[2 * g + 1];
            }
            const int64_t i = (t >> 3) * stride * 8 + (t & 7);
            ok[u] = t0 + u * step < nt && i < lim;
            x[u] = y[u] = z[u] = 0;
            if (ok[u]) {
                if constexpr (RB == 16) {
                    const uint4 r = ((const uint4 *)base)[i];
                    x[u] = r.x;
                    y[u] = r.y;
                    z[u] = r.z;
                } else {
                    const uint32_t *q = (const uint32_t *)(base + i * RB);
                    x[u] = q[0];
                    y[u] = q[1];
                    z[u] = q[2];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < PAD_SAMPLE_UNROLL; ++u)
            if (ok[u]) atomicAdd(&h[pid_of<KIND>(x[u], y[u], z[u], pp)], 1u);
    }
    __syncthreads();
    for (uint32_t p = tid; p < pp.R; p += PAD_SAMPLE_THREADS)
        if (h[p]) atomicAdd(&est[p], h[p]);
}

hipError_t launch_pad_sample(const void *in, int64_t n, int rb, int stride, const PartParams &pp, uint32_t *est,
                             hipStream_t stream, int64_t chunk, int G) {
    if (pp.R > (uint32_t)PAD_SAMPLE_MAX_R || stride < 1) return hipErrorInvalidValue;
    if (n <= 0) return hipSuccess;
    const int64_t nt = pp.chunks ? pad_chunk_slots(chunk, stride) * G : pad_sampled_records(n, stride) + 8;
    const int64_t per = (int64_t)PAD_SAMPLE_THREADS * PAD_SAMPLE_UNROLL;
    const int64_t want = (nt + per - 1) / per;
    const int grid = (int)(want < 1 ? 1 : want > PAD_SAMPLE_GRID ? PAD_SAMPLE_GRID : want);
    const char *c = (const char *)in;
    if (rb == 16 && pp.kind == SGX_PART_HASH)
        hipLaunchKernelGGL((k_pad_sample<SGX_PART_HASH, 16>), dim3(grid), dim3(PAD_SAMPLE_THREADS), 0, stream, c, n,
                           stride, pp, est, chunk, G);
    else if (rb == 100 && pp.kind == SGX_PART_RANGE_BYTES10)
        hipLaunchKernelGGL((k_pad_sample<SGX_PART_RANGE_BYTES10, 100>), dim3(grid), dim3(PAD_SAMPLE_THREADS), 0, stream,
                           c, n, stride, pp, est, chunk, G);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// The tail of a padded write whose K4 laid the sub-bins out (launch_pad_finish in sgx_internal.h).
__global__ __launch_bounds__(256) void k_pad_finish(const uint32_t *__restrict__ layout, int R, int G, uint32_t olim,
                                                    uint32_t *__restrict__ fstart, uint32_t *__restrict__ cnt,
                                                    uint32_t *flags, uint32_t *__restrict__ zero, int64_t nzero) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < nzero) zero[i] = 0u;
    bool ovf = false;
    if (i < (int64_t)R * G) {
        const int p = (int)(i / G), g = (int)(i - (int64_t)p * G);
        const uint32_t cap = layout[p];
        // (pad_layout_starts' layout: chunk-major, a chunk's region = the sum of the capacities)
        const uint64_t total = (uint64_t)layout[R + R - 1] + layout[R - 1];
        const uint64_t at = SGX_PAD_CHUNK_MAJOR ? (uint64_t)g * total + layout[R + p]
                                                : (uint64_t)layout[R + p] + (uint64_t)g * cap;
        const uint32_t f = (uint32_t)min<uint64_t>(at, (uint64_t)olim);
        const uint32_t c = cnt[i] - f;  // K4 left the stream's end position
        fstart[i] = f;
        cnt[i] = c;
        ovf = c > cap;
    }
    const uint64_t any = __ballot(ovf);
    if (any && __lane_id() == (uint32_t)__ffsll((unsigned long long)any) - 1) atomicOr(flags, PAD_OVERFLOW);
}

hipError_t launch_pad_finish(const uint32_t *layout, int R, int G, uint32_t olim, uint32_t *fstart, uint32_t *cnt,
                             uint32_t *flags, uint32_t *zero, int64_t nzero, hipStream_t stream) {
    int64_t m = (int64_t)R * G;
    if (nzero > m) m = nzero;
    if (m < 1) m = 1;
    hipLaunchKernelGGL(k_pad_finish, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, layout, R, G, olim,
                       fstart, cnt, flags, zero, nzero);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_pad_reset(uint32_t *flags, uint32_t *flags_out, uint32_t *est, int R) {
    if (threadIdx.x == 0) {
        *flags_out = *flags;
        *flags = 0u;
    }
    for (int p = threadIdx.x; p < R; p += 256) est[p] = 0u;
}

hipError_t launch_pad_reset(uint32_t *flags, uint32_t *flags_out, uint32_t *est, int R, hipStream_t stream) {
    hipLaunchKernelGGL(k_pad_reset, dim3(1), dim3(256), 0, stream, flags, flags_out, est, R);
    return hipGetLastError();
}

// The padded split's overflow fallback histogram (launch_hist16_fallback): the per-(partition,
// chunk) counts of the map, [R][G], one wave per chunk, ballot-matched partitions and one
// global atomic per partition present in each 64 records.  No LDS, so like the rest of the
// split's tail it runs beside the next write's K4s; a no-op unless *guard has PAD_OVERFLOW.
// (The split cannot take its counts from the padded write as the 16 B path does: an
// overflowing level-1 sub-bin corrupts the scratch level 2 partitions.)  counts: zeroed.
template <int KIND>
__global__ __launch_bounds__(64) void k_hist16_fb(const uint4 *__restrict__ in, int64_t n, int64_t chunk,
                                                  PartParams pp, uint32_t *counts, int G, const uint32_t *guard) {
    if (!(*guard & PAD_OVERFLOW)) return;
    const int g = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const int64_t begin = (int64_t)g * chunk;
    const int64_t len = min(n, begin + chunk) - begin;
    for (int64_t i0 = 0; i0 < len; i0 += 64) {
        const int64_t i = i0 + lane;
        const bool valid = i < len;
        const uint4 r = valid ? in[begin + i] : make_uint4(0, 0, 0, 0);
        const uint32_t p = valid ? pid_of<KIND>(r.x, r.y, r.z, pp) : 0u;
        const uint64_t peers = match_peers(p, __ballot(valid), pp.nbits);
        const uint32_t leader = peers ? (uint32_t)__ffsll((unsigned long long)peers) - 1 : 0u;
        if (valid && lane == leader) atomicAdd(&counts[(int64_t)p * G + g], (uint32_t)__popcll(peers));
    }
}

hipError_t launch_hist16_fallback(const void *in, int64_t n, int64_t chunk, int G, const PartParams &pp,
                                  uint32_t *counts, const uint32_t *guard, hipStream_t stream) {
    if (n <= 0 || G <= 0) return hipSuccess;
    if (pp.kind != SGX_PART_HASH || pp.chunks) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_hist16_fb<SGX_PART_HASH>, dim3(G), dim3(64), 0, stream, (const uint4 *)in, n, chunk, pp, counts,
                       G, guard);
    return hipGetLastError();
}

// The padded 16 B write's overflow fallback (launch_scatter16_fallback): one wave per chunk
// walks its records in order, 64 at a time; a record's rank among the wave's records of its
// partition comes from ballot matching, the stream's cursor from one global atomic per
// partition present.  Slow (a global round trip per 64 records) and only ever run when a
// sub-bin overflowed.
template <int KIND>
__global__ __launch_bounds__(64) void k_scatter16_fb(const uint4 *__restrict__ in, uint4 *__restrict__ out, int64_t n,
                                                     int64_t chunk, PartParams pp, const uint32_t *__restrict__ foff,
                                                     uint32_t *cur, int G, const uint32_t *guard, uint32_t *err) {
    if (!(*guard & PAD_OVERFLOW)) return;
    const int g = blockIdx.x;
    const uint32_t lane = threadIdx.x, R = pp.R;
    for (uint32_t p = lane; p < R; p += 64)
        __hip_atomic_store(&cur[(int64_t)p * G + g], foff[(int64_t)p * G + g], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    __syncthreads();
    const int64_t begin = (int64_t)g * chunk;
    const uint4 *cin = in + begin;
    int64_t len = min(n, begin + chunk) - begin;
    if (pp.chunks) {
        cin = (const uint4 *)((const char *)in + pp.chunks[2 * g]);
        len = pp.chunks[2 * g + 1];
    }
    bool bad = false;
    for (int64_t i0 = 0; i0 < len; i0 += 64) {
        const int64_t i = i0 + lane;
        const bool valid = i < len;
        const uint4 r = valid ? cin[i] : make_uint4(0, 0, 0, 0);
        const uint32_t p = valid ? pid_of<KIND>(r.x, r.y, r.z, pp) : 0u;
        const uint64_t peers = match_peers(p, __ballot(valid), pp.nbits);
        const uint32_t leader = peers ? (uint32_t)__ffsll((unsigned long long)peers) - 1 : 0u;
        uint32_t b = 0;
        if (valid && lane == leader) b = atomicAdd(&cur[(int64_t)p * G + g], (uint32_t)__popcll(peers));
        b = __shfl(b, (int)leader, 64);
        const uint64_t pos = (uint64_t)b + (uint64_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (valid) {
            if (pos < (uint64_t)n) out[pos] = r;
            else bad = true;
        }
    }
    if (bad) atomicOr(err, ERR_SCATTER_OOB);
}

// The same for 100 B TeraSort records under their RangePartitioner: a record's lane copies its
// 25 dwords (the bounds searched in global memory).
template <int KIND>
__global__ __launch_bounds__(64) void k_scatter_wide_fb(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                        int64_t n, int64_t chunk, PartParams pp,
                                                        const uint32_t *__restrict__ foff, uint32_t *cur, int G,
                                                        const uint32_t *guard, uint32_t *err) {
    constexpr int DW = 25;
    if (!(*guard & PAD_OVERFLOW)) return;
    const int g = blockIdx.x;
    const uint32_t lane = threadIdx.x, R = pp.R;
    for (uint32_t p = lane; p < R; p += 64)
        __hip_atomic_store(&cur[(int64_t)p * G + g], foff[(int64_t)p * G + g], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    __syncthreads();
    const int64_t begin = (int64_t)g * chunk;
    const uint32_t *cin = in + begin * DW;
    int64_t len = min(n, begin + chunk) - begin;
    if (pp.chunks) {
        cin = (const uint32_t *)((const char *)in + pp.chunks[2 * g]);
        len = pp.chunks[2 * g + 1];
    }
    bool bad = false;
    for (int64_t i0 = 0; i0 < len; i0 += 64) {
        const int64_t i = i0 + lane;
        const bool valid = i < len;
        const uint32_t *r = cin + (valid ? i : 0) * DW;
        const uint32_t p = valid ? pid_of<KIND>(r[0], r[1], r[2], pp) : 0u;
        const uint64_t peers = match_peers(p, __ballot(valid), pp.nbits);
        const uint32_t leader = peers ? (uint32_t)__ffsll((unsigned long long)peers) - 1 : 0u;
        uint32_t b = 0;
        if (valid && lane == leader) b = atomicAdd(&cur[(int64_t)p * G + g], (uint32_t)__popcll(peers));
        b = __shfl(b, (int)leader, 64);
        const uint64_t pos = (uint64_t)b + (uint64_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (valid) {
            if (pos < (uint64_t)n)
                for (int d = 0; d < DW; ++d) out[pos * DW + d] = r[d];
            else
                bad = true;
        }
    }
    if (bad) atomicOr(err, ERR_SCATTER_OOB);
}

hipError_t launch_scatter16_fallback(const void *in, void *out, int64_t n, int64_t chunk, int G, const PartParams &pp,
                                     const uint32_t *foff, uint32_t *cur, const uint32_t *guard, uint32_t *err,
                                     hipStream_t stream, int rb) {
    if (n <= 0 || G <= 0) return hipSuccess;
    if (rb == 16 && pp.kind == SGX_PART_HASH)
        hipLaunchKernelGGL(k_scatter16_fb<SGX_PART_HASH>, dim3(G), dim3(64), 0, stream, (const uint4 *)in, (uint4 *)out,
                           n, chunk, pp, foff, cur, G, guard, err);
    else if (rb == 100 && pp.kind == SGX_PART_RANGE_BYTES10)
        hipLaunchKernelGGL(k_scatter_wide_fb<SGX_PART_RANGE_BYTES10>, dim3(G), dim3(64), 0, stream,
                           (const uint32_t *)in, (uint32_t *)out, n, chunk, pp, foff, cur, G, guard, err);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

constexpr int PAD_CAPS_THREADS = 1024;

constexpr int PAD_CAPS_PER = 4;  // partitions per thread: R <= 4096

__global__ __launch_bounds__(PAD_CAPS_THREADS) void k_pad_caps(const uint32_t *__restrict__ est, int R, double scale,
                                                               double a, int G, uint32_t olim,
                                                               uint32_t *__restrict__ pcap,
                                                               uint32_t *__restrict__ fstart, uint32_t *err_pad) {
    __shared__ uint64_t s_x[PAD_CAPS_THREADS];
    __shared__ uint32_t s_cap[PAD_CAPS_THREADS * PAD_CAPS_PER];
    __shared__ uint64_t s_base[PAD_CAPS_THREADS * PAD_CAPS_PER];
    const int tid = (int)threadIdx.x;
    uint32_t cap[PAD_CAPS_PER];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < PAD_CAPS_PER; ++k) {
        const int p = tid * PAD_CAPS_PER + k;
        cap[k] = 0;
        if (p < R) cap[k] = pad_cap_of(est[p], scale, a);
        s_cap[tid * PAD_CAPS_PER + k] = cap[k];
        sum += SGX_PAD_CHUNK_MAJOR ? (uint64_t)cap[k] : (uint64_t)cap[k] * (uint64_t)G;
    }
    s_x[tid] = sum;
    __syncthreads();
    // inclusive scan of the per-thread sums (Hillis-Steele, 64-bit: a total above olim is
    // detected, not wrapped)
    for (int d = 1; d < PAD_CAPS_THREADS; d <<= 1) {
        const uint64_t y = tid >= d ? s_x[tid - d] : 0ull;
        __syncthreads();
        s_x[tid] += y;
        __syncthreads();
    }
    uint64_t run = s_x[tid] - sum;
#pragma unroll
    for (int k = 0; k < PAD_CAPS_PER; ++k) {
        s_base[tid * PAD_CAPS_PER + k] = run;
        run += SGX_PAD_CHUNK_MAJOR ? (uint64_t)cap[k] : (uint64_t)cap[k] * (uint64_t)G;
    }
    __syncthreads();
    if (blockIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < PAD_CAPS_PER; ++k)
            if (tid * PAD_CAPS_PER + k < R) pcap[tid * PAD_CAPS_PER + k] = cap[k];
        const uint64_t whole = SGX_PAD_CHUNK_MAJOR ? s_x[PAD_CAPS_THREADS - 1] * (uint64_t)G : s_x[PAD_CAPS_THREADS - 1];
        if (tid == 0 && whole > (uint64_t)olim) atomicOr(err_pad, PAD_OVERFLOW);
    }
    // this workgroup's partitions [p0, p1): fstart[p*G + g] (coalesced) -- chunk-major
    // (pad_layout_starts): g * total + base[p]; partition-major: base[p] + g * cap[p]
    const uint64_t total = s_x[PAD_CAPS_THREADS - 1];
    const int per = (R + (int)gridDim.x - 1) / (int)gridDim.x;
    const int p0 = min(R, (int)blockIdx.x * per), p1 = min(R, p0 + per);
    for (int64_t i = (int64_t)p0 * G + tid; i < (int64_t)p1 * G; i += PAD_CAPS_THREADS) {
        const int p = (int)(i / G), g = (int)(i - (int64_t)p * G);
        const uint64_t base = s_base[p];
        const uint64_t at = SGX_PAD_CHUNK_MAJOR ? (uint64_t)g * total + base : base + (uint64_t)g * s_cap[p];
        fstart[i] = (uint32_t)min<uint64_t>(at, (uint64_t)olim);
    }
}

hipError_t launch_pad_caps(const uint32_t *est, int R, int64_t sampled, int64_t chunk, int G, uint32_t olim,
                           uint32_t *pcap, uint32_t *fstart, uint32_t *err_pad, hipStream_t stream) {
    if (R < 1 || R > PAD_CAPS_THREADS * PAD_CAPS_PER || sampled < 1 || G < 1) return hipErrorInvalidValue;
    const double scale = (double)chunk / (double)sampled, a = 1.0 + scale;
    const int grid = min(R, 64);
    hipLaunchKernelGGL(k_pad_caps, dim3(grid), dim3(PAD_CAPS_THREADS), 0, stream, est, R, scale, a, G, olim, pcap,
                       fstart, err_pad);
    return hipGetLastError();
}

int64_t pad_capacity_bound(int64_t n, int R, int64_t chunk, int G, int64_t sampled) {
    if (n <= 0 || sampled < 1) return -1;
    // cap[p] <= mu[p] + k sqrt(a mu[p] + 16) + 16, sum mu = chunk, and by Cauchy-Schwarz
    // sum sqrt(a mu + 16) <= sqrt(R (a chunk + 16 R))
    const double a = 1.0 + (double)chunk / (double)sampled;
    const double per = (double)chunk + PAD_SIGMAS * sqrt((double)R * (a * (double)chunk + 16.0 * R)) + 16.0 * R;
    const double total = (double)G * per + 1024.0;
    if (total >= 4294967040.0) return -1;
    return (int64_t)total;
}

constexpr int FRAG_THREADS = 256;

// Copy `bytes` from s to d by one workgroup: 16 B units when both ends and the size are
// 16 B-aligned, else dwords (fixed-width records are whole dwords).
__device__ __forceinline__ void frag_copy(const char *s, char *d, uint64_t bytes, uint32_t tid) {
    if ((((uintptr_t)s | (uintptr_t)d | bytes) & 15) == 0) {
        const uint4 *s4 = (const uint4 *)s;
        uint4 *d4 = (uint4 *)d;
        const uint64_t c = bytes >> 4;
        uint64_t k = tid;
        for (; k + 3 * FRAG_THREADS < c; k += 4 * FRAG_THREADS) {
            const uint4 v0 = s4[k], v1 = s4[k + FRAG_THREADS], v2 = s4[k + 2 * FRAG_THREADS],
                        v3 = s4[k + 3 * FRAG_THREADS];
            d4[k] = v0;
            d4[k + FRAG_THREADS] = v1;
            d4[k + 2 * FRAG_THREADS] = v2;
            d4[k + 3 * FRAG_THREADS] = v3;
        }
        for (; k < c; k += FRAG_THREADS) d4[k] = s4[k];
    } else {
        const uint32_t *s1 = (const uint32_t *)s;
        uint32_t *d1 = (uint32_t *)d;
        const uint64_t c = bytes >> 2;
        uint64_t k = tid;
        for (; k + 3 * FRAG_THREADS < c; k += 4 * FRAG_THREADS) {
            const uint32_t v0 = s1[k], v1 = s1[k + FRAG_THREADS], v2 = s1[k + 2 * FRAG_THREADS],
                           v3 = s1[k + 3 * FRAG_THREADS];
            d1[k] = v0;
            d1[k + FRAG_THREADS] = v1;
            d1[k + 2 * FRAG_THREADS] = v2;
            d1[k + 3 * FRAG_THREADS] = v3;
        }
        for (; k < c; k += FRAG_THREADS) d1[k] = s1[k];
    }
}

__global__ __launch_bounds__(FRAG_THREADS) void k_gather_frags(const int64_t *__restrict__ desc, int64_t nblocks) {
    const uint32_t g = blockIdx.x, tid = threadIdx.x;
    for (int64_t b = blockIdx.y; b < nblocks; b += gridDim.y) {
        const int64_t *d = desc + FRAG_DESC_WORDS * b;
        const uint32_t p = (uint32_t)d[5], G = (uint32_t)d[6];
        const uint64_t rb = (uint64_t)d[7];
        if (g >= G) continue;
        const uint32_t *fstart = (const uint32_t *)(uintptr_t)d[1];
        const uint32_t *foff = (const uint32_t *)(uintptr_t)d[2];
        const uint32_t *cnt = (const uint32_t *)(uintptr_t)d[3];
        const int64_t i = (int64_t)p * G + g;
        frag_copy((const char *)(uintptr_t)d[0] + (uint64_t)fstart[i] * rb,
                  (char *)(uintptr_t)d[4] + (uint64_t)(foff[i] - foff[(int64_t)p * G]) * rb, (uint64_t)cnt[i] * rb, tid);
    }
}

// Cross-GPU visibility of the peer gather.  A peer's receive buffer is ordinary
// device memory mapped over xGMI, so the gather's stores may sit dirty in this GPU's L2s, and the
// owner's L2s may hold lines of the buffer from an earlier round.  k_l2_release writes back every
// XCD's L2 (a system-scope release) behind the gather, before the round's barrier;
// k_l2_acquire drops every XCD's non-coherent lines (a system-scope acquire) behind the barrier,
// before any read of the round.  Workgroups are dispatched round-robin over the XCDs: 64 of
// them reach all eight.
__global__ __launch_bounds__(64) void k_l2_release(uint32_t *sink) {
    __threadfence_system();
    __builtin_amdgcn_s_waitcnt(0);  // the write-back has completed before the wave ends
    if (sink && threadIdx.x == 0 && blockIdx.x == 0) sink[0] = 0u;
}
__global__ __launch_bounds__(64) void k_l2_acquire(uint32_t *sink) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (sink && threadIdx.x == 0 && blockIdx.x == 0) sink[0] = 0u;
}

hipError_t launch_l2_fence(bool release, hipStream_t stream) {
    if (release)
        hipLaunchKernelGGL(k_l2_release, dim3(64), dim3(64), 0, stream, (uint32_t *)nullptr);
    else
        hipLaunchKernelGGL(k_l2_acquire, dim3(64), dim3(64), 0, stream, (uint32_t *)nullptr);
    return hipGetLastError();
}

hipError_t launch_gather_frags(const int64_t *desc, int64_t nblocks, int G, hipStream_t stream, int max_rows) {
    if (nblocks <= 0 || G <= 0) return hipSuccess;
    const int64_t rows = max_rows < 1 ? 1 : max_rows > 65535 ? 65535 : max_rows;
    const dim3 grid((unsigned)G, (unsigned)(nblocks < rows ? nblocks : rows));
    hipLaunchKernelGGL(k_gather_frags, grid, dim3(FRAG_THREADS), 0, stream, desc, nblocks);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// A streaming map committed in one pass (sgx_map_commit, deferred batches) and framed by
// UnsafeShuffleWriter's fast merge: every (partition p, spill b) segment's first record in the
// contiguous output = the pass's offset of stream (p, the batch's first chunk g0[b]) -- the
// batch's chunks follow each other in every partition -- or, past the last chunk, the
// partition's end.  out[R*S] = the record count.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_spill_seg_offs(const uint32_t *__restrict__ offs,
                                                         const uint32_t *__restrict__ part_off, int R, int G, int S,
                                                         const int32_t *__restrict__ g0, uint32_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nseg = (int64_t)R * S;
    if (i > nseg) return;
    if (i == nseg) {
        out[i] = part_off[R];
        return;
    }
    const int p = (int)(i / S), b = (int)(i - (int64_t)p * S);
    const int g = g0[b];
    out[i] = g < G ? offs[(int64_t)p * G + g] : part_off[p + 1];
}

hipError_t launch_spill_seg_offs(const uint32_t *offs, const uint32_t *part_off, int R, int G, int S,
                                 const int32_t *g0, uint32_t *out, hipStream_t stream) {
    const int64_t m = (int64_t)R * S + 1;
    hipLaunchKernelGGL(k_spill_seg_offs, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream, offs, part_off, R, G,
                       S, g0, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// Synthetic input generators (same definitions as oracle/shuffle_oracle.c).
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_gen_uniform16(uint4 *dst, int64_t n, uint64_t seed, int64_t vbase) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = splitmix64_at(seed, (uint64_t)i);
        const uint64_t v = (uint64_t)(vbase + i);
        dst[i] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), (uint32_t)v, (uint32_t)(v >> 32));
    }
}

__global__ void k_gen_zipf16(uint4 *dst, int64_t n, uint64_t seed, int64_t vbase,
                             const double *__restrict__ cdf, int64_t K) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double u = (double)(splitmix64_at(seed, (uint64_t)i) >> 11) * 0x1.0p-53;
        int64_t lo = 0, hi = K - 1;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (cdf[mid] > u) hi = mid; else lo = mid + 1;
        }
        const uint64_t k = (uint64_t)(lo + 1), v = (uint64_t)(vbase + i);
        dst[i] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), (uint32_t)v, (uint32_t)(v >> 32));
    }
}

__global__ void k_gen_terasort100(uint32_t *dst, int64_t n, uint64_t seed, int64_t ibase) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t a = splitmix64_at(seed, 2 * (uint64_t)i);
        const uint64_t b = splitmix64_at(seed, 2 * (uint64_t)i + 1);
        const uint64_t idx = (uint64_t)(ibase + i);
        uint8_t bytes[100];
        for (int j = 0; j < 8; ++j) bytes[j] = (uint8_t)(a >> (8 * j));
        bytes[8] = (uint8_t)b;
        bytes[9] = (uint8_t)(b >> 8);
        for (int j = 0; j < 8; ++j) bytes[10 + j] = (uint8_t)(idx >> (8 * j));
        for (int j = 18; j < 100; ++j) bytes[j] = (uint8_t)(idx + (uint64_t)j);
        uint32_t *d = dst + 25 * i;
        for (int q = 0; q < 25; ++q)
            d[q] = (uint32_t)bytes[4 * q] | ((uint32_t)bytes[4 * q + 1] << 8) |
                   ((uint32_t)bytes[4 * q + 2] << 16) | ((uint32_t)bytes[4 * q + 3] << 24);
    }
}

static dim3 gen_grid(int64_t n) {
    int64_t b = (n + 255) / 256;
    if (b > 65536) b = 65536;
    if (b < 1) b = 1;
    return dim3((unsigned)b);
}

hipError_t launch_gen_uniform16(void *dst, int64_t n, uint64_t seed, int64_t vbase, hipStream_t s) {
    hipLaunchKernelGGL(k_gen_uniform16, gen_grid(n), dim3(256), 0, s, (uint4 *)dst, n, seed, vbase);
    return hipGetLastError();
}
hipError_t launch_gen_zipf16(void *dst, int64_t n, uint64_t seed, int64_t vbase, const double *cdf,
                             int64_t K, hipStream_t s) {
    hipLaunchKernelGGL(k_gen_zipf16, gen_grid(n), dim3(256), 0, s, (uint4 *)dst, n, seed, vbase, cdf, K);
    return hipGetLastError();
}
hipError_t launch_gen_terasort100(void *dst, int64_t n, uint64_t seed, int64_t ibase, hipStream_t s) {
    hipLaunchKernelGGL(k_gen_terasort100, gen_grid(n), dim3(256), 0, s, (uint32_t *)dst, n, seed, ibase);
    return hipGetLastError();
}

}  // namespace sgx
