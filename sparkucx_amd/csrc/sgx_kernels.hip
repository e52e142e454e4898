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

// ------------------------------------------------------------------------------------
// Partition ids
// ------------------------------------------------------------------------------------

// Lemire fastmod (exact for every 32-bit u and divisor d >= 1).
__device__ __forceinline__ uint32_t fastmod_u32(uint32_t u, uint64_t M, uint32_t d) {
    const uint64_t low = M * (uint64_t)u;
    return (uint32_t)__umul64hi(low, (uint64_t)d);
}

// nonNegativeMod((int)(k ^ (k >>> 32)), R) with k = khi:klo.
// h (signed) mod R == ((h + 2^31) mod R - 2^31 mod R) mod R, evaluated unsigned.
__device__ __forceinline__ uint32_t hash_pid(uint32_t klo, uint32_t khi, const PartParams &pp) {
    const uint32_t u = (klo ^ khi) ^ 0x80000000u;
    const uint32_t r = fastmod_u32(u, pp.fm_M, pp.R);
    const uint32_t t = r + pp.R - pp.c31;
    return t >= pp.R ? t - pp.R : t;
}

__device__ __forceinline__ uint32_t range_pid_i64(int64_t key, const PartParams &pp) {
    const int64_t *b = (const int64_t *)pp.bounds;
    const int nb = pp.nb;
    int p = 0;
    if (nb <= 128) {
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
    return (uint32_t)(pp.ascending ? p : nb - p);
}

__device__ __forceinline__ bool k10_lt(uint64_t ahi, uint32_t alo, uint64_t bhi, uint32_t blo) {
    return ahi < bhi || (ahi == bhi && alo < blo);
}

__device__ __forceinline__ uint32_t range_pid_k10(uint64_t khi, uint32_t klo, const PartParams &pp) {
    const Key10 *b = (const Key10 *)pp.bounds;
    const int nb = pp.nb;
    int p = 0;
    if (nb <= 128) {
        while (p < nb && k10_lt(b[p].hi, b[p].lo, khi, klo)) ++p;
    } else {
        int low = 0, high = nb - 1;
        bool found = false;
        while (low <= high) {
            const int mid = (int)(((unsigned)low + (unsigned)high) >> 1);
            const Key10 mv = b[mid];
            if (k10_lt(mv.hi, mv.lo, khi, klo)) low = mid + 1;
            else if (k10_lt(khi, klo, mv.hi, mv.lo)) high = mid - 1;
            else { p = mid; found = true; break; }
        }
        if (!found) p = low;
        if (p > nb) p = nb;
    }
    return (uint32_t)(pp.ascending ? p : nb - p);
}

// Partition id from the first 12 bytes of a record (x, y, z little-endian dwords).
template <int KIND>
__device__ __forceinline__ uint32_t pid_of(uint32_t x, uint32_t y, uint32_t z, const PartParams &pp) {
    if constexpr (KIND == SGX_PART_HASH) {
        return hash_pid(x, y, pp);
    } else if constexpr (KIND == SGX_PART_RANGE_I64) {
        return range_pid_i64((int64_t)(((uint64_t)y << 32) | x), pp);
    } else {
        const uint64_t hi = ((uint64_t)__builtin_bswap32(x) << 32) | __builtin_bswap32(y);
        const uint32_t lo = __builtin_bswap32(z) >> 16;
        return range_pid_k10(hi, lo, pp);
    }
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
__device__ void block_exclusive_scan(const uint32_t *in, uint32_t *out, uint32_t R,
                                     uint32_t *scratch) {
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
        out[i] = run;
        run += c;
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------
// K1+K2: partition ids + per-chunk histogram
// ------------------------------------------------------------------------------------
constexpr int HIST_THREADS = 512;
constexpr int HIST_UNROLL = 8;

template <int KIND, bool REC16>
__global__ __launch_bounds__(HIST_THREADS) void k_hist(const char *__restrict__ in, int64_t n,
                                                       int rb, int64_t chunk, PartParams pp,
                                                       uint32_t *__restrict__ counts, int G) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint32_t *hist = (uint32_t *)smem;
    const uint32_t tid = threadIdx.x, T = blockDim.x;
    for (uint32_t p = tid; p < pp.R; p += T) hist[p] = 0;
    __syncthreads();
    const int g = blockIdx.x;
    const int64_t begin = (int64_t)g * chunk;
    const int64_t end = min(n, begin + chunk);
    for (int64_t base = begin; base < end; base += (int64_t)T * HIST_UNROLL) {
        uint32_t x[HIST_UNROLL], y[HIST_UNROLL], z[HIST_UNROLL];
#pragma unroll
        for (int u = 0; u < HIST_UNROLL; ++u) {
            const int64_t i = base + (int64_t)u * T + tid;
            x[u] = y[u] = z[u] = 0;
            if (i < end) {
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
        for (int u = 0; u < HIST_UNROLL; ++u) {
            const int64_t i = base + (int64_t)u * T + tid;
            if (i < end) atomicAdd(&hist[pid_of<KIND>(x[u], y[u], z[u], pp)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t p = tid; p < pp.R; p += T) counts[(int64_t)p * G + g] = hist[p];
}

hipError_t launch_hist(const void *in, int64_t n, int rb, int64_t chunk, int G,
                       const PartParams &pp, uint32_t *counts, hipStream_t stream) {
    const size_t lds = (size_t)pp.R * 4;
    const char *p = (const char *)in;
    const bool r16 = (rb == 16);
#define SGX_HIST(K, B) \
    hipLaunchKernelGGL((k_hist<K, B>), dim3(G), dim3(HIST_THREADS), lds, stream, p, n, rb, chunk, pp, counts, G)
    switch (pp.kind) {
    case SGX_PART_HASH: if (r16) SGX_HIST(SGX_PART_HASH, true); else SGX_HIST(SGX_PART_HASH, false); break;
    case SGX_PART_RANGE_I64: if (r16) SGX_HIST(SGX_PART_RANGE_I64, true); else SGX_HIST(SGX_PART_RANGE_I64, false); break;
    default: if (r16) SGX_HIST(SGX_PART_RANGE_BYTES10, true); else SGX_HIST(SGX_PART_RANGE_BYTES10, false); break;
    }
#undef SGX_HIST
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

__global__ __launch_bounds__(SCAN_THREADS) void k_scan(const uint32_t *__restrict__ in,
                                                       uint32_t *__restrict__ out, int64_t len,
                                                       uint64_t *status, uint32_t *ticket_err,
                                                       uint32_t *__restrict__ part_off, int G,
                                                       int R) {
    __shared__ uint32_t s_tile, s_prefix_lo;
    __shared__ uint32_t s_wsum[SCAN_THREADS / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(&ticket_err[0], 1u);
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
                    if (++spins > (1u << 26)) { atomicOr(&ticket_err[1], 1u); break; }
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
                       uint32_t *ticket_err, uint32_t *part_off, int G, int R, hipStream_t stream) {
    const int64_t tiles = scan_tiles(len);
    hipLaunchKernelGGL(k_scan, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, stream, counts, offs,
                       len, status, ticket_err, part_off, G, R);
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
constexpr int SC_WAVES = 8;
constexpr int SC_THREADS = SC_WAVES * 64;
constexpr size_t LDS_MAX = 160 * 1024;

static size_t scatter_lds16(uint32_t R, int tile) {
    return (size_t)tile * 16 + (size_t)SC_WAVES * R * 2 + (size_t)3 * R * 4 + 64;
}

ScatterGeom scatter_geom16(uint32_t R) {
    static const int cand[] = {16, 12, 8, 6, 4, 3, 2, 1};
    for (int items : cand) {
        const int tile = SC_WAVES * items * 64;
        const size_t lds = scatter_lds16(R, tile);
        if (lds <= LDS_MAX) return ScatterGeom{SC_WAVES, items, tile, lds};
    }
    return ScatterGeom{SC_WAVES, 0, 0, 0};
}

static size_t scatter_lds_wide(uint32_t R) {
    return (size_t)SC_WAVES * R * 2 + (size_t)2 * R * 4 + 64;
}

ScatterGeom scatter_geom_wide(uint32_t R, int /*rb*/) {
    const size_t lds = scatter_lds_wide(R);
    if (lds > LDS_MAX) return ScatterGeom{SC_WAVES, 0, 0, 0};
    return ScatterGeom{SC_WAVES, 4, SC_WAVES * 4 * 64, lds};
}

// Slot -> partition for the drain: the last p with lstart[p] <= s (empty partitions
// before p share p's start, every later partition starts after s).
__device__ __forceinline__ uint32_t slot_partition(const uint32_t *lstart, uint32_t R, uint32_t s) {
    uint32_t lo = 0, hi = R - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (lstart[mid] <= s) lo = mid; else hi = mid - 1;
    }
    return lo;
}

template <int ITEMS>
__device__ __forceinline__ void rank_items(const uint32_t (&pid)[ITEMS], const bool (&valid)[ITEMS],
                                           uint32_t (&rank)[ITEMS], uint16_t *mycnt, uint32_t nbits,
                                           uint32_t lane) {
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const uint64_t vm = __ballot(valid[k]);
        const uint32_t p = pid[k];
        const uint64_t peers = match_peers(p, vm, nbits);
        const uint64_t below = peers & lt;
        uint32_t base = 0;
        if (valid[k]) base = mycnt[p];
        rank[k] = base + (uint32_t)__popcll(below);
        if (valid[k] && below == 0) mycnt[p] = (uint16_t)(base + (uint32_t)__popcll(peers));
    }
}

template <int KIND, int ITEMS>
__global__ __launch_bounds__(SC_THREADS, 1) void k_scatter16(const uint4 *__restrict__ in,
                                                             uint4 *__restrict__ out, int64_t n,
                                                             int64_t chunk, PartParams pp,
                                                             const uint32_t *__restrict__ offs,
                                                             int G) {
    constexpr int TILE = SC_WAVES * ITEMS * 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t R = pp.R;
    uint4 *stage = (uint4 *)smem;
    uint16_t *wcnt = (uint16_t *)(smem + (size_t)TILE * 16);
    uint32_t *lstart = (uint32_t *)(smem + (size_t)TILE * 16 + (((size_t)SC_WAVES * R * 2 + 15) & ~(size_t)15));
    uint32_t *cursor = lstart + R;
    uint32_t *tcnt = cursor + R;
    uint32_t *scratch = tcnt + R;

    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int g = blockIdx.x;
    const int64_t begin = (int64_t)g * chunk;
    const int64_t end = min(n, begin + chunk);
    for (uint32_t p = tid; p < R; p += SC_THREADS) cursor[p] = offs[(int64_t)p * G + g];

    for (int64_t tbase = begin; tbase < end; tbase += TILE) {
        for (uint32_t i = tid; i < SC_WAVES * R / 2; i += SC_THREADS) ((uint32_t *)wcnt)[i] = 0;
        // load this wave's sub-tile (coalesced: 1 KiB per wave-instruction)
        uint4 rec[ITEMS];
        uint32_t pid[ITEMS], rank[ITEMS];
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
        rank_items<ITEMS>(pid, valid, rank, wcnt + (size_t)w * R, pp.nbits, lane);
        __syncthreads();
        for (uint32_t p = tid; p < R; p += SC_THREADS) {
            uint32_t s = 0;
#pragma unroll
            for (int v = 0; v < SC_WAVES; ++v) {
                const uint32_t c = wcnt[(size_t)v * R + p];
                wcnt[(size_t)v * R + p] = (uint16_t)s;
                s += c;
            }
            tcnt[p] = s;
        }
        __syncthreads();
        block_exclusive_scan(tcnt, lstart, R, scratch);
        const uint16_t *mycnt = wcnt + (size_t)w * R;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            if (valid[k]) {
                const uint32_t p = pid[k];
                stage[lstart[p] + mycnt[p] + rank[k]] = rec[k];
            }
        }
        __syncthreads();
        const uint32_t tile_n = (uint32_t)min<int64_t>(TILE, end - tbase);
        for (uint32_t s = tid; s < tile_n; s += SC_THREADS) {
            const uint4 r = stage[s];
            uint32_t p;
            if constexpr (KIND == SGX_PART_HASH) p = hash_pid(r.x, r.y, pp);
            else p = slot_partition(lstart, R, s);
            out[(size_t)(cursor[p] + (s - lstart[p]))] = r;
        }
        __syncthreads();
        for (uint32_t p = tid; p < R; p += SC_THREADS) cursor[p] += tcnt[p];
    }
}

// Wide records (record_bytes multiple of 4, e.g. TeraSort's 100 B): same ranking, each
// lane then copies its record straight to its destination.
template <int KIND, int ITEMS>
__global__ __launch_bounds__(SC_THREADS, 1) void k_scatter_wide(const char *__restrict__ in,
                                                                char *__restrict__ out, int64_t n,
                                                                int rb, int64_t chunk,
                                                                PartParams pp,
                                                                const uint32_t *__restrict__ offs,
                                                                int G) {
    constexpr int TILE = SC_WAVES * ITEMS * 64;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const uint32_t R = pp.R;
    uint16_t *wcnt = (uint16_t *)smem;
    uint32_t *cursor = (uint32_t *)(smem + (((size_t)SC_WAVES * R * 2 + 15) & ~(size_t)15));
    uint32_t *tcnt = cursor + R;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int g = blockIdx.x;
    const int64_t begin = (int64_t)g * chunk;
    const int64_t end = min(n, begin + chunk);
    const int dw = rb >> 2;
    for (uint32_t p = tid; p < R; p += SC_THREADS) cursor[p] = offs[(int64_t)p * G + g];

    for (int64_t tbase = begin; tbase < end; tbase += TILE) {
        for (uint32_t i = tid; i < SC_WAVES * R / 2; i += SC_THREADS) ((uint32_t *)wcnt)[i] = 0;
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
        rank_items<ITEMS>(pid, valid, rank, wcnt + (size_t)w * R, pp.nbits, lane);
        __syncthreads();
        for (uint32_t p = tid; p < R; p += SC_THREADS) {
            uint32_t s = 0;
#pragma unroll
            for (int v = 0; v < SC_WAVES; ++v) {
                const uint32_t c = wcnt[(size_t)v * R + p];
                wcnt[(size_t)v * R + p] = (uint16_t)s;
                s += c;
            }
            tcnt[p] = s;
        }
        __syncthreads();
        const uint16_t *mycnt = wcnt + (size_t)w * R;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            if (valid[k]) {
                const int64_t i = wbase + (int64_t)k * 64;
                const uint32_t p = pid[k];
                const uint64_t dst = (uint64_t)cursor[p] + mycnt[p] + rank[k];
                const uint32_t *s = (const uint32_t *)(in + i * rb);
                uint32_t *d = (uint32_t *)(out + dst * (uint64_t)rb);
                for (int q = 0; q < dw; ++q) d[q] = s[q];
            }
        }
        __syncthreads();
        for (uint32_t p = tid; p < R; p += SC_THREADS) cursor[p] += tcnt[p];
    }
}

hipError_t launch_scatter(const void *in, void *out, int64_t n, int rb, int64_t chunk, int G,
                          const PartParams &pp, const uint32_t *offs, hipStream_t stream) {
    if (rb == 16) {
        const ScatterGeom geo = scatter_geom16(pp.R);
        if (geo.items == 0) return hipErrorInvalidValue;
        const uint4 *i4 = (const uint4 *)in;
        uint4 *o4 = (uint4 *)out;
#define SGX_SC16(K, I)                                                                          \
    do {                                                                                        \
        (void)hipFuncSetAttribute((const void *)k_scatter16<K, I>,                             \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)geo.lds_bytes); \
        hipLaunchKernelGGL((k_scatter16<K, I>), dim3(G), dim3(SC_THREADS), geo.lds_bytes, stream,  \
                           i4, o4, n, chunk, pp, offs, G);                                     \
    } while (0)
#define SGX_SC16_K(K)                                \
    switch (geo.items) {                             \
    case 16: SGX_SC16(K, 16); break;                 \
    case 12: SGX_SC16(K, 12); break;                 \
    case 8: SGX_SC16(K, 8); break;                   \
    case 6: SGX_SC16(K, 6); break;                   \
    case 4: SGX_SC16(K, 4); break;                   \
    case 3: SGX_SC16(K, 3); break;                   \
    case 2: SGX_SC16(K, 2); break;                   \
    default: SGX_SC16(K, 1); break;                  \
    }
        switch (pp.kind) {
        case SGX_PART_HASH: SGX_SC16_K(SGX_PART_HASH); break;
        case SGX_PART_RANGE_I64: SGX_SC16_K(SGX_PART_RANGE_I64); break;
        default: SGX_SC16_K(SGX_PART_RANGE_BYTES10); break;
        }
#undef SGX_SC16_K
#undef SGX_SC16
    } else {
        const ScatterGeom geo = scatter_geom_wide(pp.R, rb);
        if (geo.items == 0 || (rb & 3) != 0 || rb < 12) return hipErrorInvalidValue;
        const char *ic = (const char *)in;
        char *oc = (char *)out;
#define SGX_SCW(K)                                                                              \
    do {                                                                                        \
        (void)hipFuncSetAttribute((const void *)k_scatter_wide<K, 4>,                          \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)geo.lds_bytes); \
        hipLaunchKernelGGL((k_scatter_wide<K, 4>), dim3(G), dim3(SC_THREADS), geo.lds_bytes,     \
                           stream, ic, oc, n, rb, chunk, pp, offs, G);                         \
    } while (0)
        switch (pp.kind) {
        case SGX_PART_HASH: SGX_SCW(SGX_PART_HASH); break;
        case SGX_PART_RANGE_I64: SGX_SCW(SGX_PART_RANGE_I64); break;
        default: SGX_SCW(SGX_PART_RANGE_BYTES10); break;
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
