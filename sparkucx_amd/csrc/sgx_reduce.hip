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

constexpr int RT = 256;  // threads per workgroup

// groupByKey / reduceByKey(_ + _) over the key-sorted records in ONE pass (k_group_fused):
// a tile of GTILE records is read once, coalesced; each thread walks a contiguous run of GI of
// them (keys -- and values for SUM -- staged in LDS), flags key changes, and the tile's
// offset comes from a decoupled look-back over the tiles in ticket order.  The scanned value
// is a segmented sum: (groups started, sum of the group still open at the end, any start),
// combined left to right as (c1 + c2, f2 ? s2 : s1 + s2, f1 | f2), so a group's Long sum is
// complete when the next group starts, wherever its records lie.
//   keys[g], starts[g] = key and first record of group g (starts may be NULL);
//   GROUP: vals[i] = value of record i (groups are contiguous runs, arrival order kept);
//   SUM:   vals[g] = wrapping 64-bit sum of group g's values;
//   *ngroups = number of groups (written by the thread holding the last record).
// Replaces four passes (flags, a scan, emit, and for SUM three prefix-sum kernels plus a
// gather): one read of the records and the outputs' writes.
// ------------------------------------------------------------------------------------
#ifndef SGX_GROUP_GT  // (A/B builds: -DSGX_GROUP_GT / -DSGX_GROUP_GI)
#define SGX_GROUP_GT 256
#endif
#ifndef SGX_GROUP_GI
#define SGX_GROUP_GI 16
#endif
constexpr int GT = SGX_GROUP_GT, GI = SGX_GROUP_GI, GTILE = GT * GI;
// the group outputs (keys, starts, values: the caller's arrays, read after the call) stored
// nontemporal (A/B: -DSGX_GROUP_NT=0)
#ifndef SGX_GROUP_NT
#define SGX_GROUP_NT 1
#endif
__device__ __forceinline__ void gst(int64_t *p, int64_t v) {
    if (SGX_GROUP_NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
// LDS slot of tile record j: one pad element per GI, so a thread's contiguous run (stride
// GI + 1 elements between lanes) does not put every lane on the same banks
__device__ __forceinline__ int gslot(int j) { return j + j / GI; }
struct Seg {
    uint64_t c, s;
    uint32_t f;
};
__device__ __forceinline__ Seg seg_combine(const Seg &l, const Seg &r) {
    return Seg{l.c + r.c, r.f ? r.s : l.s + r.s, l.f | r.f};
}
__device__ __forceinline__ Seg seg_shfl_up(const Seg &x, int d) {
    return Seg{__shfl_up(x.c, d, 64), __shfl_up(x.s, d, 64), (uint32_t)__shfl_up((int)x.f, d, 64)};
}

// A tile's published value, (count, sum, start) with count < 2^31, in two 64-bit words that
// each carry the publication's kind (AGG: the tile alone, PRE: inclusive of every earlier
// tile), written with relaxed atomics: a reader takes the pair only when both words show the
// same kind, so no fence is needed (agent-scope release / acquire flush and invalidate the
// non-coherent L2s on this chip, per tile).
//   w1 = kind << 62 | start << 61 | count << 30 | sum[0, 30)      w2 = kind << 62 | sum[30, 64)
constexpr uint64_t GS_AGG = 1, GS_PRE = 2;
__device__ __forceinline__ uint64_t gs_w1(uint64_t kind, const Seg &q) {
    return kind << 62 | (uint64_t)(q.f ? 1u : 0u) << 61 | (q.c & 0x7FFFFFFFull) << 30 | (q.s & 0x3FFFFFFFull);
}
__device__ __forceinline__ uint64_t gs_w2(uint64_t kind, const Seg &q) { return kind << 62 | q.s >> 30; }
__device__ __forceinline__ Seg gs_value(uint64_t w1, uint64_t w2) {
    return Seg{(w1 >> 30) & 0x7FFFFFFFull, (w1 & 0x3FFFFFFFull) | (w2 & 0x3FFFFFFFFull) << 30, (uint32_t)(w1 >> 61) & 1u};
}


template <bool SUM>
__global__ __launch_bounds__(GT) void k_group_fused(const ulonglong2 *__restrict__ rec, int64_t n,
                                                    uint64_t *st1, uint64_t *st2,
                                                    uint32_t *ticket, uint32_t *err, int64_t *__restrict__ keys,
                                                    int64_t *__restrict__ starts, int64_t *__restrict__ vals,
                                                    int64_t *__restrict__ ngroups) {
    __shared__ uint64_t s_key[GTILE + GTILE / GI];                // then the tile's group keys
    __shared__ uint64_t s_val[SUM ? GTILE + GTILE / GI : 1];      // then the tile's closed group sums
    __shared__ uint16_t s_st[GTILE];                              // the tile's group starts (tile offsets)
    __shared__ uint64_t s_wc[GT / 64], s_ws[GT / 64];
    __shared__ uint32_t s_wf[GT / 64];
    __shared__ uint64_t s_tc, s_ts, s_prev;
    __shared__ uint32_t s_tf, s_tile;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(ticket, 1u);  // tiles in dispatch order: the look-back always progresses
    __syncthreads();
    const uint32_t tile = s_tile;
    const int64_t t0 = (int64_t)tile * GTILE;
#pragma unroll
    for (int k = 0; k < GI; ++k) {
        const int64_t i = t0 + k * GT + tid;
        if (i < n) {
            const ulonglong2 r = rec[i];
            s_key[gslot(k * GT + tid)] = r.x;
            if constexpr (SUM) s_val[gslot(k * GT + tid)] = r.y;
            else gst(vals + i, (int64_t)r.y);
        }
    }
    if (tid == 0) s_prev = t0 > 0 ? rec[t0 - 1].x : 0ull;
    __syncthreads();
    // this thread's run [t0 + tid*GI, +GI): group starts and the segmented sum
    const int64_t i0 = t0 + (int64_t)tid * GI;
    uint64_t prev = tid == 0 ? s_prev : s_key[gslot(tid * GI - 1)];
    uint32_t fm = 0;
    Seg a{0, 0, 0};
    uint64_t kreg[GI], vreg[SUM ? GI : 1];
#pragma unroll
    for (int k = 0; k < GI; ++k) {
        const int64_t i = i0 + k;
        kreg[k] = s_key[gslot(tid * GI + k)];
        if constexpr (SUM) vreg[k] = s_val[gslot(tid * GI + k)];
        if (i < n) {
            const uint64_t key = kreg[k];
            if (i == 0 || key != prev) {
                fm |= 1u << k;
                a.c += 1;
                a.s = 0;
                a.f = 1;
            }
            prev = key;
            if constexpr (SUM) a.s += vreg[k];
        }
    }
    // inclusive scan over the workgroup's threads, then the tile's exclusive prefix
    Seg x = a;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const Seg y = seg_shfl_up(x, d);
        if (lane >= (uint32_t)d) x = seg_combine(y, x);
    }
    if (lane == 63) {
        s_wc[w] = x.c;
        s_ws[w] = x.s;
        s_wf[w] = x.f;
    }
    __syncthreads();
    Seg wex{0, 0, 0}, tagg{0, 0, 0};
#pragma unroll
    for (uint32_t v = 0; v < GT / 64; ++v) {
        const Seg sv{s_wc[v], s_ws[v], s_wf[v]};
        if (v < w) wex = seg_combine(wex, sv);
        tagg = seg_combine(tagg, sv);
    }
    Seg up = seg_shfl_up(x, 1);
    if (lane == 0) up = Seg{0, 0, 0};
    const Seg tex_thread = seg_combine(wex, up);
    // decoupled look-back by wave 0, 64 predecessors per step: lane l reads tile t-1-l; the
    // window is combined oldest-first up to the nearest inclusive prefix (PRE), else whole
    if (w == 0) {
        auto publish = [&](uint64_t kind, const Seg &q) {
            __hip_atomic_store(&st1[tile], gs_w1(kind, q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&st2[tile], gs_w2(kind, q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        };
        Seg tex{0, 0, 0};
        if (tile == 0) {
            if (lane == 0) publish(GS_PRE, tagg);
        } else {
            if (lane == 0) publish(GS_AGG, tagg);
            int64_t top = (int64_t)tile - 1;  // the window's newest tile
            uint32_t spins = 0;
            while (top >= 0) {
                const int64_t j = top - (int64_t)lane;
                uint64_t w1 = 0, w2 = 0;
                if (j >= 0) {
                    w1 = __hip_atomic_load(&st1[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    w2 = __hip_atomic_load(&st2[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                const uint64_t kind = (w1 >> 62) == (w2 >> 62) ? w1 >> 62 : 0;  // 0: not (fully) published
                const uint64_t ready = __ballot(kind != 0 || j < 0), pre = __ballot(kind == GS_PRE);
                const uint64_t need = pre ? (pre & (0ull - pre)) * 2 - 1 : ~0ull;  // lanes up to the nearest PRE
                if ((ready & need) != need) {
                    if (++spins > (1u << 24)) {
                        if (lane == 0) atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                Seg x = j >= 0 && ((need >> lane) & 1ull) ? gs_value(w1, w2) : Seg{0, 0, 0};
                // oldest (highest lane) first: lane 0 ends with the window's combination
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const Seg y{__shfl_down(x.c, d, 64), __shfl_down(x.s, d, 64), (uint32_t)__shfl_down((int)x.f, d, 64)};
                    if (lane + d < 64) x = seg_combine(y, x);
                }
                x = Seg{__shfl(x.c, 0, 64), __shfl(x.s, 0, 64), (uint32_t)__shfl((int)x.f, 0, 64)};
                tex = seg_combine(x, tex);
                if (pre) break;
                top -= 64;
            }
            if (lane == 0) publish(GS_PRE, seg_combine(tex, tagg));
        }
        if (lane == 0) {
            s_tc = tex.c;
            s_ts = tex.s;
            s_tf = tex.f;
        }
    }
    __syncthreads();
    const Seg ex = seg_combine(Seg{s_tc, s_ts, s_tf}, tex_thread);
    // emit: group g = ex.c + starts seen so far; a start closes group g - 1 with its sum.  The
    // tile's groups are [gt0, gt0 + tagg.c): staged in LDS (s_key / s_val are free: every
    // thread read its keys and values before the scan's barrier), then written coalesced
    const uint64_t gt0 = s_tc;
    uint64_t *s_gkey = s_key, *s_gsum = s_val;
    uint64_t g = ex.c, run = ex.s;
#pragma unroll
    for (int k = 0; k < GI; ++k) {
        const int64_t i = i0 + k;
        if (i < n) {
            if ((fm >> k) & 1u) {
                const uint32_t q = (uint32_t)(g - gt0);
                if constexpr (SUM) {
                    if (q > 0) s_gsum[q - 1] = run;
                    else if (g > 0) vals[g - 1] = (int64_t)run;  // the group open at the tile's start
                }
                s_gkey[q] = kreg[k];
                s_st[q] = (uint16_t)(tid * GI + k);
                ++g;
                run = 0;
            }
            if constexpr (SUM) run += vreg[k];
            if (i == n - 1) {
                if constexpr (SUM) vals[g - 1] = (int64_t)run;
                *ngroups = (int64_t)g;
            }
        }
    }
    __syncthreads();
    const uint32_t ngt = (uint32_t)tagg.c;
    for (uint32_t q = tid; q < ngt; q += GT) {
        gst(keys + gt0 + q, (int64_t)s_gkey[q]);
        if (starts) gst(starts + gt0 + q, t0 + (int64_t)s_st[q]);
        if constexpr (SUM)
            if (q + 1 < ngt) gst(vals + gt0 + q, (int64_t)s_gsum[q]);  // (the tile's last group is still open)
    }
}

int64_t group_tiles(int64_t n) { return (n + GTILE - 1) / GTILE; }

hipError_t launch_group_fused(const void *rec, int64_t n, bool sum, uint64_t *status, uint32_t *ticket, uint32_t *err,
                              int64_t *keys, int64_t *starts, int64_t *vals, int64_t *ngroups, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const int64_t tiles = group_tiles(n);
    uint64_t *st2 = status + tiles;
    if (sum)
        hipLaunchKernelGGL(k_group_fused<true>, dim3((unsigned)tiles), dim3(GT), 0, st, (const ulonglong2 *)rec, n,
                           status, st2, ticket, err, keys, starts, vals, ngroups);
    else
        hipLaunchKernelGGL(k_group_fused<false>, dim3((unsigned)tiles), dim3(GT), 0, st, (const ulonglong2 *)rec, n,
                           status, st2, ticket, err, keys, starts, vals, ngroups);
    return hipGetLastError();
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
        const uint64_t act = __ballot(1);
#pragma unroll
        for (int d = 0; d < ND; ++d) {
            uint32_t b = (w[d >> 2] >> ((d & 3) * 8)) & 0xFFu;
            if (RB == 16 && d == 7) b ^= 0x80u;
            // a byte the whole wave shares (the high bytes of small keys: Zipf ranks < 2^24 leave
            // five of eight constant) is one atomic of the wave's count, not 64 on one counter
            const uint32_t b0 = __builtin_amdgcn_readfirstlane(b);
            if (__ballot(b == b0) == act) {
                if ((uint64_t)__lane_id() == (uint64_t)(__ffsll((unsigned long long)act) - 1))
                    atomicAdd(&h[d * 256 + b0], (uint32_t)__popcll(act));
            } else {
                atomicAdd(&h[d * 256 + b], 1u);
            }
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
