// sgx_plan.cpp — pure-host exchange planning (no HIP): the send / receive counts of the
// all-to-all that replaces the per-block UCX fetches (ucx/UcxWorkerWrapper.scala:96-186) and
// the regroup copy list of the canonical per-reducer order (SURVEY §8(a) parity note).
// Compiled into libsgx.so and, on its own, into the sanitizer build of the CPU suite.
#include <cstddef>
#include <vector>

#include "../../include/sgx.h"
#include "sgx_host.h"

extern "C" int32_t sgx_reducer_owner(int32_t r, int32_t R, int32_t P) {
    if (R < 1 || P < 1 || r < 0 || r >= R) return -1;
    return sgx::reducer_owner(r, R, P);
}

extern "C" int sgx_even_ranges(int32_t P, int32_t R, int32_t *bounds) {
    if (P < 1 || R < 0 || !bounds) return sgx::fail_msg(SGX_ERR_INVALID, "sgx_even_ranges: bad arguments");
    for (int32_t j = 0; j < P; ++j) {
        int32_t r0, r1;
        sgx::my_reducers(R, P, j, &r0, &r1);
        bounds[j] = r0;
    }
    bounds[P] = R;
    return SGX_OK;
}

// Linear partition of the per-reducer totals T[r] = sum_j L[j][r] into P contiguous ranges
// minimising the largest range total: the smallest X for which greedy left-to-right cuts
// (close a range before it would pass X) need at most P ranges, found by binary search;
// then the same greedy cuts at that X.  O(R log sum).
extern "C" int sgx_balanced_ranges(const int64_t *L, int32_t P, int32_t R, int32_t *bounds) {
    if (!L || P < 1 || R < 1 || !bounds) return sgx::fail_msg(SGX_ERR_INVALID, "sgx_balanced_ranges: bad arguments");
    std::vector<int64_t> T((size_t)R, 0);
    int64_t total = 0, big = 0;
    for (int32_t j = 0; j < P; ++j)
        for (int32_t r = 0; r < R; ++r) {
            const int64_t v = L[(int64_t)j * R + r];
            if (v < 0) return sgx::fail_msg(SGX_ERR_INVALID, "sgx_balanced_ranges: negative length");
            T[(size_t)r] += v;
        }
    for (int32_t r = 0; r < R; ++r) {
        total += T[(size_t)r];
        big = T[(size_t)r] > big ? T[(size_t)r] : big;
    }
    if (total == 0) return sgx_even_ranges(P, R, bounds);
    auto ranges_at = [&](int64_t X, int32_t *b) {  // greedy cuts; returns the number of ranges
        int32_t k = 0;
        int64_t acc = 0;
        if (b) b[0] = 0;
        for (int32_t r = 0; r < R; ++r) {
            if (acc > 0 && acc + T[(size_t)r] > X) {
                ++k;
                if (b && k < P) b[k] = r;
                acc = 0;
            }
            acc += T[(size_t)r];
        }
        return k + 1;
    };
    int64_t lo = big, hi = total;  // ranges_at(hi) == 1 <= P
    while (lo < hi) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (ranges_at(mid, nullptr) <= P) hi = mid;
        else lo = mid + 1;
    }
    const int32_t k = ranges_at(lo, bounds);
    for (int32_t j = k; j <= P; ++j) bounds[j] = R;  // ranks past the last cut hold nothing
    return SGX_OK;
}

extern "C" int sgx_plan_exchange(const int64_t *L, int32_t P, int32_t R, int32_t rank, int64_t item_bytes,
                                 int64_t *send_counts, int64_t *send_displs, int64_t *recv_counts,
                                 int64_t *recv_displs, int64_t *items, int64_t *n_items) {
    if (P < 1 || R < 1) return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange: bad arguments");
    std::vector<int32_t> b((size_t)P + 1);
    sgx_even_ranges(P, R, b.data());
    return sgx_plan_exchange_ranges(L, P, R, rank, b.data(), item_bytes, send_counts, send_displs, recv_counts,
                                    recv_displs, items, n_items);
}

extern "C" int sgx_plan_exchange_ranges(const int64_t *L, int32_t P, int32_t R, int32_t rank, const int32_t *bounds,
                                        int64_t item_bytes, int64_t *send_counts, int64_t *send_displs,
                                        int64_t *recv_counts, int64_t *recv_displs, int64_t *items,
                                        int64_t *n_items) {
    if (!L || P < 1 || R < 1 || rank < 0 || rank >= P || !bounds || !send_counts || !send_displs || !recv_counts ||
        !recv_displs || !n_items || *n_items < 0 || item_bytes < 0)
        return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange: bad arguments");
    if (bounds[0] != 0 || bounds[P] != R)
        return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange: ranges must cover [0, %d)", R);
    for (int32_t j = 0; j < P; ++j)
        if (bounds[j] > bounds[j + 1])
            return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange: ranges out of order at rank %d", j);
    const int64_t *mine = L + (int64_t)rank * R;
    for (int32_t j = 0; j < P; ++j) {
        send_counts[j] = 0;
        for (int32_t r = bounds[j]; r < bounds[j + 1]; ++r) {
            if (mine[r] < 0) return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange: negative length at %d", r);
            send_counts[j] += mine[r];
        }
    }
    int64_t run = 0;
    for (int32_t j = 0; j < P; ++j) {
        send_displs[j] = run;
        run += send_counts[j];
    }
    const int32_t r0 = bounds[rank], r1 = bounds[rank + 1];
    run = 0;
    for (int32_t sidx = 0; sidx < P; ++sidx) {
        int64_t c = 0;
        for (int32_t r = r0; r < r1; ++r) {
            const int64_t v = L[(int64_t)sidx * R + r];
            if (v < 0) return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange: negative length of rank %d", sidx);
            c += v;
        }
        recv_counts[sidx] = c;
        recv_displs[sidx] = run;
        run += c;
    }
    const int64_t cap = *n_items;
    int64_t cnt = 0, dst = 0;
    std::vector<int64_t> src_run(recv_displs, recv_displs + P);
    for (int32_t r = r0; r < r1; ++r) {
        for (int32_t sidx = 0; sidx < P; ++sidx) {
            int64_t len = L[(int64_t)sidx * R + r];
            int64_t so = src_run[(size_t)sidx];
            src_run[(size_t)sidx] += len;
            while (len > 0) {
                const int64_t piece = (item_bytes > 0 && len > item_bytes) ? item_bytes : len;
                if (items && cnt < cap) {
                    items[3 * cnt] = so;
                    items[3 * cnt + 1] = dst;
                    items[3 * cnt + 2] = piece;
                }
                ++cnt;
                so += piece;
                dst += piece;
                len -= piece;
            }
        }
    }
    *n_items = cnt;
    if (items && cnt > cap)
        return sgx::fail_msg(SGX_ERR_INVALID, "item capacity %lld < %lld", (long long)cap, (long long)cnt);
    return SGX_OK;
}

// The per-shuffle exchange (sgx_exchange / sgx_exchange_maps): rank j contributes
// maps_per_rank[j] maps, lengths [M][R] source-rank-major.  This rank's send to rank d is its
// maps' bytes of d's reducers, map after map (packed [d][my map] at send_displs); what it
// receives from rank j is j's maps' bytes of my reducers, map after map, at recv_displs[j];
// block_off[M][nmine] is where block (map m, my reducer r) lands in the receive buffer.
extern "C" int sgx_plan_exchange_maps(const int64_t *L, const int64_t *maps_per_rank, int32_t P, int32_t R,
                                      int32_t rank, const int32_t *bounds, int64_t *send_counts,
                                      int64_t *send_displs, int64_t *recv_counts, int64_t *recv_displs,
                                      int64_t *block_off) {
    if (!maps_per_rank || P < 1 || R < 1 || rank < 0 || rank >= P || !bounds || !send_counts || !send_displs ||
        !recv_counts || !recv_displs)
        return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange_maps: bad arguments");
    if (bounds[0] != 0 || bounds[P] != R)
        return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange_maps: ranges must cover [0, %d)", R);
    for (int32_t j = 0; j < P; ++j)
        if (bounds[j] > bounds[j + 1])
            return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange_maps: ranges out of order at rank %d", j);
    std::vector<int64_t> first((size_t)P + 1, 0);  // index of rank j's first map
    for (int32_t j = 0; j < P; ++j) {
        if (maps_per_rank[j] < 0) return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange_maps: negative map count");
        first[(size_t)j + 1] = first[(size_t)j] + maps_per_rank[j];
    }
    const int64_t M = first[(size_t)P];
    if (M > 0 && !L) return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange_maps: lengths are NULL");
    for (int64_t i = 0; i < M * R; ++i)
        if (L[i] < 0) return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange_maps: negative length");
    int64_t run = 0;
    for (int32_t d = 0; d < P; ++d) {
        int64_t c = 0;
        for (int64_t m = first[(size_t)rank]; m < first[(size_t)rank + 1]; ++m)
            for (int32_t r = bounds[d]; r < bounds[d + 1]; ++r) c += L[m * R + r];
        send_counts[d] = c;
        send_displs[d] = run;
        run += c;
    }
    const int32_t r0 = bounds[rank], r1 = bounds[rank + 1], nmine = r1 - r0;
    run = 0;
    for (int32_t j = 0; j < P; ++j) {
        recv_displs[j] = run;
        for (int64_t m = first[(size_t)j]; m < first[(size_t)j + 1]; ++m)
            for (int32_t r = r0; r < r1; ++r) {
                if (block_off) block_off[m * nmine + (r - r0)] = run;
                run += L[m * R + r];
            }
        recv_counts[j] = run - recv_displs[j];
    }
    return SGX_OK;
}
