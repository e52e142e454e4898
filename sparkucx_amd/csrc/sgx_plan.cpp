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

extern "C" int sgx_plan_exchange(const int64_t *L, int32_t P, int32_t R, int32_t rank, int64_t item_bytes,
                                 int64_t *send_counts, int64_t *send_displs, int64_t *recv_counts,
                                 int64_t *recv_displs, int64_t *items, int64_t *n_items) {
    if (!L || P < 1 || R < 1 || rank < 0 || rank >= P || !send_counts || !send_displs || !recv_counts ||
        !recv_displs || !n_items || *n_items < 0 || item_bytes < 0)
        return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange: bad arguments");
    const int64_t *mine = L + (int64_t)rank * R;
    for (int32_t j = 0; j < P; ++j) send_counts[j] = 0;
    for (int32_t r = 0; r < R; ++r) {
        if (mine[r] < 0) return sgx::fail_msg(SGX_ERR_INVALID, "sgx_plan_exchange: negative length at %d", r);
        send_counts[sgx::reducer_owner(r, R, P)] += mine[r];
    }
    int64_t run = 0;
    for (int32_t j = 0; j < P; ++j) {
        send_displs[j] = run;
        run += send_counts[j];
    }
    int32_t r0, r1;
    sgx::my_reducers(R, P, rank, &r0, &r1);
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
