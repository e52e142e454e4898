// sgx_exchange.cpp — the reduce-side exchange that replaces the per-block UCX Active Message
// fetch path (ucx/UcxWorkerWrapper.scala:96-186, spark_3_0/UcxShuffleClient.scala:17-47):
// every rank pushes one map output to the reducer owners with ONE all-to-all (reducer r lives
// on rank floor(r*P/R), so the partition-contiguous map output is already grouped by
// destination), after a counts all-gather that tells every receiver the (map, reducer) block
// sizes.  Two collective backends behind the same code:
//   * RCCL (sgx_comm_init): ncclAllGather + ncclAllToAllv over xGMI on the engine's exchange
//     stream, asynchronous; waits poll ncclCommGetAsyncError and give up after the engine's
//     timeout (the reference spins forever, UcxShuffleClient.scala:44-46);
//   * host (sgx_comm_init_host): the caller's all-gather / all-to-all over host memory --
//     the fake backend of SURVEY §4, and the path for ranks sharing one GPU.
#include "sgx_engine.h"

#include <chrono>
#include <cstring>
#include <thread>

using namespace sgx;

extern "C" int sgx_get_unique_id(uint8_t out_id[128]) {
    if (!out_id) return fail_msg(SGX_ERR_INVALID, "NULL id");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(out_id, id.internal, 128);
    return SGX_OK;
}

extern "C" int sgx_comm_init(sgx_engine *e, int32_t nranks, int32_t rank, const uint8_t id[128]) {
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail_msg(SGX_ERR_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(e->comm_mu);
    if (e->comm || e->host_comm) return fail_msg(SGX_ERR_STATE, "communicator already initialised");
    HIP_TRY(hipSetDevice(e->device));
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, 128);
    NCCL_TRY(ncclCommInitRank(&e->comm, nranks, uid, rank));
    e->nranks = nranks;
    e->rank = rank;
    return SGX_OK;
}

extern "C" int sgx_comm_init_host(sgx_engine *e, int32_t nranks, int32_t rank, const sgx_host_comm *hc) {
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e || !hc || !hc->allgather || !hc->alltoallv || nranks < 1 || rank < 0 || rank >= nranks)
        return fail_msg(SGX_ERR_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(e->comm_mu);
    if (e->comm || e->host_comm) return fail_msg(SGX_ERR_STATE, "communicator already initialised");
    e->hc = *hc;
    e->host_comm = true;
    e->nranks = nranks;
    e->rank = rank;
    return SGX_OK;
}

extern "C" int sgx_comm_size(sgx_engine *e, int32_t *nranks, int32_t *rank) {
    if (!e || !nranks || !rank) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    *nranks = e->nranks;
    *rank = e->rank;
    return SGX_OK;
}

// Caller holds comm_mu.  Waits for everything on the exchange stream.  With RCCL the wait
// polls the communicator's asynchronous error and is bounded by comm_timeout_ms: a peer that
// died or stopped calling aborts the communicator (ncclCommAbort) and the call fails, so the
// executor's task fails and Spark can retry it -- instead of the reference's endless progress
// spin (UcxShuffleClient.scala:44-46, UcxWorkerWrapper.scala:320).
int sgx::comm_wait(sgx_engine *e) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (;;) {
        const hipError_t q = hipStreamQuery(e->s_comm);
        if (q == hipSuccess) return SGX_OK;
        if (q != hipErrorNotReady) return fail_msg(SGX_ERR_HIP, "exchange stream: %s", hipGetErrorString(q));
        if (e->comm) {
            ncclResult_t ar = ncclSuccess;
            if (ncclCommGetAsyncError(e->comm, &ar) == ncclSuccess && ar != ncclSuccess && ar != ncclInProgress) {
                (void)ncclCommAbort(e->comm);
                e->comm = nullptr;
                e->comm_broken = true;
                return fail_msg(SGX_ERR_COMM, "RCCL asynchronous error: %s (communicator aborted)",
                                ncclGetErrorString(ar));
            }
        }
        const auto waited = std::chrono::duration_cast<std::chrono::milliseconds>(clk::now() - t0).count();
        if (waited > e->comm_timeout_ms) {
            if (e->comm) {
                (void)ncclCommAbort(e->comm);
                e->comm = nullptr;
                e->comm_broken = true;
            }
            return fail_msg(SGX_ERR_TIMEOUT, "exchange did not complete within %lld ms (communicator aborted)",
                            (long long)e->comm_timeout_ms);
        }
        // spin (yielding) through the first 2 ms -- the common wait, one collective -- then
        // back off, so a long or stuck exchange does not burn a core
        if (waited < 2) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

extern "C" int sgx_exchange(sgx_engine *e, int32_t shuffle_id, int64_t map_id) {
    sgx::TraceRange trace_("sgx_exchange");
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    std::shared_ptr<Shuffle> s;
    std::shared_ptr<MapOut> m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    std::lock_guard<std::mutex> clk(e->comm_mu);
    std::vector<int64_t> mylens;
    int64_t out_bytes = 0;
    {
        std::lock_guard<std::mutex> lk(m->mu);
        if (m->open) return fail_msg(SGX_ERR_STATE, "map %lld is still open", (long long)map_id);
        SGX_TRY(finish_lengths(e, *c, *s, *m));
        mylens = m->lengths;
        out_bytes = m->out_bytes;
    }
    const int32_t P = e->nranks, R = s->R;
    auto rd = std::make_shared<Round>();
    rd->map_ids.assign((size_t)P, 0);
    rd->lens.assign((size_t)P * R, 0);
    my_reducers(R, P, e->rank, &rd->r0, &rd->r1);  // the collective path re-places after the all-gather
    if (e->comm_broken) return fail_msg(SGX_ERR_STATE, "the communicator was aborted after an exchange failure");
    if (P == 1 && !e->comm && !e->host_comm) {
        rd->map_ids[0] = map_id;
        std::memcpy(rd->lens.data(), mylens.data(), sizeof(int64_t) * (size_t)R);
        rd->block_off.assign((size_t)R, 0);
        int64_t off = 0;
        for (int32_t r = 0; r < R; ++r) {
            rd->block_off[(size_t)r] = off;
            off += mylens[(size_t)r];
        }
        rd->alias = m;
        HIP_TRY(rd->done.record(c->st));
        std::lock_guard<std::mutex> sl(s->mu);
        for (auto it = s->rounds.begin(); it != s->rounds.end(); ++it)
            if ((*it)->map_ids == rd->map_ids) {
                s->rounds.erase(it);
                break;
            }
        s->rounds.push_back(std::move(rd));
        return SGX_OK;
    }
    if (!e->comm && !e->host_comm) return fail_msg(SGX_ERR_STATE, "sgx_comm_init was not called (world of %d ranks)", P);
    hipStream_t st = e->s_comm;
    // (1) counts exchange: all-gather {map_id, lengths[R]}
    const size_t row = (size_t)R + 1;
    SGX_TRY(e->ag_host.ensure(row * 8 * (size_t)(P + 1)));
    int64_t *agh = (int64_t *)e->ag_host.p;
    agh[0] = map_id;
    std::memcpy(agh + 1, mylens.data(), sizeof(int64_t) * (size_t)R);
    hipEvent_t a0 = e->ev(), a1 = e->ev(), a2 = e->ev(), a3 = e->ev();
    if (e->comm) {
        SGX_TRY(e->ag_send.ensure(row * 8));
        SGX_TRY(e->ag_recv.ensure(row * 8 * (size_t)P));
        HIP_TRY(hipEventRecord(a0, st));
        HIP_TRY(hipMemcpyAsync(e->ag_send.p, agh, row * 8, hipMemcpyHostToDevice, st));
        NCCL_TRY(ncclAllGather(e->ag_send.p, e->ag_recv.p, row, ncclInt64, e->comm, st));
        HIP_TRY(hipMemcpyAsync(agh + row, e->ag_recv.p, row * 8 * (size_t)P, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipEventRecord(a1, st));
        SGX_TRY(comm_wait(e));  // also drains the previous round's all-to-all (one stream, one order)
    } else {
        SGX_TRY(comm_wait(e));
        HIP_TRY(hipEventRecord(a0, st));
        if (e->hc.allgather(e->hc.user, agh, (int64_t)(row * 8), agh + row) != 0)
            return fail_msg(SGX_ERR_COMM, "host all-gather of the partition lengths failed");
        HIP_TRY(hipEventRecord(a1, st));
    }
    for (int32_t j = 0; j < P; ++j) {
        rd->map_ids[(size_t)j] = agh[row * (size_t)(j + 1)];
        std::memcpy(&rd->lens[(size_t)j * R], agh + row * (size_t)(j + 1) + 1, sizeof(int64_t) * (size_t)R);
    }
    // (2) placement (the same on every rank: it depends on the all-gathered lengths only) and
    //     plan: send/recv counts and displacements (no copy list: blocks stay where they land)
    std::vector<int32_t> bounds((size_t)P + 1);
    if (s->placement.load() == SGX_PLACE_BYTES)
        SGX_TRY(sgx_balanced_ranges(rd->lens.data(), P, R, bounds.data()));
    else
        SGX_TRY(sgx_even_ranges(P, R, bounds.data()));
    rd->r0 = bounds[(size_t)e->rank];
    rd->r1 = bounds[(size_t)e->rank + 1];
    const int32_t nmine = rd->r1 - rd->r0;
    std::vector<int64_t> sc(P), sd(P), rc(P), rdp(P);
    int64_t nitems = 0;
    SGX_TRY(sgx_plan_exchange_ranges(rd->lens.data(), P, R, e->rank, bounds.data(), 0, sc.data(), sd.data(), rc.data(),
                                     rdp.data(), nullptr, &nitems));
    if (sd[(size_t)P - 1] + sc[(size_t)P - 1] != out_bytes)
        return fail_msg(SGX_ERR_HIP, "internal error: send plan covers %lld of %lld bytes",
                        (long long)(sd[(size_t)P - 1] + sc[(size_t)P - 1]), (long long)out_bytes);
    int64_t total_recv = 0;
    for (int32_t j = 0; j < P; ++j) total_recv += rc[(size_t)j];
    rd->block_off.assign((size_t)P * nmine, 0);
    for (int32_t j = 0; j < P; ++j) {
        int64_t off = rdp[(size_t)j];
        for (int32_t r = rd->r0; r < rd->r1; ++r) {
            rd->block_off[(size_t)j * nmine + (size_t)(r - rd->r0)] = off;
            off += rd->lens[(size_t)j * R + r];
        }
    }
    // A round with the same source maps replaces the previous one (a re-attempt): reuse
    // its HBM when nobody else still reads it.
    {
        std::lock_guard<std::mutex> sl(s->mu);
        for (auto it = s->rounds.begin(); it != s->rounds.end(); ++it) {
            if ((*it)->map_ids == rd->map_ids) {
                if (it->use_count() == 1) {
                    HIP_TRY((*it)->done.wait_host());
                    rd->data.swap((*it)->data);
                }
                s->rounds.erase(it);
                break;
            }
        }
    }
    // (3) all-to-all of the partition-contiguous map output (already destination-grouped):
    //     no pack step before, no regroup after
    SGX_TRY(rd->data.ensure((size_t)total_recv));
    HIP_TRY(hipStreamWaitEvent(st, m->done.ev, 0));
    const void *view = m->view();
    if (e->comm) {
        std::vector<size_t> scz(P), sdz(P), rcz(P), rdz(P);
        for (int32_t j = 0; j < P; ++j) {
            scz[(size_t)j] = (size_t)sc[(size_t)j];
            sdz[(size_t)j] = (size_t)sd[(size_t)j];
            rcz[(size_t)j] = (size_t)rc[(size_t)j];
            rdz[(size_t)j] = (size_t)rdp[(size_t)j];
        }
        HIP_TRY(hipEventRecord(a2, st));
        NCCL_TRY(ncclAllToAllv(view, scz.data(), sdz.data(), rd->data.p, rcz.data(), rdz.data(), ncclUint8, e->comm, st));
        HIP_TRY(hipEventRecord(a3, st));
    } else {
        // host backend: stage the map output out, exchange on the host, stage the blocks in
        SGX_TRY(e->x_send.ensure((size_t)std::max<int64_t>(out_bytes, 16)));
        SGX_TRY(e->x_recv.ensure((size_t)std::max<int64_t>(total_recv, 16)));
        HIP_TRY(hipEventRecord(a2, st));
        if (out_bytes > 0) HIP_TRY(hipMemcpyAsync(e->x_send.p, view, (size_t)out_bytes, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (e->hc.alltoallv(e->hc.user, e->x_send.p, sc.data(), sd.data(), e->x_recv.p, rc.data(), rdp.data()) != 0)
            return fail_msg(SGX_ERR_COMM, "host all-to-all of the map output failed");
        if (total_recv > 0)
            HIP_TRY(hipMemcpyAsync(rd->data.p, e->x_recv.p, (size_t)total_recv, hipMemcpyHostToDevice, st));
        HIP_TRY(hipEventRecord(a3, st));
        HIP_TRY(hipStreamSynchronize(st));  // the pinned staging buffers are reused next round
    }
    HIP_TRY(rd->done.record(st));
    HIP_TRY(m->read_done.record(st));
    e->record_stage(SGX_STAGE_ALLGATHER, a0, a1);
    e->record_stage(SGX_STAGE_ALLTOALL, a2, a3);
    std::lock_guard<std::mutex> sl(s->mu);
    s->rounds.push_back(std::move(rd));
    return SGX_OK;
}

extern "C" int sgx_copy_items(sgx_engine *e, const void *src, void *dst, const int64_t *items, int64_t n_items,
                              int32_t align) {
    if (!e || n_items < 0 || (n_items > 0 && (!items || !src || !dst)) || (align != 4 && align != 16))
        return fail_msg(SGX_ERR_INVALID, "sgx_copy_items: bad arguments");
    for (int64_t i = 0; i < n_items; ++i)
        if (items[3 * i] % align || items[3 * i + 1] % align || items[3 * i + 2] % align || items[3 * i + 2] < 0)
            return fail_msg(SGX_ERR_INVALID, "sgx_copy_items: item %lld not %d-byte aligned", (long long)i, align);
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    if (n_items == 0) return SGX_OK;
    SGX_TRY(c->items_dev.ensure((size_t)n_items * 24));
    HIP_TRY(hipMemcpyAsync(c->items_dev.p, items, (size_t)n_items * 24, hipMemcpyHostToDevice, c->st));
    HIP_TRY(launch_copy_items(src, dst, (const int64_t *)c->items_dev.p, n_items, align, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SGX_OK;
}

extern "C" int sgx_round_reducers(sgx_engine *e, int32_t shuffle_id, int64_t map_id, int32_t *r0, int32_t *r1) {
    if (!e || !r0 || !r1) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    std::lock_guard<std::mutex> sl(s->mu);
    for (auto it = s->rounds.rbegin(); it != s->rounds.rend(); ++it)
        for (int64_t m : (*it)->map_ids)
            if (m == map_id) {
                *r0 = (*it)->r0;
                *r1 = (*it)->r1;
                return SGX_OK;
            }
    return fail_msg(SGX_ERR_NOT_FOUND, "no exchange round of shuffle %d carried map %lld", shuffle_id,
                    (long long)map_id);
}
