// sgx_exchange.cpp — the reduce-side exchange that replaces the per-block UCX Active Message
// fetch path (ucx/UcxWorkerWrapper.scala:96-186, spark_3_0/UcxShuffleClient.scala:17-47):
// sgx_exchange(e, shuffle_id) is one collective per shuffle (or per batch of maps, for
// pipelining): every rank contributes the map outputs it holds -- any number, none included,
// as Spark's map tasks land on executors independently -- and afterwards every rank holds its
// reducers' blocks of every map of every rank.  Reducer r lives on one rank for the whole
// shuffle (contiguous ranges, floor(r*P/R) or byte-balanced, fixed by the shuffle's first
// round), so each partition-contiguous map output is already grouped by destination and is
// sent without a pack step.  Two collective backends behind the same code:
//   * RCCL (sgx_comm_init): ncclAllGather of the map counts and lengths, then one grouped
//     ncclSend / ncclRecv exchange over xGMI on the engine's exchange stream, asynchronous;
//     waits poll ncclCommGetAsyncError and give up after the engine's timeout (the reference
//     spins forever, UcxShuffleClient.scala:44-46);
//   * host (sgx_comm_init_host): the caller's all-gather / all-to-all over host memory --
//     the fake backend of SURVEY §4, and the path for ranks sharing one GPU.
#include "sgx_engine.h"

#include <algorithm>
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

// All-gather of int64 rows: every rank contributes `n` values, `recv` receives P * n,
// rank-major.  Caller holds comm_mu.  With RCCL the call also drains the exchange stream
// (the previous round's all-to-all: one communicator, one stream, the same order on every
// rank).
static int allgather_i64(sgx_engine *e, const int64_t *send, size_t n, int64_t *recv) {
    const int32_t P = e->nranks;
    hipStream_t st = e->s_comm;
    if (e->comm) {
        SGX_TRY(e->ag_send.ensure(n * 8));
        SGX_TRY(e->ag_recv.ensure(n * 8 * (size_t)P));
        SGX_TRY(e->ag_host.ensure(n * 8 * (size_t)(P + 1)));
        int64_t *h = (int64_t *)e->ag_host.p;
        std::memcpy(h, send, n * 8);
        HIP_TRY(hipMemcpyAsync(e->ag_send.p, h, n * 8, hipMemcpyHostToDevice, st));
        NCCL_TRY(ncclAllGather(e->ag_send.p, e->ag_recv.p, n, ncclInt64, e->comm, st));
        HIP_TRY(hipMemcpyAsync(h + n, e->ag_recv.p, n * 8 * (size_t)P, hipMemcpyDeviceToHost, st));
        SGX_TRY(comm_wait(e));
        std::memcpy(recv, h + n, n * 8 * (size_t)P);
        return SGX_OK;
    }
    SGX_TRY(comm_wait(e));
    if (e->hc.allgather(e->hc.user, send, (int64_t)(n * 8), recv) != 0)
        return fail_msg(SGX_ERR_COMM, "host all-gather of the partition lengths failed");
    return SGX_OK;
}

// A source rank holding several maps whose (map, destination) pieces average below this sends
// ONE packed piece per destination (its pieces gathered on the device first) instead of one
// RCCL send per (map, destination): Spark executors hold hundreds of map outputs per shuffle,
// and every point-to-point operation has a fixed cost.  Every rank decides it for every
// source from the all-gathered lengths, so receivers post matching receives.
static constexpr int64_t PACK_PIECE_BYTES = 4ll << 20;

static bool packs_sends(int64_t nmaps, int64_t bytes, int32_t P) {
    return nmaps > 1 && bytes < PACK_PIECE_BYTES * nmaps * (int64_t)P;
}

namespace {
struct LocalMap {
    int64_t id;
    std::shared_ptr<MapOut> m;
    std::vector<int64_t> lens;
    int64_t bytes = 0;
};
}  // namespace

// Unmap peers' receive buffers no round used in the last few (their last gather finished; all
// with `all`, after waiting).  Caller holds comm_mu.
static void p2p_release(sgx_engine *e, bool all) {
    constexpr uint64_t KEEP_ROUNDS = 4;
    for (auto it = e->p2p_cache.begin(); it != e->p2p_cache.end();) {
        sgx_engine::PeerMap &pm = it->second;
        const bool stale = all || e->p2p_rounds - pm.last_round > KEEP_ROUNDS;
        if (!stale || (!all && pm.done && hipEventQuery(pm.done) == hipErrorNotReady)) {
            ++it;
            continue;
        }
        if (pm.done) {
            (void)hipEventSynchronize(pm.done);
            (void)hipEventDestroy(pm.done);
        }
        (void)hipIpcCloseMemHandle(pm.ptr);
        it = e->p2p_cache.erase(it);
    }
}

// Direct peer gather: rank `me` writes the blocks of its maps that rank d owns
// straight into d's receive buffer, at the place d's plan gives them -- a padded map's blocks
// from their fragments (one workgroup per fragment), a contiguous map's as byte ranges -- in
// one gather launch per kind on the exchange stream.  Peers' buffers are mapped into this
// process through IPC handles all-gathered by the backend (the image's dmabuf IPC; this rank's
// own buffer directly), and a second all-gather says every rank has mapped its peers (or
// fails the round on every rank).  Completion: with RCCL a one-word ncclAllReduce on the
// exchange stream behind the gather (the round stays asynchronous; readers wait for the
// round's event), with host collectives a host barrier after the gather.  No pack step and no
// contiguous copy of a padded map: each map's published bytes leave it exactly once, sent
// bytes = the blocks' lengths.
// p2p_data's answer when some rank could not get or map a receive buffer's IPC handle: every
// rank learns it from the same all-gather before anything was written, so every rank falls
// back together (exchange_round)
constexpr int P2P_UNAVAILABLE = 1 << 20;

static int p2p_data(sgx_engine *e, Shuffle &s, Round &rd, const std::vector<LocalMap> &mine,
                    const std::vector<int32_t> &bounds, const std::vector<int64_t> &lens,
                    const std::vector<int32_t> &srcs, hipStream_t st) {
    const int32_t P = e->nranks, me = e->rank, R = s.R;
    const size_t M = srcs.size();
    ++e->p2p_rounds;
    p2p_release(e, false);
    // any rank's failure before the gather fails the round on every rank (status all-gather);
    // `refused` notes that the all-gather itself worked and some rank reported a failure
    bool refused = false;
    auto agree = [&](int rc, const std::string &msg, const int64_t *extra, size_t nextra,
                     std::vector<int64_t> *all) -> int {
        std::vector<int64_t> mine_w(nextra + 1, 0);
        mine_w[0] = rc;
        for (size_t i = 0; i < nextra; ++i) mine_w[i + 1] = extra[i];
        std::vector<int64_t> tmp((nextra + 1) * (size_t)P, 0);
        SGX_TRY(allgather_i64(e, mine_w.data(), nextra + 1, tmp.data()));
        for (int32_t j = 0; j < P; ++j)
            if (tmp[(size_t)j * (nextra + 1)] != SGX_OK) {
                refused = true;
                if (j == me) return fail_msg(rc, "%s (every rank fails this exchange)", msg.c_str());
                return fail_msg(SGX_ERR_STATE, "exchange of shuffle %d failed on rank %d: every rank fails it", s.id, j);
            }
        if (all) *all = std::move(tmp);
        return SGX_OK;
    };
    // (a) every rank's receive buffer as an IPC handle
    constexpr size_t HW = (sizeof(hipIpcMemHandle_t) + 7) / 8 + 1;  // the handle, then its serial
    std::vector<int64_t> all_h;
    int local_rc = SGX_OK;
    std::string local_msg;
    if (P > 1) {
        int64_t hw[HW] = {0};
        const hipError_t he = (e->flags & SGX_FLAG_TEST_P2P_UNAVAILABLE) ? hipErrorNotSupported
                              : rd.ipc_valid                             ? hipSuccess
                                                                         : hipIpcGetMemHandle(&rd.ipc, rd.data.p);
        if (he == hipSuccess && !rd.ipc_valid) rd.ipc_gen = ++e->p2p_gen;
        rd.ipc_valid = he == hipSuccess;
        if (he != hipSuccess) {
            local_rc = SGX_ERR_HIP;
            hipPointerAttribute_t pa{};
            const hipError_t ae = hipPointerGetAttributes(&pa, rd.data.p);
            char buf[256];
            std::snprintf(buf, sizeof buf, "hipIpcGetMemHandle(%p, %zu B): %s (pointer attributes: %s, type %d, device %d)",
                          rd.data.p, rd.data.cap, hipGetErrorString(he), hipGetErrorString(ae), (int)pa.type, pa.device);
            local_msg = buf;
        } else {
            std::memcpy(hw, &rd.ipc, sizeof(rd.ipc));
            hw[HW - 1] = (int64_t)rd.ipc_gen;
        }
        const int arc = agree(local_rc, local_msg, hw, HW, &all_h);
        if (arc != SGX_OK) return refused ? P2P_UNAVAILABLE : arc;
    }
    // (b) where my contribution starts in every rank's receive buffer: [source][its maps][d's
    //     reducers], i.e. after the blocks of d's reducers of every map of lower ranks
    std::vector<int64_t> at((size_t)P, 0), to((size_t)P, 0);
    for (int32_t d = 0; d < P; ++d) {
        int64_t o = 0;
        for (size_t m = 0; m < M && srcs[m] < me; ++m)
            for (int32_t r = bounds[(size_t)d]; r < bounds[(size_t)d + 1]; ++r) o += lens[m * R + r];
        at[(size_t)d] = o;
    }
    for (auto &lm : mine)
        for (int32_t d = 0; d < P; ++d)
            for (int32_t r = bounds[(size_t)d]; r < bounds[(size_t)d + 1]; ++r) to[(size_t)d] += lm.lens[(size_t)r];
    // (c) the destinations: mine directly, the peers' through their handles
    std::vector<void *> peer((size_t)P, nullptr);
    std::vector<sgx_engine::PeerMap *> used;
    peer[(size_t)me] = rd.data.p;
    for (int32_t d = 0; d < P && local_rc == SGX_OK; ++d) {
        if (d == me || to[(size_t)d] == 0) continue;
        hipIpcMemHandle_t h;
        const int64_t *w = &all_h[(size_t)d * (HW + 1) + 1];
        std::memcpy(&h, w, sizeof(h));
        const int64_t tag[2] = {d, w[HW - 1]};
        const std::string key = std::string((const char *)tag, sizeof(tag)) + std::string((const char *)&h, sizeof(h));
        auto it = e->p2p_cache.find(key);
        if (it == e->p2p_cache.end()) {
            void *q = nullptr;
            const hipError_t he = hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess);
            if (he != hipSuccess) {
                local_rc = SGX_ERR_HIP;
                local_msg = std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(he);
                break;
            }
            it = e->p2p_cache.emplace(key, sgx_engine::PeerMap{q, 0, nullptr}).first;
        }
        it->second.last_round = e->p2p_rounds;
        peer[(size_t)d] = it->second.ptr;
        used.push_back(&it->second);
    }
    // (d) the gathers: padded maps by fragment table (one descriptor per block), contiguous
    //     maps by byte ranges (64 KiB items)
    std::vector<int64_t> frag, items;
    int Gmax = 0;
    bool al16 = true, al4 = true;
    int64_t sent = 0, kept = 0;
    std::vector<int64_t> off_in((size_t)P, 0);  // bytes of my earlier maps' pieces to each rank
    for (size_t k = 0; k < mine.size() && local_rc == SGX_OK; ++k) {
        MapOut &m = *mine[k].m;
        const uint32_t *po = (const uint32_t *)m.part_off.p;  // record offsets (fixed codec)
        for (int32_t d = 0; d < P; ++d) {
            const int32_t b0 = bounds[(size_t)d], b1 = bounds[(size_t)d + 1];
            int64_t l = 0, o = 0;
            for (int32_t r = 0; r < b0; ++r) o += mine[k].lens[(size_t)r];
            for (int32_t r = b0; r < b1; ++r) l += mine[k].lens[(size_t)r];
            char *dst = (char *)peer[(size_t)d] + at[(size_t)d] + off_in[(size_t)d];
            off_in[(size_t)d] += l;
            (d == me ? kept : sent) += l;
            if (l == 0) continue;
            if (m.padded) {
                const int G = m.frag_G;
                Gmax = std::max(Gmax, G);
                const uint32_t *fs = (const uint32_t *)m.frag.p;
                const int64_t len = (int64_t)R * G;
                for (int32_t p = b0; p < b1; ++p) {
                    if (mine[k].lens[(size_t)p] == 0) continue;
                    frag.insert(frag.end(), {(int64_t)(uintptr_t)m.data.p, (int64_t)(uintptr_t)fs,
                                             (int64_t)(uintptr_t)(fs + len), (int64_t)(uintptr_t)(fs + 2 * len),
                                             (int64_t)(uintptr_t)(dst + (int64_t)(po[p] - po[b0]) * s.rb), p, G, s.rb});
                }
            } else {
                const char *src = (const char *)m.view() + o;
                for (int64_t done = 0; done < l; done += 65536) {
                    const int64_t b = std::min<int64_t>(65536, l - done);
                    items.insert(items.end(), {(int64_t)(uintptr_t)(src + done), (int64_t)(uintptr_t)(dst + done), b});
                    const uintptr_t u = (uintptr_t)(src + done) | (uintptr_t)(dst + done) | (uintptr_t)b;
                    al16 = al16 && (u & 15) == 0;
                    al4 = al4 && (u & 3) == 0;
                }
            }
        }
    }
    // the mappings this round writes through stay open until its gather has finished
    auto mark_used = [&]() -> int {
        for (sgx_engine::PeerMap *pm : used) {
            if (!pm->done) HIP_TRY(hipEventCreateWithFlags(&pm->done, hipEventDisableTiming));
            HIP_TRY(hipEventRecord(pm->done, st));
        }
        return SGX_OK;
    };
    if (P > 1) {  // every rank has mapped the buffers it writes to (or the round fails everywhere)
        const int arc = agree(local_rc, local_msg, nullptr, 0, nullptr);
        if (arc != SGX_OK) return refused ? P2P_UNAVAILABLE : arc;
    }
    auto launch = [&]() -> int {
        for (auto &lm : mine) HIP_TRY(hipStreamWaitEvent(st, lm.m->done.ev, 0));
        const size_t fb = frag.size() * 8, ib = items.size() * 8;
        if (fb + ib == 0) return SGX_OK;
        HIP_TRY(e->x_items_up.wait_host());  // the last round's descriptors have been uploaded
        SGX_TRY(e->x_items.ensure(fb + ib));
        SGX_TRY(e->x_items_dev.ensure(fb + ib));
        std::memcpy(e->x_items.p, frag.data(), fb);
        std::memcpy((char *)e->x_items.p + fb, items.data(), ib);
        HIP_TRY(hipMemcpyAsync(e->x_items_dev.p, e->x_items.p, fb + ib, hipMemcpyHostToDevice, st));
        HIP_TRY(e->x_items_up.record(st));
        if (!frag.empty())
            // a few workgroups per CU, each looping over blocks: the next map's sample and K4
            // share the CUs with the gather instead of queueing behind ~R x G workgroups
            HIP_TRY(launch_gather_frags((const int64_t *)e->x_items_dev.p, (int64_t)(frag.size() / FRAG_DESC_WORDS),
                                        Gmax, st, std::max(1, 4 * e->num_cus / std::max(1, Gmax))));
        if (!items.empty())
            HIP_TRY(launch_gather_items((const int64_t *)((char *)e->x_items_dev.p + fb), (int64_t)(items.size() / 3),
                                        al16 ? 16 : al4 ? 4 : 1, st));
        return debug_sync(e, st, "exchange peer gather");
    };
    int rc = launch();
    // peers' buffers are written through this GPU's L2s: write them back before the barrier
    if (rc == SGX_OK && P > 1 && sent > 0) {
        const hipError_t fe = launch_l2_fence(true, st);
        if (fe != hipSuccess) rc = fail_msg(SGX_ERR_HIP, "peer gather release: %s", hipGetErrorString(fe));
    }
    if (P > 1 && e->comm) {
        // completion barrier on the stream: a peer's allreduce runs after its gather, so once
        // this one completes every block of my reducers has landed (a rank whose launch failed
        // still joins it, then fails)
        SGX_TRY(e->p2p_word.ensure(16));
        const ncclResult_t nr = ncclAllReduce(e->p2p_word.p, (char *)e->p2p_word.p + 8, 1, ncclInt64, ncclSum,
                                              e->comm, st);
        if (nr != ncclSuccess && rc == SGX_OK)
            rc = fail_msg(SGX_ERR_COMM, "ncclAllReduce (peer gather barrier) failed: %s", ncclGetErrorString(nr));
        const int mrc = mark_used();
        if (rc != SGX_OK) return rc;
        SGX_TRY(mrc);
        // the peers' stores into my buffer are in HBM now: drop my L2s' older lines of it
        HIP_TRY(launch_l2_fence(false, st));
    } else if (P > 1) {
        // host collectives: the gather has finished on every rank once the barrier returns
        if (rc == SGX_OK) rc = comm_wait(e);
        const std::string msg = rc == SGX_OK ? std::string() : std::string(sgx_last_error());
        const int brc = agree(rc, msg, nullptr, 0, nullptr);
        if (brc != SGX_OK) return brc;
        SGX_TRY(mark_used());
        HIP_TRY(launch_l2_fence(false, st));
    } else if (rc != SGX_OK) {
        return rc;
    }
    std::lock_guard<std::mutex> lk(e->stats_mu);
    e->x_bytes[0] += sent;
    e->x_bytes[1] += kept;
    e->x_bytes[2] += 1;
    return SGX_OK;
}

// One exchange round of shuffle s with this rank's maps `mine` (any number, the same call
// order on every rank).  (1) all-gather of every rank's map count, then of {map id, R
// lengths} per map; (2) the shuffle's reducer ranges -- fixed by its first round, so every
// round sends a reducer's blocks to the same rank; (3) one grouped point-to-point exchange
// (RCCL: ncclSend / ncclRecv per (map, peer) straight out of the partition-contiguous map
// outputs, which are already destination-grouped -- no pack step -- into the receive layout
// [source rank][its maps][my reducers]; host backend: the same bytes through the caller's
// all-to-all).
// Caller holds comm_mu (taken before the maps were selected, so two concurrent exchanges of
// one shuffle cannot both carry a map).  A rank whose maps fail locally (still open, a
// failed write) still joins the first all-gather, with an error mark, so every rank fails
// the round together instead of waiting in a collective for it.
static int exchange_round(sgx_engine *e, Ctx *c, const std::shared_ptr<Shuffle> &s, std::vector<LocalMap> mine,
                          int local_rc = SGX_OK, std::string local_msg = std::string()) {
    const int32_t P = e->nranks, R = s->R;
    // the direct peer gather moves the blocks (a padded map's from its fragments); RCCL's
    // send / recv and the host all-to-all move contiguous byte ranges
    const bool p2p = (e->comm || e->host_comm) && !(e->flags & SGX_FLAG_NO_P2P_EXCHANGE) && !e->p2p_off.load();
    for (auto &lm : mine) {
        if (local_rc != SGX_OK) break;
        std::lock_guard<std::mutex> lk(lm.m->mu);
        int rc = lm.m->open ? fail_msg(SGX_ERR_STATE, "map %lld is still open", (long long)lm.id) : SGX_OK;
        if (rc == SGX_OK) rc = finish_lengths(e, *c, *s, *lm.m);
        if (rc == SGX_OK && !p2p) rc = materialize(e, *c, *s, *lm.m);
        if (rc != SGX_OK) {
            local_rc = rc;
            local_msg = sgx_last_error();
            break;
        }
        lm.lens = lm.m->lengths;
        lm.bytes = lm.m->out_bytes;
    }
    if (e->comm_broken) return fail_msg(SGX_ERR_STATE, "the communicator was aborted after an exchange failure");
    const bool collective = e->comm || e->host_comm;
    if (local_rc != SGX_OK && !collective) return fail_msg(local_rc, "%s", local_msg.c_str());
    if (P > 1 && !collective) return fail_msg(SGX_ERR_STATE, "sgx_comm_init was not called (world of %d ranks)", P);
    hipStream_t st = collective ? e->s_comm : c->st;
    hipEvent_t a0 = e->ev(), a1 = e->ev(), a2 = e->ev(), a3 = e->ev();
    if (local_rc == SGX_OK) {
        // a failing record is a local error like any other: it still joins the all-gather
        const hipError_t he = hipEventRecord(a0, st);
        if (he != hipSuccess) {
            if (!collective) return fail_msg(SGX_ERR_HIP, "hipEventRecord: %s", hipGetErrorString(he));
            local_rc = SGX_ERR_HIP;
            local_msg = std::string("hipEventRecord: ") + hipGetErrorString(he);
        }
    }
    // (1) who holds which maps, and their lengths
    std::vector<int64_t> counts((size_t)P, 0);
    std::vector<int64_t> ids, lens;  // [M], [M][R], source-rank-major
    std::vector<int32_t> srcs;
    const size_t row = (size_t)R + 1;
    if (!collective) {
        counts[0] = (int64_t)mine.size();
        for (auto &lm : mine) {
            ids.push_back(lm.id);
            srcs.push_back(0);
            lens.insert(lens.end(), lm.lens.begin(), lm.lens.end());
        }
    } else {
        // first all-gather: [map count | the first map's {id, lengths}] per rank -- the whole
        // round when every rank holds at most one map (the pipelined exchange_maps step)
        // a local failure travels as a negative map count: -1 - (the error code's magnitude)
        const int64_t nloc = local_rc != SGX_OK ? -1 + (int64_t)local_rc : (int64_t)mine.size();
        std::vector<int64_t> first(1 + row, 0), firsts((1 + row) * (size_t)P, 0);
        first[0] = nloc;
        if (nloc > 0) {
            first[1] = mine[0].id;
            std::memcpy(&first[2], mine[0].lens.data(), sizeof(int64_t) * (size_t)R);
        }
        SGX_TRY(allgather_i64(e, first.data(), first.size(), firsts.data()));
        int64_t mmax = 0;
        for (int32_t j = 0; j < P; ++j) {
            counts[(size_t)j] = firsts[(size_t)j * (1 + row)];
            if (counts[(size_t)j] < 0) {
                if (j == e->rank) return fail_msg(local_rc, "%s (every rank fails this exchange)", local_msg.c_str());
                return fail_msg(SGX_ERR_STATE, "exchange of shuffle %d failed on rank %d (code %lld): every rank fails it",
                                s->id, j, (long long)(-1 - counts[(size_t)j]));
            }
            mmax = std::max(mmax, counts[(size_t)j]);
        }
        if (mmax <= 1) {
            for (int32_t j = 0; j < P; ++j)
                if (counts[(size_t)j] == 1) {
                    const int64_t *q = &firsts[(size_t)j * (1 + row) + 1];
                    ids.push_back(q[0]);
                    srcs.push_back(j);
                    lens.insert(lens.end(), q + 1, q + 1 + R);
                }
        } else {  // second all-gather: every map's {id, lengths}, padded to the largest count
            std::vector<int64_t> send(row * (size_t)mmax, 0), recv(row * (size_t)mmax * (size_t)P, 0);
            for (size_t k = 0; k < mine.size(); ++k) {
                send[k * row] = mine[k].id;
                std::memcpy(&send[k * row + 1], mine[k].lens.data(), sizeof(int64_t) * (size_t)R);
            }
            SGX_TRY(allgather_i64(e, send.data(), send.size(), recv.data()));
            for (int32_t j = 0; j < P; ++j)
                for (int64_t k = 0; k < counts[(size_t)j]; ++k) {
                    const int64_t *q = &recv[((size_t)j * (size_t)mmax + (size_t)k) * row];
                    ids.push_back(q[0]);
                    srcs.push_back(j);
                    lens.insert(lens.end(), q + 1, q + 1 + R);
                }
        }
    }
    HIP_TRY(hipEventRecord(a1, st));
    const size_t M = ids.size();
    {
        std::vector<int64_t> sorted_ids(ids);
        std::sort(sorted_ids.begin(), sorted_ids.end());
        if (std::adjacent_find(sorted_ids.begin(), sorted_ids.end()) != sorted_ids.end())
            return fail_msg(SGX_ERR_INVALID, "an exchange round of shuffle %d carries a map id twice", s->id);
    }
    // (2) placement: the shuffle's reducer ranges, fixed by its first round (the same on
    //     every rank: it depends on the all-gathered lengths only)
    std::vector<int32_t> bounds;
    {
        std::lock_guard<std::mutex> sl(s->mu);
        bounds = s->place_bounds;
    }
    if (bounds.size() != (size_t)P + 1) {
        bounds.assign((size_t)P + 1, 0);
        if (s->placement.load() == SGX_PLACE_BYTES && M > 0) {
            std::vector<int64_t> per_rank((size_t)P * R, 0);  // [P][R]: each rank's maps summed
            for (size_t m = 0; m < M; ++m)
                for (int32_t r = 0; r < R; ++r) per_rank[(size_t)srcs[m] * R + r] += lens[m * R + r];
            SGX_TRY(sgx_balanced_ranges(per_rank.data(), P, R, bounds.data()));
        } else {
            SGX_TRY(sgx_even_ranges(P, R, bounds.data()));
        }
        std::lock_guard<std::mutex> sl(s->mu);
        if (s->place_bounds.empty()) s->place_bounds = bounds;
        bounds = s->place_bounds;
    }
    auto rd = std::make_shared<Round>();
    rd->map_ids = ids;
    rd->src = srcs;
    rd->lens = lens;
    rd->r0 = bounds[(size_t)e->rank];
    rd->r1 = bounds[(size_t)e->rank + 1];
    const int32_t nmine = rd->r1 - rd->r0;
    std::vector<int64_t> sc(P), sd(P), rc(P), rdp(P);
    rd->block_off.assign(M * (size_t)nmine, 0);
    SGX_TRY(sgx_plan_exchange_maps(lens.data(), counts.data(), P, R, e->rank, bounds.data(), sc.data(), sd.data(),
                                   rc.data(), rdp.data(), rd->block_off.data()));
    int64_t out_total = 0, total_recv = 0;
    for (auto &lm : mine) out_total += lm.bytes;
    for (int32_t j = 0; j < P; ++j) total_recv += rc[(size_t)j];
    if (sd[(size_t)P - 1] + sc[(size_t)P - 1] != out_total)
        return fail_msg(SGX_ERR_HIP, "internal error: send plan covers %lld of %lld bytes",
                        (long long)(sd[(size_t)P - 1] + sc[(size_t)P - 1]), (long long)out_total);
    // A round with the same maps replaces the previous one (a re-run): reuse its HBM when
    // nobody else still reads it.
    {
        std::lock_guard<std::mutex> sl(s->mu);
        for (auto it = s->rounds.begin(); it != s->rounds.end(); ++it) {
            if ((*it)->import_id == 0 && (*it)->map_ids == rd->map_ids) {
                if (it->use_count() == 1 && (*it)->alias.empty()) {
                    HIP_TRY((*it)->done.wait_host());
                    rd->data.swap((*it)->data);
                    std::swap(rd->ipc, (*it)->ipc);
                    std::swap(rd->ipc_valid, (*it)->ipc_valid);
                    std::swap(rd->ipc_gen, (*it)->ipc_gen);
                }
                s->rounds.erase(it);
                break;
            }
        }
    }
    // (3) the bytes.  Piece (my map k, destination d) = map k's reducers [bounds[d],
    //     bounds[d+1]), contiguous in the partition-contiguous map output.
    auto piece = [&](size_t k, int32_t d, int64_t *off, int64_t *len) {
        int64_t o = 0, l = 0;
        for (int32_t r = 0; r < bounds[(size_t)d]; ++r) o += mine[k].lens[(size_t)r];
        for (int32_t r = bounds[(size_t)d]; r < bounds[(size_t)d + 1]; ++r) l += mine[k].lens[(size_t)r];
        *off = o;
        *len = l;
    };
    if (!collective) {
        // one rank, no communicator: the blocks are the map outputs themselves
        rd->r0 = 0;
        rd->r1 = R;
        for (size_t k = 0; k < M; ++k) {
            rd->alias.push_back(mine[k].m);
            int64_t o = 0;
            for (int32_t r = 0; r < R; ++r) {
                rd->block_off[k * (size_t)R + (size_t)r] = o;
                o += mine[k].lens[(size_t)r];
            }
        }
        HIP_TRY(hipEventRecord(a2, st));
    } else if (p2p) {
        // peers write into the receive buffer through its IPC handle (a new allocation gets a
        // new handle)
        const void *was = rd->data.p;
        SGX_TRY(rd->data.ensure((size_t)std::max<int64_t>(total_recv, 16)));
        if (rd->data.p != was) rd->ipc_valid = false;
        HIP_TRY(hipEventRecord(a2, st));
        const int prc = p2p_data(e, *s, *rd, mine, bounds, lens, srcs, st);
        if (prc == P2P_UNAVAILABLE) {
            // nothing has moved on any rank: the round again over contiguous pieces, and the
            // engine's later maps two-pass (use_padded)
            if (!e->p2p_off.exchange(true))
                std::fprintf(stderr, "sgx: rank %d: direct peer gather unavailable (%s); exchanging contiguous pieces\n",
                             e->rank, sgx_last_error());
            e->release_events({a0, a1, a2, a3});
            return exchange_round(e, c, s, std::move(mine));
        }
        SGX_TRY(prc);
    } else {
        SGX_TRY(rd->data.ensure((size_t)std::max<int64_t>(total_recv, 16)));
        for (auto &lm : mine) HIP_TRY(hipStreamWaitEvent(st, lm.m->done.ev, 0));
        HIP_TRY(hipEventRecord(a2, st));
        if (e->comm) {
            // every source rank's choice: packed (one piece per destination) or per map
            std::vector<char> packed((size_t)P, 0);
            {
                size_t m = 0;
                for (int32_t j = 0; j < P; ++j) {
                    int64_t bytes = 0;
                    for (int64_t k = 0; k < counts[(size_t)j]; ++k, ++m)
                        for (int32_t r = 0; r < R; ++r) bytes += lens[m * R + r];
                    packed[(size_t)j] = packs_sends(counts[(size_t)j], bytes, P) ? 1 : 0;
                }
            }
            const bool pack_mine = packed[(size_t)e->rank] != 0;
            if (pack_mine && out_total > 0) {
                // my pieces, [destination][map] at the plan's send displacements, in one gather
                // launch on the exchange stream (ahead of the sends in stream order)
                std::vector<int64_t> items;
                bool al16 = true, al4 = true;
                SGX_TRY(e->x_pack.ensure((size_t)out_total));
                for (int32_t d = 0; d < P; ++d) {
                    int64_t pos = sd[(size_t)d];
                    for (size_t k = 0; k < mine.size(); ++k) {
                        int64_t o, l;
                        piece(k, d, &o, &l);
                        for (int64_t done = 0; done < l; done += 65536) {
                            const int64_t b = std::min<int64_t>(65536, l - done);
                            const uintptr_t src = (uintptr_t)mine[k].m->view() + (uintptr_t)(o + done);
                            const uintptr_t dst = (uintptr_t)e->x_pack.p + (uintptr_t)(pos + done);
                            items.push_back((int64_t)src);
                            items.push_back((int64_t)dst);
                            items.push_back(b);
                            al16 = al16 && ((src | dst | (uintptr_t)b) & 15) == 0;
                            al4 = al4 && ((src | dst | (uintptr_t)b) & 3) == 0;
                        }
                        pos += l;
                    }
                }
                const int64_t ni = (int64_t)items.size() / 3;
                SGX_TRY(e->x_items.ensure(items.size() * 8));
                SGX_TRY(e->x_items_dev.ensure(items.size() * 8));
                std::memcpy(e->x_items.p, items.data(), items.size() * 8);
                HIP_TRY(hipMemcpyAsync(e->x_items_dev.p, e->x_items.p, items.size() * 8, hipMemcpyHostToDevice, st));
                HIP_TRY(launch_gather_items((const int64_t *)e->x_items_dev.p, ni, al16 ? 16 : al4 ? 4 : 1, st));
                SGX_TRY(debug_sync(e, st, "exchange send pack"));
            }
            // grouped point-to-point: my sends to d go map after map (or as one packed piece),
            // and d posts its receives from me the same way (it knows my map count and lengths
            // from (1))
            // every ncclSend / ncclRecv of the group, then ncclGroupEnd even when one of them
            // failed (an open group would poison the communicator's next call)
            ncclResult_t gr = ncclGroupStart();
            if (gr != ncclSuccess) return fail_msg(SGX_ERR_COMM, "ncclGroupStart failed: %s", ncclGetErrorString(gr));
            ncclResult_t first = ncclSuccess;
            auto note = [&](ncclResult_t r) {
                if (r != ncclSuccess && first == ncclSuccess) first = r;
            };
            for (int32_t d = 0; d < P && first == ncclSuccess; ++d) {
                if (pack_mine) {
                    if (sc[(size_t)d] > 0)
                        note(ncclSend((const char *)e->x_pack.p + sd[(size_t)d], (size_t)sc[(size_t)d], ncclUint8, d,
                                      e->comm, st));
                    continue;
                }
                for (size_t k = 0; k < mine.size() && first == ncclSuccess; ++k) {
                    int64_t o, l;
                    piece(k, d, &o, &l);
                    if (l > 0) note(ncclSend((const char *)mine[k].m->view() + o, (size_t)l, ncclUint8, d, e->comm, st));
                }
            }
            size_t m = 0;
            for (int32_t j = 0; j < P && first == ncclSuccess; ++j) {
                if (packed[(size_t)j]) {
                    if (rc[(size_t)j] > 0)
                        note(ncclRecv((char *)rd->data.p + rdp[(size_t)j], (size_t)rc[(size_t)j], ncclUint8, j,
                                      e->comm, st));
                    m += (size_t)counts[(size_t)j];
                    continue;
                }
                int64_t off = rdp[(size_t)j];
                for (int64_t k = 0; k < counts[(size_t)j]; ++k, ++m) {
                    int64_t l = 0;
                    for (int32_t r = rd->r0; r < rd->r1; ++r) l += lens[m * R + r];
                    if (l > 0) note(ncclRecv((char *)rd->data.p + off, (size_t)l, ncclUint8, j, e->comm, st));
                    off += l;
                }
            }
            note(ncclGroupEnd());
            if (first != ncclSuccess)
                return fail_msg(SGX_ERR_COMM, "grouped ncclSend / ncclRecv failed: %s", ncclGetErrorString(first));
        } else {
            // host backend: stage my pieces out packed [destination][map], exchange on the
            // host, stage the received bytes in
            SGX_TRY(e->x_send.ensure((size_t)std::max<int64_t>(out_total, 16)));
            SGX_TRY(e->x_recv.ensure((size_t)std::max<int64_t>(total_recv, 16)));
            int64_t pos = 0;
            for (int32_t d = 0; d < P; ++d)
                for (size_t k = 0; k < mine.size(); ++k) {
                    int64_t o, l;
                    piece(k, d, &o, &l);
                    if (l > 0)
                        HIP_TRY(hipMemcpyAsync((char *)e->x_send.p + pos, (const char *)mine[k].m->view() + o,
                                               (size_t)l, hipMemcpyDeviceToHost, st));
                    pos += l;
                }
            HIP_TRY(hipStreamSynchronize(st));
            if (e->hc.alltoallv(e->hc.user, e->x_send.p, sc.data(), sd.data(), e->x_recv.p, rc.data(), rdp.data()) != 0)
                return fail_msg(SGX_ERR_COMM, "host all-to-all of the map outputs failed");
            if (total_recv > 0)
                HIP_TRY(hipMemcpyAsync(rd->data.p, e->x_recv.p, (size_t)total_recv, hipMemcpyHostToDevice, st));
            HIP_TRY(hipStreamSynchronize(st));  // the pinned staging buffers are reused next round
        }
    }
    if (collective && !p2p) {  // RCCL send / recv or the host all-to-all: contiguous pieces
        std::lock_guard<std::mutex> lk(e->stats_mu);
        e->x_bytes[0] += out_total - sc[(size_t)e->rank];
        e->x_bytes[1] += sc[(size_t)e->rank];
        e->x_bytes[2] += 1;
    }
    HIP_TRY(hipEventRecord(a3, st));
    HIP_TRY(rd->done.record(st));
    for (auto &lm : mine) {
        std::lock_guard<std::mutex> lk(lm.m->mu);
        if (collective) HIP_TRY(lm.m->read_done.record(st));
        lm.m->exchanged = true;
    }
    e->record_stage(SGX_STAGE_ALLGATHER, a0, a1);
    e->record_stage(SGX_STAGE_ALLTOALL, a2, a3);
    std::lock_guard<std::mutex> sl(s->mu);
    s->rounds.push_back(std::move(rd));
    return SGX_OK;
}

// The round's first all-gather ([count | the first map's {id, R lengths}], as exchange_round
// sizes it) joined with a failure mark: every rank then fails the round together instead of
// waiting in the collective.  Caller holds comm_mu.
static int join_failed(sgx_engine *e, int32_t R, int code, const std::string &why) {
    if (e->comm_broken) return fail_msg(SGX_ERR_STATE, "the communicator was aborted after an exchange failure");
    if (!(e->comm || e->host_comm)) return fail_msg(code, "%s", why.c_str());
    std::vector<int64_t> first((size_t)R + 2, 0), all(first.size() * (size_t)e->nranks, 0);
    first[0] = -1 + (int64_t)code;
    SGX_TRY(allgather_i64(e, first.data(), first.size(), all.data()));
    return fail_msg(code, "%s (every rank fails this exchange)", why.c_str());
}

// hipSetDevice + the calling thread's context; a failure on a collective engine joins the
// round marked failed (the shuffle is known, so is the all-gather's size)
static Ctx *exchange_ctx(sgx_engine *e, const Shuffle &s, int *rc) {
    const hipError_t he = hipSetDevice(e->device);
    Ctx *c = he == hipSuccess ? e->ctx() : nullptr;
    if (c) return c;
    const std::string why = he != hipSuccess ? std::string("hipSetDevice: ") + hipGetErrorString(he)
                                             : std::string(sgx_last_error());
    std::lock_guard<std::mutex> clk(e->comm_mu);
    *rc = join_failed(e, s.R, SGX_ERR_HIP, why);
    return nullptr;
}

extern "C" int sgx_exchange(sgx_engine *e, int32_t shuffle_id) {
    sgx::TraceRange trace_("sgx_exchange");
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    // an unknown shuffle cannot size the round's all-gather: a collective caller that failed
    // to register it joins the round through sgx_exchange_fail(e, R, code) instead
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    int rc = SGX_OK;
    Ctx *c = exchange_ctx(e, *s, &rc);
    if (!c) return rc;
    // every committed map output no earlier round carried, in map id order (snapshot now:
    // the call's place in the caller's program order decides what it carries), selected under
    // comm_mu: the round marks them exchanged before another exchange can select
    std::lock_guard<std::mutex> clk(e->comm_mu);
    std::vector<LocalMap> mine;
    {
        std::lock_guard<std::mutex> sl(s->mu);
        for (auto &kv : s->maps) mine.push_back(LocalMap{kv.first, kv.second, {}, 0});
    }
    std::vector<LocalMap> take;
    for (auto &lm : mine) {
        std::lock_guard<std::mutex> lk(lm.m->mu);
        if (lm.m->written && !lm.m->open && !lm.m->exchanged) take.push_back(std::move(lm));
    }
    return exchange_round(e, c, s, std::move(take));
}

extern "C" int sgx_exchange_maps(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t n) {
    sgx::TraceRange trace_("sgx_exchange_maps");
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e || n < 0 || (n > 0 && !map_ids)) return fail_msg(SGX_ERR_INVALID, "bad arguments");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    int rc = SGX_OK;
    Ctx *c = exchange_ctx(e, *s, &rc);
    if (!c) return rc;
    std::vector<LocalMap> mine;
    std::string msg;
    for (int64_t i = 0; i < n && rc == SGX_OK; ++i) {
        std::shared_ptr<Shuffle> s2;
        std::shared_ptr<MapOut> m;
        rc = find_map(e, shuffle_id, map_ids[i], &s2, &m);
        if (rc == SGX_OK) mine.push_back(LocalMap{map_ids[i], m, {}, 0});
        else msg = sgx_last_error();
    }
    // an unknown map still joins the round's first all-gather, marked failed
    std::lock_guard<std::mutex> clk(e->comm_mu);
    return exchange_round(e, c, s, std::move(mine), rc, msg);
}

extern "C" int sgx_exchange_fail(sgx_engine *e, int32_t num_partitions, int32_t code) {
    sgx::TraceRange trace_("sgx_exchange_fail");
    if (!e || num_partitions < 1 || code >= 0) return fail_msg(SGX_ERR_INVALID, "sgx_exchange_fail: bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    std::lock_guard<std::mutex> clk(e->comm_mu);
    return join_failed(e, num_partitions, code, "this rank failed the exchange before it began");
}

// ------------------------------------------------------------------------------------
// blocks fetched from elsewhere (a reduce task Spark placed off the reducers' owner)
// ------------------------------------------------------------------------------------
// The reference's reader takes any block from anywhere (spark_3_0/UcxShuffleReader.scala:
// 74-103); here a reduce task on an executor that does not own its reducers fetches their
// raw blocks from the owners (over Spark RPC) and hands them to its own engine, which then
// runs the reads (sgx_read_records / _sorted / _grouped, sgx_fetch_blocks) over them on the
// GPU exactly as over exchanged blocks: the import is a round of its own.
extern "C" int sgx_import_blocks(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                                 int32_t start_partition, int32_t end_partition, const void *data,
                                 int32_t mem_kind, const int64_t *lengths, int64_t *out_import_id) {
    sgx::TraceRange trace_("sgx_import_blocks");
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e || !out_import_id || nmaps < 0 || (nmaps > 0 && !map_ids))
        return fail_msg(SGX_ERR_INVALID, "sgx_import_blocks: bad arguments");
    if (mem_kind != SGX_MEM_HOST && mem_kind != SGX_MEM_DEVICE)
        return fail_msg(SGX_ERR_INVALID, "unknown mem_kind %d", mem_kind);
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    const int32_t R = s->R;
    if (start_partition < 0 || end_partition > R || start_partition > end_partition)
        return fail_msg(SGX_ERR_INVALID, "partition range [%d, %d) outside [0, %d)", start_partition, end_partition, R);
    const int32_t nmine = end_partition - start_partition;
    const int64_t nblk = (int64_t)nmine * nmaps;
    if (nblk > 0 && !lengths) return fail_msg(SGX_ERR_INVALID, "lengths is NULL");
    {
        std::vector<int64_t> ids(map_ids, map_ids + nmaps);
        std::sort(ids.begin(), ids.end());
        if (std::adjacent_find(ids.begin(), ids.end()) != ids.end())
            return fail_msg(SGX_ERR_INVALID, "an import lists a map id twice");
    }
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    auto rd = std::make_shared<Round>();
    rd->map_ids.assign(map_ids, map_ids + nmaps);
    rd->src.assign((size_t)nmaps, -1);
    rd->r0 = start_partition;
    rd->r1 = end_partition;
    rd->lens.assign((size_t)nmaps * (size_t)R, 0);
    rd->block_off.assign((size_t)nblk, 0);
    // `data` holds the blocks in the canonical order: reducer-major, then map (what
    // sgx_fetch_blocks returns for the same list)
    int64_t off = 0;
    for (int32_t r = 0; r < nmine; ++r)
        for (int64_t j = 0; j < nmaps; ++j) {
            const int64_t L = lengths[(size_t)r * nmaps + j];
            if (L < 0) return fail_msg(SGX_ERR_INVALID, "negative block length");
            if (s->ser == SGX_SER_FIXED && L % s->rb)
                return fail_msg(SGX_ERR_INVALID, "block of %lld bytes is not whole %d B records", (long long)L, s->rb);
            rd->lens[(size_t)j * R + (size_t)(start_partition + r)] = L;
            rd->block_off[(size_t)j * nmine + (size_t)r] = off;
            off += L;
        }
    if (off > 0 && !data) return fail_msg(SGX_ERR_INVALID, "data is NULL");
    SGX_TRY(rd->data.ensure((size_t)std::max<int64_t>(off, 16) + 64));  // readers may read 32 B past
    if (off > 0)
        HIP_TRY(hipMemcpyAsync(rd->data.p, data, (size_t)off,
                               mem_kind == SGX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->st));
    HIP_TRY(rd->done.record(c->st));
    HIP_TRY(hipStreamSynchronize(c->st));  // the caller's buffer may go once this returns
    std::lock_guard<std::mutex> sl(s->mu);
    rd->import_id = s->next_import++;
    *out_import_id = rd->import_id;
    s->rounds.push_back(std::move(rd));
    return SGX_OK;
}

extern "C" int sgx_release_import(sgx_engine *e, int32_t shuffle_id, int64_t import_id) {
    if (e) e->mutated();
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    std::shared_ptr<Round> gone;  // freed outside the lock (its destructor waits for readers)
    {
        std::lock_guard<std::mutex> sl(s->mu);
        for (auto it = s->rounds.begin(); it != s->rounds.end(); ++it)
            if ((*it)->import_id == import_id && import_id != 0) {
                gone = *it;
                s->rounds.erase(it);
                break;
            }
    }
    if (!gone) return fail_msg(SGX_ERR_NOT_FOUND, "shuffle %d has no import %lld", shuffle_id, (long long)import_id);
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
        for (int64_t m : (*it)->import_id ? std::vector<int64_t>() : (*it)->map_ids)
            if (m == map_id) {
                *r0 = (*it)->r0;
                *r1 = (*it)->r1;
                return SGX_OK;
            }
    return fail_msg(SGX_ERR_NOT_FOUND, "no exchange round of shuffle %d carried map %lld", shuffle_id,
                    (long long)map_id);
}

extern "C" int sgx_shuffle_reducers(sgx_engine *e, int32_t shuffle_id, int32_t *r0, int32_t *r1) {
    if (!e || !r0 || !r1) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    std::lock_guard<std::mutex> sl(s->mu);
    if (s->place_bounds.size() != (size_t)e->nranks + 1)
        return fail_msg(SGX_ERR_STATE, "shuffle %d has not been exchanged yet", shuffle_id);
    *r0 = s->place_bounds[(size_t)e->rank];
    *r1 = s->place_bounds[(size_t)e->rank + 1];
    return SGX_OK;
}
