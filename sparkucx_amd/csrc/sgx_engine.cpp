// sgx_engine.cpp — engine lifetime, per-thread contexts, the shuffle registry, progress /
// sync and stage statistics of the C ABI (include/sgx.h).
//
// One engine per GPU (= per Spark executor).  It replaces, on the hot path:
//   * the map-output writer + NVKV storage (ucx/NvkvShuffleMapOutputWriter.scala:105-148,
//     ucx/NvkvHandler.scala:213-265): map outputs are partitioned by HIP kernels and kept
//     resident in HBM, engine-owned (sgx_map.cpp);
//   * the index commit (IndexShuffleBlockResolver.scala:161-217) when a file is wanted
//     (sgx_index.cpp);
//   * the UCX fetch path (ucx/UcxWorkerWrapper.scala:96-186, spark_3_0/UcxShuffleClient.scala
//     :17-91): one counts all-gather + ncclAllToAllv over xGMI, then block fetches served from
//     HBM (sgx_exchange.cpp, sgx_read.cpp).
// There is no CPU fallback: every data-path call runs the HIP kernels or fails.
#include "sgx_engine.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

using namespace sgx;

// ------------------------------------------------------------------------------------
// contexts, events, stats
// ------------------------------------------------------------------------------------
#ifndef SGX_TAIL_LOW_PRIORITY
#define SGX_TAIL_LOW_PRIORITY 0
#endif

// A host memcpy split over up to 8 threads (pieces of >= 4 MiB): the pinned staging of host
// batches (sgx_map_append), where one thread's copy bounded the ingest (29 -> 53 GB/s,
// bench.py --batches 64 --host-batches).
void sgx::host_copy_parallel(char *dst, const char *src, size_t bytes) {
    constexpr size_t PART_MIN = (size_t)4 << 20;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = std::min<size_t>({(size_t)8, (size_t)hw, std::max<size_t>(1, bytes / PART_MIN)});
    const size_t part = ((bytes + nt - 1) / nt + 63) & ~(size_t)63;
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; ++t) {
        const size_t o = t * part;
        if (o >= bytes) break;
        th.emplace_back([=] { std::memcpy(dst + o, src + o, std::min(part, bytes - o)); });
    }
    std::memcpy(dst, src, std::min(part, bytes));
    for (auto &x : th) x.join();
}

Ctx *sgx_engine::ctx() {
    std::lock_guard<std::mutex> lk(reg_mu);
    auto &slot = ctxs[std::this_thread::get_id()];
    if (!slot) {
        std::unique_ptr<Ctx> c(new Ctx());
        // (A/B: -DSGX_TAIL_LOW_PRIORITY=1 puts the padded write's tail on a low-priority
        // stream, so the next write's sample and K4 are dispatched ahead of it)
        int lo = 0, hi = 0;
        if (!SGX_TAIL_LOW_PRIORITY || hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
        if (hipStreamCreateWithPriority(&c->st, hipStreamNonBlocking, hi) != hipSuccess ||
            hipStreamCreateWithPriority(&c->st_tail, hipStreamNonBlocking, lo) != hipSuccess ||
            hipStreamCreateWithFlags(&c->st_pre, hipStreamNonBlocking) != hipSuccess) {
            ctxs.erase(std::this_thread::get_id());
            fail_msg(SGX_ERR_HIP, "hipStreamCreate failed for a new calling thread");
            return nullptr;
        }
        slot = std::move(c);
    }
    slot->ops++;
    return slot.get();
}

#ifndef SGX_STAGE_EVENT_FENCE
#define SGX_STAGE_EVENT_FENCE 0
#endif

hipEvent_t sgx_engine::ev() {
    {
        std::lock_guard<std::mutex> lk(stats_mu);
        if (!ev_free.empty()) {
            hipEvent_t e = ev_free.back();
            ev_free.pop_back();
            return e;
        }
    }
    hipEvent_t e = nullptr;
    // stage events only time the kernels between them (resolve_stats; nothing waits on them
    // for ordering), so they skip the system-scope fence a default event's record performs:
    // that fence idles the GPU ~6 µs per record between a map write's kernels (kernel trace,
    // DESIGN.md §9).  A/B: -DSGX_STAGE_EVENT_FENCE=1 restores the default.
#if SGX_STAGE_EVENT_FENCE
    (void)hipEventCreate(&e);
#else
    (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
#endif
    return e;
}

void sgx_engine::record_stage(int stage, hipEvent_t a, hipEvent_t b) {
    std::lock_guard<std::mutex> lk(stats_mu);
    pending.push_back(PendingStage{stage, a, b});
}

void sgx_engine::release_events(std::initializer_list<hipEvent_t> evs) {
    std::lock_guard<std::mutex> lk(stats_mu);
    for (hipEvent_t v : evs)
        if (v && std::find(ev_free.begin(), ev_free.end(), v) == ev_free.end()) ev_free.push_back(v);
}

void sgx_engine::resolve_stats() {
    std::lock_guard<std::mutex> lk(stats_mu);
    for (auto &p : pending) {
        float ms = 0.f;
        if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            stage_ms[p.stage] += ms;
            stage_n[p.stage] += 1;
        }
        ev_free.push_back(p.a);
        ev_free.push_back(p.b);
    }
    pending.clear();
    // consecutive stages may share their boundary event: return each event once
    std::sort(ev_free.begin(), ev_free.end());
    ev_free.erase(std::unique(ev_free.begin(), ev_free.end()), ev_free.end());
}

std::shared_ptr<Shuffle> sgx_engine::find_shuffle(int32_t shuffle_id) {
    std::lock_guard<std::mutex> lk(reg_mu);
    auto it = shuffles.find(shuffle_id);
    if (it == shuffles.end()) {
        fail_msg(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
        return nullptr;
    }
    return it->second;
}

int sgx::find_map(sgx_engine *e, int32_t shuffle_id, int64_t map_id, std::shared_ptr<Shuffle> *ps,
                  std::shared_ptr<MapOut> *pm) {
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    std::lock_guard<std::mutex> lk(s->mu);
    auto mt = s->maps.find(map_id);
    if (mt == s->maps.end())
        return fail_msg(SGX_ERR_NOT_FOUND, "map %lld of shuffle %d was not written", (long long)map_id, shuffle_id);
    *ps = s;
    *pm = mt->second;
    return SGX_OK;
}

static uint32_t bits_for(uint32_t R) {
    uint32_t b = 0;
    while ((1ull << b) < R) ++b;
    return b ? b : 1;
}

int sgx::debug_sync(sgx_engine *e, hipStream_t st, const char *what) {
    if (!(e->flags & SGX_FLAG_DEBUG_SYNC)) return SGX_OK;
    const hipError_t a = hipStreamSynchronize(st);
    const hipError_t b = hipGetLastError();
    if (a != hipSuccess || b != hipSuccess)
        return fail_msg(SGX_ERR_HIP, "%s: %s / %s", what, hipGetErrorString(a), hipGetErrorString(b));
    return SGX_OK;
}

PartParams sgx::make_part_params(const Shuffle &s) {
    PartParams pp{};
    pp.kind = s.kind;
    pp.R = (uint32_t)s.R;
    mod_params((uint32_t)s.R, &pp.mg_m, &pp.mg_s);
    pp.c31 = (uint32_t)((1ull << 31) % (uint64_t)s.R);
    pp.nbits = bits_for((uint32_t)s.R);
    pp.nb = s.nb;
    pp.ascending = s.asc;
    pp.bounds = s.bounds.p;
    pp.dir = s.dir_ok ? (const uint16_t *)((const char *)s.bounds.p + s.dir_off) : nullptr;
    return pp;
}

// ------------------------------------------------------------------------------------
// lifetime
// ------------------------------------------------------------------------------------
// The default ranking's premise, checked on the device the engine runs on:
// on a violation every scatter is ranked by ballot peer matching instead (same bytes, slower).
static int check_lds_order(sgx_engine *e) {
    uint32_t *bad = nullptr;
    HIP_TRY(hipMalloc((void **)&bad, 4));
    uint32_t h = 0;
    hipError_t r = hipMemsetAsync(bad, 0, 4, e->s_comm);
    if (r == hipSuccess) r = launch_lds_order_probe(bad, e->s_comm);
    if (r == hipSuccess) r = hipMemcpyAsync(&h, bad, 4, hipMemcpyDeviceToHost, e->s_comm);
    if (r == hipSuccess) r = hipStreamSynchronize(e->s_comm);
    (void)hipFree(bad);
    HIP_TRY(r);
    e->lds_order_ok = h == 0 && !(e->flags & SGX_FLAG_ASSUME_LDS_DISORDER);
    if (!e->lds_order_ok) e->rank_mode = SGX_RANK_MATCH;
    return SGX_OK;
}

extern "C" int sgx_create(const sgx_config *cfg, sgx_engine **out) {
    if (!out) return fail_msg(SGX_ERR_INVALID, "sgx_create: out is NULL");
    *out = nullptr;
    int dev = cfg ? cfg->device : 0;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (dev < 0 || dev >= ndev) return fail_msg(SGX_ERR_INVALID, "sgx_create: device %d of %d", dev, ndev);
    if (cfg && (cfg->hist_mode < SGX_HIST_ATOMIC || cfg->hist_mode > SGX_HIST_BALLOT ||
                cfg->rank_mode < SGX_RANK_ORDERED || cfg->rank_mode > SGX_RANK_MATCH || cfg->flags < 0 ||
                cfg->flags > 32767 || cfg->comm_timeout_ms < 0 || cfg->num_chunks < 0))
        return fail_msg(SGX_ERR_INVALID, "sgx_create: bad configuration");
    HIP_TRY(hipSetDevice(dev));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, dev));
    std::unique_ptr<sgx_engine> e(new sgx_engine());
    e->device = dev;
    e->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    e->G = (cfg && cfg->num_chunks > 0) ? cfg->num_chunks : e->num_cus;
    e->G_forced = cfg && cfg->num_chunks > 0;
    if (cfg) {
        e->sc_waves = cfg->scatter_waves;
        e->sc_items = cfg->scatter_items;
        e->hist_mode = cfg->hist_mode;
        e->rank_mode = cfg->rank_mode;
        e->flags = cfg->flags;
        if (cfg->flags & SGX_FLAG_PAD_ANY_SIZE) e->pad_min = 1;
        if (cfg->flags & SGX_FLAG_NO_OVERLAP_WRITES) e->overlap_writes = false;
        if (cfg->comm_timeout_ms > 0) e->comm_timeout_ms = cfg->comm_timeout_ms;
    }
    HIP_TRY(hipStreamCreateWithFlags(&e->s_comm, hipStreamNonBlocking));
    SGX_TRY(check_lds_order(e.get()));
    *out = e.release();
    return SGX_OK;
}

extern "C" int32_t sgx_lds_order_ok(const sgx_engine *e) { return e ? (e->lds_order_ok ? 1 : 0) : -1; }

extern "C" void sgx_destroy(sgx_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    (void)hipDeviceSynchronize();
    e->resolve_stats();
    e->shuffles.clear();  // map outputs and rounds free their HBM
    e->ctxs.clear();
    for (auto &kv : e->p2p_cache) {  // peers' receive buffers the exchange mapped
        (void)hipIpcCloseMemHandle(kv.second.ptr);
        if (kv.second.done) (void)hipEventDestroy(kv.second.done);
    }
    e->p2p_cache.clear();
    for (hipEvent_t ev : e->ev_free) (void)hipEventDestroy(ev);
    if (e->comm) {
        if (e->comm_broken) (void)ncclCommAbort(e->comm);
        else (void)ncclCommDestroy(e->comm);
    }
    (void)hipStreamDestroy(e->s_comm);
    delete e;
}

extern "C" int sgx_release_thread(sgx_engine *e) {
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    HIP_TRY(hipSetDevice(e->device));
    std::unique_ptr<Ctx> c;
    {
        std::lock_guard<std::mutex> lk(e->reg_mu);
        auto it = e->ctxs.find(std::this_thread::get_id());
        if (it == e->ctxs.end()) return SGX_OK;
        c = std::move(it->second);
        e->ctxs.erase(it);
    }
    e->resolve_stats();  // pending stage events may sit on this stream
    c.reset();           // synchronises and destroys the stream
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// registerShuffle / unregisterShuffle / dependency properties
// ------------------------------------------------------------------------------------
static int max_partitions(int rb) {
    // LDS budget of the scatter kernels (sgx_kernels.hip scatter_geom*).
    for (uint32_t R = 8192; R >= 1; R -= 1) {
        ScatterGeom g = rb == 16 ? scatter_geom16(R) : scatter_geom_wide(R, rb);
        if (g.items > 0) return (int)R;
    }
    return 0;
}

extern "C" int sgx_register_shuffle(sgx_engine *e, int32_t shuffle_id, int32_t R, int32_t kind,
                                    const void *bounds, int64_t nbounds, int32_t ascending,
                                    int32_t rb) {
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    if (R < 1) return fail_msg(SGX_ERR_INVALID, "numPartitions must be positive, got %d", R);
    if (kind < SGX_PART_HASH || kind > SGX_PART_RANGE_BYTES10)
        return fail_msg(SGX_ERR_INVALID, "unknown partitioner kind %d", kind);
    if (rb < 12 || (rb & 3) != 0)
        return fail_msg(SGX_ERR_INVALID, "record_bytes must be a multiple of 4 and >= 12, got %d", rb);
    if (kind != SGX_PART_HASH && nbounds != (int64_t)R - 1)
        return fail_msg(SGX_ERR_INVALID, "RangePartitioner needs numPartitions == bounds+1 (%d vs %lld)", R,
                        (long long)nbounds);
    if (kind != SGX_PART_HASH && nbounds > 0 && !bounds)
        return fail_msg(SGX_ERR_INVALID, "range bounds pointer is NULL");
    const int rmax = max_partitions(rb);
    if (R > rmax)
        return fail_msg(SGX_ERR_UNSUPPORTED, "numPartitions %d exceeds the single-pass LDS limit %d", R, rmax);
    HIP_TRY(hipSetDevice(e->device));
    auto s = std::make_shared<Shuffle>();
    s->id = shuffle_id;
    s->R = R;
    s->kind = kind;
    s->nb = (int32_t)(kind == SGX_PART_HASH ? 0 : nbounds);
    s->asc = ascending ? 1 : 0;
    s->rb = rb;
    if (kind != SGX_PART_HASH && nbounds > 0) {
        // bounds in the kernels' layout (i64, or Key10 = big-endian 10-byte keys), then the
        // top-bits directory when the lower bound IS RangePartitioner.getPartition's answer
        std::vector<uint64_t> top((size_t)nbounds);  // bounds as unsigned-ordered 64-bit tops
        std::vector<Key10> k;
        const size_t braw = kind == SGX_PART_RANGE_I64 ? (size_t)nbounds * 8 : (size_t)nbounds * sizeof(Key10);
        const size_t boff = (braw + 15) & ~(size_t)15;
        bool strict = true, sorted = true;
        if (kind == SGX_PART_RANGE_I64) {
            const int64_t *b = (const int64_t *)bounds;
            for (int64_t i = 0; i < nbounds; ++i) {
                top[(size_t)i] = (uint64_t)b[i] ^ 0x8000000000000000ull;  // signed order -> unsigned
                if (i && b[i] <= b[i - 1]) { strict = false; sorted = sorted && b[i] == b[i - 1]; }
            }
        } else {
            k.resize((size_t)nbounds);
            const uint8_t *b = (const uint8_t *)bounds;
            for (int64_t i = 0; i < nbounds; ++i) {
                const uint8_t *q = b + 10 * i;
                uint64_t hi = 0;
                for (int j = 0; j < 8; ++j) hi = (hi << 8) | q[j];
                k[(size_t)i] = Key10{hi, ((uint32_t)q[8] << 8) | q[9], 0};
                top[(size_t)i] = hi;
                if (i) {
                    const Key10 &a = k[(size_t)i - 1], &c = k[(size_t)i];
                    const bool le = c.hi < a.hi || (c.hi == a.hi && c.lo <= a.lo);
                    if (le) { strict = false; sorted = sorted && c.hi == a.hi && c.lo == a.lo; }
                }
            }
        }
        // Spark's linear branch (<= 128 bounds) is a lower bound for any sorted bounds; its
        // binary search (JDK Arrays.binarySearch) is one for strictly increasing bounds (what
        // RangePartitioner.determineBounds produces) -- otherwise keep the exact JDK loop
        s->dir_ok = sorted && (strict || nbounds <= 128) && nbounds < 65535;
        s->dir_off = boff;
        SGX_TRY(s->bounds.ensure(boff + RDIR_BYTES));
        if (kind == SGX_PART_RANGE_I64) HIP_TRY(hipMemcpy(s->bounds.p, bounds, braw, hipMemcpyHostToDevice));
        else HIP_TRY(hipMemcpy(s->bounds.p, k.data(), braw, hipMemcpyHostToDevice));
        if (s->dir_ok) {
            std::vector<uint16_t> dir((size_t)RDIR_N);
            int64_t i = 0;
            for (int64_t j = 0; j < RDIR_N; ++j) {
                while (i < nbounds && (int64_t)(top[(size_t)i] >> (64 - RDIR_BITS)) < j) ++i;
                dir[(size_t)j] = (uint16_t)i;
            }
            HIP_TRY(hipMemcpy((char *)s->bounds.p + boff, dir.data(), dir.size() * 2, hipMemcpyHostToDevice));
        }
    }
    s->pp = make_part_params(*s);
    std::lock_guard<std::mutex> lk(e->reg_mu);
    if (e->shuffles.count(shuffle_id)) return fail_msg(SGX_ERR_STATE, "shuffle %d is already registered", shuffle_id);
    e->shuffles[shuffle_id] = s;
    return SGX_OK;
}

extern "C" int sgx_unregister_shuffle(sgx_engine *e, int32_t shuffle_id) {
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    HIP_TRY(hipSetDevice(e->device));
    std::shared_ptr<Shuffle> s;
    {
        std::lock_guard<std::mutex> lk(e->reg_mu);
        auto it = e->shuffles.find(shuffle_id);
        if (it == e->shuffles.end()) return fail_msg(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
        s = std::move(it->second);
        e->shuffles.erase(it);
    }
    // the HBM goes when the last in-flight user drops its reference (map outputs and rounds
    // wait for their producers / readers in their destructors)
    s.reset();
    return SGX_OK;
}

extern "C" int sgx_set_serializer(sgx_engine *e, int32_t shuffle_id, int32_t serializer) {
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    if (serializer != SGX_SER_FIXED && serializer != SGX_SER_KRYO)
        return fail_msg(SGX_ERR_INVALID, "unknown serializer %d", serializer);
    if (!s->configurable()) return fail_msg(SGX_ERR_STATE, "shuffle %d already has map outputs", shuffle_id);
    if (serializer == SGX_SER_KRYO && (s->rb != 16 || s->kind == SGX_PART_RANGE_BYTES10))
        return fail_msg(SGX_ERR_UNSUPPORTED, "Kryo framing is for (Long, Long) 16 B records, not %d B", s->rb);
    // LZ4 is published over the Kryo stream: a fixed-codec shuffle cannot keep it
    if (serializer != SGX_SER_KRYO && s->lz4_block > 0)
        return fail_msg(SGX_ERR_STATE, "shuffle %d is LZ4-compressed: turn compression off before leaving Kryo",
                        shuffle_id);
    s->ser = serializer;
    return SGX_OK;
}

extern "C" int sgx_set_compression(sgx_engine *e, int32_t shuffle_id, int32_t codec, int32_t block_size) {
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    if (codec != SGX_CODEC_NONE && codec != SGX_CODEC_LZ4) return fail_msg(SGX_ERR_INVALID, "unknown codec %d", codec);
    if (!s->configurable()) return fail_msg(SGX_ERR_STATE, "shuffle %d already has map outputs", shuffle_id);
    if (codec == SGX_CODEC_LZ4) {
        if (s->ser != SGX_SER_KRYO)
            return fail_msg(SGX_ERR_UNSUPPORTED,
                            "LZ4 compression is published over the Kryo stream (sgx_set_serializer first)");
        if (block_size < 64 || block_size > sgx::lz4_max_block())
            return fail_msg(SGX_ERR_UNSUPPORTED, "LZ4 block size %d outside [64, %d]", block_size,
                            sgx::lz4_max_block());
    }
    s->lz4_block = codec == SGX_CODEC_LZ4 ? block_size : 0;
    return SGX_OK;
}

extern "C" int sgx_set_map_side_combine(sgx_engine *e, int32_t shuffle_id, int32_t agg) {
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    if (agg != SGX_AGG_SUM && agg != -1)
        return fail_msg(SGX_ERR_UNSUPPORTED, "map-side combine supports SGX_AGG_SUM (reduceByKey), not %d", agg);
    if (!s->configurable()) return fail_msg(SGX_ERR_STATE, "shuffle %d already has map outputs", shuffle_id);
    if (agg == SGX_AGG_SUM && (s->rb != 16 || s->kind == SGX_PART_RANGE_BYTES10))
        return fail_msg(SGX_ERR_UNSUPPORTED, "map-side combine needs (Long, Long) 16 B records");
    if (agg == SGX_AGG_SUM && s->writer == SGX_WRITER_UNSAFE)
        return fail_msg(SGX_ERR_STATE, "shuffle %d runs UnsafeShuffleWriter, which never combines", shuffle_id);
    s->combine = agg;
    return SGX_OK;
}

extern "C" int sgx_set_map_writer(sgx_engine *e, int32_t shuffle_id, int32_t writer) {
    if (e) e->mutated();  // invalidates cached reduce-side results (sgx_read_*)
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    if (writer != SGX_WRITER_SORT && writer != SGX_WRITER_UNSAFE)
        return fail_msg(SGX_ERR_INVALID, "unknown map writer %d", writer);
    if (!s->configurable()) return fail_msg(SGX_ERR_STATE, "shuffle %d already has map outputs", shuffle_id);
    if (writer == SGX_WRITER_UNSAFE && s->combine != -1)  // SortShuffleManager.canUseSerializedShuffle
        return fail_msg(SGX_ERR_STATE, "shuffle %d combines map-side: Spark runs SortShuffleWriter for it", shuffle_id);
    s->writer = writer;
    return SGX_OK;
}

extern "C" int sgx_set_reducer_placement(sgx_engine *e, int32_t shuffle_id, int32_t placement) {
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    if (placement != SGX_PLACE_EVEN && placement != SGX_PLACE_BYTES)
        return fail_msg(SGX_ERR_INVALID, "unknown reducer placement %d", placement);
    std::shared_ptr<Shuffle> s = e->find_shuffle(shuffle_id);
    if (!s) return SGX_ERR_STATE;
    std::lock_guard<std::mutex> sl(s->mu);
    if (!s->place_bounds.empty())  // a reducer's blocks must all land on one rank
        return fail_msg(SGX_ERR_STATE, "shuffle %d was already exchanged: its reducer ranges are fixed", shuffle_id);
    s->placement.store(placement);
    return SGX_OK;
}

extern "C" int sgx_set_overlap_writes(sgx_engine *e, int32_t on) {
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    e->overlap_writes = on != 0;
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// progress / sync / stats
// ------------------------------------------------------------------------------------
extern "C" int sgx_progress(sgx_engine *e) {
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    std::vector<hipStream_t> streams;
    {
        std::lock_guard<std::mutex> lk(e->reg_mu);
        for (auto &kv : e->ctxs) {
            streams.push_back(kv.second->st);
            streams.push_back(kv.second->st_tail);
            streams.push_back(kv.second->st_pre);
        }
    }
    streams.push_back(e->s_comm);
    bool done = true;
    for (hipStream_t st : streams) {
        hipError_t q = hipStreamQuery(st);
        if (q != hipSuccess && q != hipErrorNotReady)
            return fail_msg(SGX_ERR_HIP, "stream error: %s", hipGetErrorString(q));
        done = done && q == hipSuccess;
    }
    return done ? 1 : 0;
}

extern "C" int sgx_sync(sgx_engine *e) {
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    std::vector<hipStream_t> streams;
    std::vector<std::shared_ptr<Shuffle>> all;
    {
        std::lock_guard<std::mutex> lk(e->reg_mu);
        for (auto &kv : e->ctxs) {
            streams.push_back(kv.second->st);
            streams.push_back(kv.second->st_tail);
            streams.push_back(kv.second->st_pre);
        }
        for (auto &kv : e->shuffles) all.push_back(kv.second);
    }
    for (hipStream_t st : streams) HIP_TRY(hipStreamSynchronize(st));
    {
        std::lock_guard<std::mutex> lk(e->comm_mu);
        SGX_TRY(comm_wait(e));
    }
    for (auto &s : all) {
        std::vector<std::shared_ptr<MapOut>> maps;
        {
            std::lock_guard<std::mutex> lk(s->mu);
            for (auto &kv : s->maps) maps.push_back(kv.second);
        }
        for (auto &m : maps) {
            std::lock_guard<std::mutex> lk(m->mu);
            if (m->written && !m->open) SGX_TRY(finish_lengths(e, *c, *s, *m));
        }
    }
    return SGX_OK;
}

extern "C" int sgx_stats_reset(sgx_engine *e) {
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    e->resolve_stats();
    std::lock_guard<std::mutex> lk(e->stats_mu);
    for (int i = 0; i < SGX_NUM_STAGES; ++i) {
        e->stage_ms[i] = 0;
        e->stage_n[i] = 0;
    }
    for (int64_t &b : e->x_bytes) b = 0;
    return SGX_OK;
}

extern "C" int sgx_exchange_bytes(sgx_engine *e, int64_t out[3]) {
    if (!e || !out) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(e->stats_mu);
    for (int i = 0; i < 3; ++i) out[i] = e->x_bytes[i];
    return SGX_OK;
}

extern "C" int sgx_stats_get(sgx_engine *e, double *ms, int64_t *cnt) {
    if (!e || !ms || !cnt) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    e->resolve_stats();
    std::lock_guard<std::mutex> lk(e->stats_mu);
    for (int i = 0; i < SGX_NUM_STAGES; ++i) {
        ms[i] = e->stage_ms[i];
        cnt[i] = e->stage_n[i];
    }
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// generators and memory helpers
// ------------------------------------------------------------------------------------
extern "C" int sgx_gen_uniform16(sgx_engine *e, void *dst, int64_t n, uint64_t seed, int64_t vbase) {
    if (!e || (n > 0 && !dst)) return fail_msg(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    if (n > 0) HIP_TRY(launch_gen_uniform16(dst, n, seed, vbase, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SGX_OK;
}

extern "C" int sgx_gen_zipf16(sgx_engine *e, void *dst, int64_t n, uint64_t seed, int64_t vbase,
                              const double *cdf_host, int64_t K) {
    if (!e || (n > 0 && !dst) || !cdf_host || K < 1) return fail_msg(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    SGX_TRY(c->cdf.ensure((size_t)K * 8));
    HIP_TRY(hipMemcpyAsync(c->cdf.p, cdf_host, (size_t)K * 8, hipMemcpyHostToDevice, c->st));
    if (n > 0) HIP_TRY(launch_gen_zipf16(dst, n, seed, vbase, (const double *)c->cdf.p, K, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SGX_OK;
}

extern "C" int sgx_gen_terasort100(sgx_engine *e, void *dst, int64_t n, uint64_t seed, int64_t ibase) {
    if (!e || (n > 0 && !dst)) return fail_msg(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    if (n > 0) HIP_TRY(launch_gen_terasort100(dst, n, seed, ibase, c->st));
    HIP_TRY(hipStreamSynchronize(c->st));
    return SGX_OK;
}

extern "C" int sgx_device_alloc(sgx_engine *e, int64_t bytes, void **out) {
    if (!e || !out || bytes < 0) return fail_msg(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    hipError_t er = hipMalloc(out, (size_t)(bytes ? bytes : 16));
    if (er != hipSuccess)
        return fail_msg(SGX_ERR_NOMEM, "hipMalloc(%lld): %s", (long long)bytes, hipGetErrorString(er));
    return SGX_OK;
}

extern "C" int sgx_device_free(sgx_engine *e, void *p) {
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    HIP_TRY(hipSetDevice(e->device));
    if (p) HIP_TRY(hipFree(p));
    return SGX_OK;
}

extern "C" int sgx_memcpy(sgx_engine *e, void *dst, const void *src, int64_t bytes) {
    if (!e || bytes < 0) return fail_msg(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    if (bytes > 0) HIP_TRY(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDefault));
    return SGX_OK;
}
