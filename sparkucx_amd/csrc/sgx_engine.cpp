// sgx_engine.cpp — the C-ABI engine behind include/sgx.h.
//
// One engine per GPU (= per Spark executor).  It replaces, on the hot path:
//   * the map-output writer + NVKV storage (ucx/NvkvShuffleMapOutputWriter.scala:105-148,
//     ucx/NvkvHandler.scala:213-265): map outputs are partitioned by HIP kernels and kept
//     resident in HBM, engine-owned;
//   * the index commit (IndexShuffleBlockResolver.scala:161-217) when a file is wanted;
//   * the UCX fetch path (ucx/UcxWorkerWrapper.scala:96-186, spark_3_0/UcxShuffleClient.scala
//     :17-91): one counts all-gather + ncclAllToAllv over xGMI + a regroup kernel, then
//     block fetches are served from HBM.
// There is no CPU fallback: every data-path call runs the HIP kernels or fails.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/sgx.h"
#include "sgx_internal.h"

using namespace sgx;

// ------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------
static thread_local std::string t_last_error;

static int fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_last_error = buf;
    return code;
}

// the same error path for the other host-side translation units (sgx_bootstrap.cpp)
int sgx::fail_msg(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    t_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return fail(SGX_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),    \
                        __FILE__, __LINE__);                                                   \
    } while (0)
#define NCCL_TRY(expr)                                                                         \
    do {                                                                                       \
        ncclResult_t _r = (expr);                                                              \
        if (_r != ncclSuccess)                                                                 \
            return fail(SGX_ERR_COMM, "%s failed: %s", #expr, ncclGetErrorString(_r));          \
    } while (0)
#define SGX_TRY(expr)                                                                          \
    do {                                                                                       \
        int _c = (expr);                                                                       \
        if (_c != SGX_OK) return _c;                                                           \
    } while (0)

// ------------------------------------------------------------------------------------
// device buffers
// ------------------------------------------------------------------------------------
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return SGX_OK;
        release();
        size_t want = bytes ? bytes : 16;
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(SGX_ERR_NOMEM, "hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
        }
        cap = want;
        return SGX_OK;
    }
};

// releases a scratch DevBuf when the scope ends (DevBuf itself is a plain member type)
struct DevBufScope {
    DevBuf &b;
    ~DevBufScope() { b.release(); }
};

struct HostPinned {
    void *p = nullptr;
    size_t cap = 0;
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return SGX_OK;
        release();
        size_t want = bytes ? bytes : 16;
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(SGX_ERR_NOMEM, "hipHostMalloc(%zu) failed: %s", want, hipGetErrorString(e));
        }
        cap = want;
        return SGX_OK;
    }
};

// ------------------------------------------------------------------------------------
// registry
// ------------------------------------------------------------------------------------
struct MapOut {
    DevBuf data;               // partition-contiguous records (engine-owned HBM)
    int64_t nrec = 0;
    int64_t bytes = 0;
    HostPinned part_off;       // (R+1) u32 record offsets + 1 u32 error word, landed async
    std::vector<int64_t> lengths;  // bytes per partition (valid once `ready`)
    bool ready = false;
    hipEvent_t done = nullptr;  // recorded on the compute stream after the scatter
    hipEvent_t read_done = nullptr;  // recorded on the exchange stream after the all-to-all read `data`
    // serializer KRYO (sgx_set_serializer): the map's published bytes are the Kryo stream of
    // its records (data file, fetch, exchange); `data` keeps the 16 B records
    DevBuf ser;                // Kryo-framed partition-contiguous bytes (capacity 20 n + 16)
    DevBuf ser_work;           // ser_off_dev (R+1) i64 | tile prefixes, block totals u64 | tile sums u32
    HostPinned ser_off;        // (R+1) i64 byte offsets + the error word, landed async
    int64_t out_bytes = 0;     // published bytes (n * rb, or the Kryo total once `ready`)
    DevBuf comp;               // LZ4-framed partition streams (sgx_set_compression), once `ready`
    const void *view() const { return comp.p ? comp.p : (ser.p ? ser.p : data.p); }
};

// One exchange round: every rank pushed one map; this rank holds its reducers' blocks.
// The receive buffer keeps ncclAllToAllv's layout, [source rank][my reducers]: every
// (map, reducer) block is contiguous in it, so blocks are served from it directly and the
// per-reducer canonical order (reducer, then source map) is produced by the fetch that
// asks for it (one gather launch), not by an extra pass over every received byte.
struct Round {
    std::vector<int64_t> map_ids;        // [P] the map pushed by each source rank
    std::vector<int64_t> lens;           // [P][R] bytes
    std::vector<int64_t> block_off;      // [P][nmine] byte offset in `data`
    int32_t r0 = 0, r1 = 0;              // my reducers [r0, r1)
    DevBuf data;                          // receive buffer, [source][my reducers]
    const void *alias = nullptr;          // P == 1: the local map output itself
    hipEvent_t done = nullptr;
    const void *base() const { return alias ? alias : data.p; }
};

struct Shuffle {
    int32_t R = 0, kind = 0, nb = 0, asc = 1, rb = 16;
    int32_t ser = SGX_SER_FIXED;  // dep.serializer (sgx_set_serializer)
    int32_t lz4_block = 0;        // spark.shuffle.compress with lz4 (sgx_set_compression): block size
    DevBuf bounds;
    PartParams pp{};
    std::map<int64_t, std::unique_ptr<MapOut>> maps;
    std::vector<std::unique_ptr<Round>> rounds;
};

struct PendingStage {
    int stage;
    hipEvent_t a, b;
};

struct sgx_engine {
    std::mutex mu;
    int device = 0;
    int num_cus = 256;
    int G = 256;
    bool G_forced = false;
    int sc_waves = 0, sc_items = 0;  // K4 geometry override
    int diag = 0;                    // SGX_SCATTER_DIAG: measurement-only K4 ablation (wrong output)
    int no_table = 0;                // SGX_NO_PEER_TABLE=1: ballots-only ranking (A/B)
    int direct = 0;                  // SGX_SCATTER_DIRECT=WWII: direct-store K4 (A/B)
    int use_dma = 0;                 // SGX_SCATTER_DMA=1: LDS-DMA pipelined K4 (A/B)
    int rank_match = 0;              // SGX_RANK=match: ballot/peer-table ranking in K4
    int nt = 0;                      // SGX_SCATTER_NT=1/2/3: nontemporal loads/stores; 4: double-buffered (A/B)
    int chain = 0;                   // SGX_SCATTER_CHAIN=WWII: chained look-back K4 (A/B)
    int wc = 1;                      // SGX_SCATTER_WC=0: no write-combining K4 (A/B)
    int wide2 = 1;                   // SGX_SCATTER_WIDE2=0: per-lane wide-record K4 (A/B)
    int wc_diag = 0;                 // SGX_WC_DIAG=1..3: measurement-only ablation of the wc K4 (wrong output)
    hipStream_t s_comp = nullptr, s_comm = nullptr;
    // work buffers of the map-side pipeline
    // map-side work buffers, a ring of two: with SGX_PIPELINE the next map's histogram +
    // scan (on s_hist) fill one set while the previous map's scatter (on s_comp) reads the other
    struct WorkSet {
        DevBuf offs, status;  // status: counts | ticket | look-back status | partition offsets | error
        hipEvent_t used = nullptr;  // recorded on s_comp after the scatter that read this set
    } ws[2];
    int ws_next = 0;
    int pipeline = 0;                // SGX_PIPELINE=1: hist+scan of map k+1 overlap map k's scatter
    hipStream_t s_hist = nullptr;
    DevBuf input_stage, junk;
    const uint32_t *last_off_dev = nullptr;  // device (R+1) record offsets of the last partition pass
    // reduce side: sort ping-pong buffers, per-pass error words, grouping work buffers
    DevBuf kryo_in, kryo_work;  // reduce side of a Kryo shuffle: fetched stream, decoder state
    DevBuf sort_buf[2], sort_err, grp_flags, grp_offs, grp_status, grp_out, grp_prefix;
    // RangePartitioner.sketch: XORShiftRandom jump table, reservoir winners and keys
    DevBuf jump_dev, sample_winner, sample_keys;
    DevBuf digit_hist;               // sorted read: [digits][256] histogram of the fetched keys
    int sort_skip = 1;               // SGX_SORT_SKIP=0: run every digit pass (A/B, tests)
    int hist_variant = 0;            // SGX_HIST_VARIANT=2..6: histogram geometry A/B
    DevBuf ag_send, ag_recv, recv, items_dev, chain_buf, gather_stage;
    HostPinned gather_items;
    HostPinned ag_host;
    std::map<int32_t, Shuffle> shuffles;
    // RCCL
    ncclComm_t comm = nullptr;
    int32_t nranks = 1, rank = 0;
    // stats
    std::vector<hipEvent_t> ev_free;
    std::vector<PendingStage> pending;
    double stage_ms[SGX_NUM_STAGES] = {0};
    int64_t stage_n[SGX_NUM_STAGES] = {0};

    hipEvent_t ev() {
        if (!ev_free.empty()) {
            hipEvent_t e = ev_free.back();
            ev_free.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
    void resolve_stats() {
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
};

static uint32_t bits_for(uint32_t R) {
    uint32_t b = 0;
    while ((1ull << b) < R) ++b;
    return b ? b : 1;
}

static PartParams make_part_params(const Shuffle &s) {
    PartParams pp{};
    pp.kind = s.kind;
    pp.R = (uint32_t)s.R;
    mod_params((uint32_t)s.R, &pp.mg_m, &pp.mg_s);
    pp.c31 = (uint32_t)((1ull << 31) % (uint64_t)s.R);
    pp.nbits = bits_for((uint32_t)s.R);
    pp.nb = s.nb;
    pp.ascending = s.asc;
    pp.bounds = s.bounds.p;
    return pp;
}

// ------------------------------------------------------------------------------------
// lifetime
// ------------------------------------------------------------------------------------
extern "C" const char *sgx_last_error(void) { return t_last_error.c_str(); }
extern "C" int32_t sgx_abi_version(void) { return SGX_ABI_VERSION; }

extern "C" int sgx_create(const sgx_config *cfg, sgx_engine **out) {
    if (!out) return fail(SGX_ERR_INVALID, "sgx_create: out is NULL");
    *out = nullptr;
    int dev = cfg ? cfg->device : 0;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (dev < 0 || dev >= ndev) return fail(SGX_ERR_INVALID, "sgx_create: device %d of %d", dev, ndev);
    HIP_TRY(hipSetDevice(dev));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, dev));
    std::unique_ptr<sgx_engine> e(new sgx_engine());
    e->device = dev;
    e->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    e->G = (cfg && cfg->num_chunks > 0) ? cfg->num_chunks : e->num_cus;
    e->G_forced = cfg && cfg->num_chunks > 0;
    e->sc_waves = cfg ? cfg->scatter_waves : 0;
    e->sc_items = cfg ? cfg->scatter_items : 0;
    if (const char *d = getenv("SGX_SCATTER_DIAG")) e->diag = atoi(d);
    if (const char *d = getenv("SGX_NO_PEER_TABLE")) e->no_table = atoi(d);
    if (const char *d = getenv("SGX_SCATTER_DIRECT")) e->direct = atoi(d);
    if (const char *d = getenv("SGX_SCATTER_DMA")) e->use_dma = atoi(d);
    if (const char *d = getenv("SGX_SCATTER_NT")) e->nt = atoi(d);
    if (const char *d = getenv("SGX_RANK")) e->rank_match = std::strcmp(d, "match") == 0;
    if (const char *d = getenv("SGX_SCATTER_CHAIN")) e->chain = atoi(d);
    if (const char *d = getenv("SGX_SCATTER_WC")) e->wc = atoi(d);
    if (const char *d = getenv("SGX_SCATTER_WIDE2")) e->wide2 = atoi(d);
    if (const char *d = getenv("SGX_WC_DIAG")) e->wc_diag = atoi(d);
    HIP_TRY(hipStreamCreateWithFlags(&e->s_comp, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&e->s_comm, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&e->s_hist, hipStreamNonBlocking));
    if (const char *d = getenv("SGX_PIPELINE")) e->pipeline = atoi(d);
    if (const char *d = getenv("SGX_SORT_SKIP")) e->sort_skip = atoi(d);
    if (const char *d = getenv("SGX_HIST_VARIANT")) e->hist_variant = atoi(d);
    *out = e.release();
    return SGX_OK;
}

static void free_map(MapOut &m) {
    if (m.read_done) (void)hipEventSynchronize(m.read_done);  // an all-to-all may still read `data`
    if (m.read_done) (void)hipEventDestroy(m.read_done);
    m.read_done = nullptr;
    m.data.release();
    m.part_off.release();
    m.ser.release();
    m.comp.release();
    m.ser_work.release();
    m.ser_off.release();
    if (m.done) (void)hipEventDestroy(m.done);
    m.done = nullptr;
}
static void free_round(Round &r) {
    r.data.release();
    if (r.done) (void)hipEventDestroy(r.done);
    r.done = nullptr;
}

extern "C" void sgx_destroy(sgx_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    (void)hipDeviceSynchronize();
    e->resolve_stats();
    for (auto &kv : e->shuffles) {
        for (auto &m : kv.second.maps) free_map(*m.second);
        for (auto &r : kv.second.rounds) free_round(*r);
        kv.second.bounds.release();
    }
    for (auto &w : e->ws) {
        for (DevBuf *b : {&w.offs, &w.status}) b->release();
        if (w.used) (void)hipEventDestroy(w.used);
        w.used = nullptr;
    }
    for (DevBuf *b : {&e->kryo_in, &e->kryo_work, &e->sort_buf[0], &e->sort_buf[1], &e->sort_err, &e->grp_flags, &e->grp_offs, &e->grp_status,
                      &e->grp_out, &e->grp_prefix, &e->jump_dev, &e->sample_winner, &e->sample_keys,
                      &e->digit_hist})
        b->release();
    for (DevBuf *b : {&e->junk, &e->input_stage, &e->ag_send,
                      &e->ag_recv, &e->recv, &e->items_dev, &e->chain_buf, &e->gather_stage})
        b->release();
    e->ag_host.release();
    e->gather_items.release();
    for (hipEvent_t ev : e->ev_free) (void)hipEventDestroy(ev);
    if (e->comm) (void)ncclCommDestroy(e->comm);
    (void)hipStreamDestroy(e->s_comp);
    (void)hipStreamDestroy(e->s_comm);
    (void)hipStreamDestroy(e->s_hist);
    delete e;
}

// ------------------------------------------------------------------------------------
// registerShuffle / unregisterShuffle
// ------------------------------------------------------------------------------------
static int max_partitions(int kind, int rb) {
    (void)kind;
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
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    if (R < 1) return fail(SGX_ERR_INVALID, "numPartitions must be positive, got %d", R);
    if (kind < SGX_PART_HASH || kind > SGX_PART_RANGE_BYTES10)
        return fail(SGX_ERR_INVALID, "unknown partitioner kind %d", kind);
    if (rb < 12 || (rb & 3) != 0)
        return fail(SGX_ERR_INVALID, "record_bytes must be a multiple of 4 and >= 12, got %d", rb);
    if (kind != SGX_PART_HASH && nbounds != (int64_t)R - 1)
        return fail(SGX_ERR_INVALID, "RangePartitioner needs numPartitions == bounds+1 (%d vs %lld)",
                    R, (long long)nbounds);
    if (kind != SGX_PART_HASH && nbounds > 0 && !bounds)
        return fail(SGX_ERR_INVALID, "range bounds pointer is NULL");
    const int rmax = max_partitions(kind, rb);
    if (R > rmax)
        return fail(SGX_ERR_UNSUPPORTED, "numPartitions %d exceeds the single-pass LDS limit %d", R, rmax);
    if (e->shuffles.count(shuffle_id))
        return fail(SGX_ERR_STATE, "shuffle %d is already registered", shuffle_id);
    HIP_TRY(hipSetDevice(e->device));
    Shuffle &s = e->shuffles[shuffle_id];
    s.R = R;
    s.kind = kind;
    s.nb = (int32_t)(kind == SGX_PART_HASH ? 0 : nbounds);
    s.asc = ascending ? 1 : 0;
    s.rb = rb;
    if (kind == SGX_PART_RANGE_I64 && nbounds > 0) {
        int rc = s.bounds.ensure((size_t)nbounds * 8);
        if (rc) { e->shuffles.erase(shuffle_id); return rc; }
        HIP_TRY(hipMemcpy(s.bounds.p, bounds, (size_t)nbounds * 8, hipMemcpyHostToDevice));
    } else if (kind == SGX_PART_RANGE_BYTES10 && nbounds > 0) {
        std::vector<Key10> k((size_t)nbounds);
        const uint8_t *b = (const uint8_t *)bounds;
        for (int64_t i = 0; i < nbounds; ++i) {
            const uint8_t *q = b + 10 * i;
            uint64_t hi = 0;
            for (int j = 0; j < 8; ++j) hi = (hi << 8) | q[j];
            k[(size_t)i] = Key10{hi, ((uint32_t)q[8] << 8) | q[9], 0};
        }
        int rc = s.bounds.ensure((size_t)nbounds * sizeof(Key10));
        if (rc) { e->shuffles.erase(shuffle_id); return rc; }
        HIP_TRY(hipMemcpy(s.bounds.p, k.data(), k.size() * sizeof(Key10), hipMemcpyHostToDevice));
    }
    s.pp = make_part_params(s);
    return SGX_OK;
}

extern "C" int sgx_unregister_shuffle(sgx_engine *e, int32_t shuffle_id) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->s_comp));
    HIP_TRY(hipStreamSynchronize(e->s_comm));
    for (auto &m : it->second.maps) free_map(*m.second);
    for (auto &r : it->second.rounds) free_round(*r);
    it->second.bounds.release();
    e->shuffles.erase(it);
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// map-side write: K1+K2 hist -> K3 scan -> K4 scatter (all on the compute stream)
// ------------------------------------------------------------------------------------
static int lz4_frame_impl(sgx_engine *e, const void *stream_dev, const int64_t *part_offsets, int32_t R,
                          int32_t block_size, DevBuf *alloc_dst, void *dst_dev, int64_t dst_cap,
                          int64_t *out_lengths);

static int lz4_unframe_impl(sgx_engine *e, const void *framed_dev, int64_t framed_bytes, DevBuf *alloc_dst,
                            void *dst_dev, int64_t dst_cap, int64_t *out_bytes);

static int finish_lengths(sgx_engine *e, Shuffle &s, MapOut &m) {
    if (m.ready) return SGX_OK;
    HIP_TRY(hipEventSynchronize(m.done));
    const uint32_t *po = (const uint32_t *)m.part_off.p;
    if (po[s.R + 1] & 1u) return fail(SGX_ERR_TIMEOUT, "scan look-back spin gave up (device flag %u)", po[s.R + 1]);
    if (po[s.R + 1] & 2u)
        return fail(SGX_ERR_HIP, "internal error: a scatter destination was out of range (device flag %u)",
                    po[s.R + 1]);
    if ((int64_t)po[s.R] != m.nrec)
        return fail(SGX_ERR_HIP, "partition offsets do not sum to the record count (%u vs %lld)", po[s.R],
                    (long long)m.nrec);
    m.lengths.assign((size_t)s.R, 0);
    if (s.ser == SGX_SER_KRYO) {
        const int64_t *so = (const int64_t *)m.ser_off.p;
        int64_t prev = 0;
        for (int32_t p = 0; p < s.R; ++p) {
            m.lengths[(size_t)p] = so[p + 1] - so[p];
            if (so[p] != prev || m.lengths[(size_t)p] < 0 || m.lengths[(size_t)p] > 20 * ((int64_t)po[p + 1] - po[p]))
                return fail(SGX_ERR_HIP, "internal error: Kryo partition offsets inconsistent at %d", p);
            prev = so[p + 1];
        }
        m.out_bytes = so[s.R];
    } else {
        for (int32_t p = 0; p < s.R; ++p) m.lengths[(size_t)p] = ((int64_t)po[p + 1] - (int64_t)po[p]) * s.rb;
        m.out_bytes = m.nrec * s.rb;
    }
    if (s.lz4_block > 0) {  // publish the LZ4-framed partition streams instead
        std::vector<int64_t> offs((size_t)s.R + 1, 0);
        for (int32_t p = 0; p < s.R; ++p) offs[(size_t)p + 1] = offs[(size_t)p] + m.lengths[(size_t)p];
        std::vector<int64_t> clen((size_t)s.R, 0);
        SGX_TRY(lz4_frame_impl(e, m.view(), offs.data(), s.R, s.lz4_block, &m.comp, nullptr, 0, clen.data()));
        int64_t total = 0;
        for (int32_t p = 0; p < s.R; ++p) total += clen[(size_t)p];
        m.lengths = clen;
        m.out_bytes = total;
    }
    m.ready = true;
    return SGX_OK;
}

static void record_stage(sgx_engine *e, int stage, hipEvent_t a, hipEvent_t b) {
    e->pending.push_back(PendingStage{stage, a, b});
}

// One stable partition pass (K1+K2 hist -> K3 scan -> K4 scatter) of `n` records of `rb`
// bytes from device memory `in` to `out` under partitioner `spp` (R partitions, `kind`, `nb`
// range bounds).  Asynchronous on e->s_comp (the histogram + scan on e->s_hist when the
// pipelined mode applies).  The (R+1) record offsets and the device error word land in
// `host_off` (R+2 u32, pinned) when given; the error word alone in `err_slot` (device) when
// given.  `stats` records the per-stage events.
static int partition_pass(sgx_engine *e, const void *in, void *out, int64_t n, int rb, const PartParams &spp,
                          int32_t R, int32_t kind, int32_t nb, int32_t mem_kind, uint32_t *host_off,
                          uint32_t *err_slot, bool stats) {
    hipStream_t st = e->s_comp;
    // chunking: G chunks, each a whole number of scatter tiles where possible
    ScatterGeom geo = rb == 16 ? scatter_geom16((uint32_t)R, e->sc_waves, e->sc_items)
                               : scatter_geom_wide((uint32_t)R, rb);
    if (e->diag > 0 && rb == 16) geo = scatter_geom16((uint32_t)R, 8, 16);
    // experiment hook: SGX_SCATTER_DIRECT=<waves><items as 2 digits> selects the direct kernel
    if (e->direct > 0 && rb == 16) {
        const ScatterGeom d = scatter_geom16_direct((uint32_t)R, e->direct / 100, e->direct % 100);
        if (d.items) geo = d;
    }
    if (rb == 16 && kind == SGX_PART_HASH && e->sc_waves == 0 && e->sc_items == 0 && e->diag == 0 &&
        e->direct == 0 && e->use_dma) {
        const ScatterGeom d = scatter_geom16_dma((uint32_t)R);
        if (d.items) geo = d;
    }
    geo.nt = e->nt;
    // default K4 for hash partitioners: lane-ordered ranking (SGX_RANK=match keeps the
    // ballot/peer-table ranker; the A/B kernels above keep theirs)
    if (rb == 16 && kind == SGX_PART_HASH && !e->rank_match && e->diag == 0 && e->direct == 0 &&
        !e->use_dma && e->nt == 0 && e->chain == 0) {
        const ScatterGeom o = scatter_geom16_ord((uint32_t)R, e->sc_waves, e->sc_items);
        if (o.items) geo = o;
        // write-combining K4 (whole 128 B lines only) where its LDS fits (R <= 1024)
        if (e->wc && e->sc_waves == 0 && e->sc_items == 0) {
            ScatterGeom w = scatter_geom16_wc((uint32_t)R);
            if ((e->wc_diag >= 1 && e->wc_diag <= 4) || e->wc_diag == 8 || e->wc_diag == 16 || e->wc_diag == 32 ||
                e->wc_diag == 64 || e->wc_diag == 96)
                w.nt = 100 + e->wc_diag;
            if (w.items) geo = w;
        }
    }
    // wide records: the LDS-staged dword-stream kernel where it applies (16 B-aligned input)
    if (rb != 16 && e->wide2 && ((uintptr_t)in & 15) == 0) {
        const ScatterGeom w2 = scatter_geom_wide2((uint32_t)R, rb, kind, nb);
        if (w2.items) geo = w2;
    }
    // the reduce side's digit passes run on the write-combining / wide-record kernels only
    if (kind == KIND_DIGIT) {
        if (rb == 16) geo = scatter_geom16_wc((uint32_t)R);
        if (geo.waves < WC_GEOM_BASE && geo.waves != WIDE2_GEOM_TAG)
            return fail(SGX_ERR_UNSUPPORTED, "digit pass on %d B records at this alignment", rb);
    }
    if (geo.items == 0)
        return fail(SGX_ERR_UNSUPPORTED, "no scatter geometry (waves %d, items %d) fits R=%d", e->sc_waves,
                    e->sc_items, R);
    const int tile = geo.tile;
    int Gt = e->G;
    if (is_direct_geom(geo.waves) && !e->G_forced) {
        // several direct-store workgroups per CU: one chunk per resident workgroup
        const int wv = geo.waves - DIRECT_GEOM_BASE;
        int occ = (int)((160 * 1024) / geo.lds_bytes);
        if (occ > 32 / wv) occ = 32 / wv;
        Gt = e->num_cus * (occ > 0 ? occ : 1);
    }
    int64_t chunk = n > 0 ? (n + Gt - 1) / Gt : 1;
    chunk = (chunk + tile - 1) / tile * tile;
    const int G = n > 0 ? (int)((n + chunk - 1) / chunk) : 1;
    const int64_t len = (int64_t)R * G;
    const int64_t tiles = scan_tiles(len);
    // the pipelined map side: device input, and the write-combining K4 it was sized for
    const bool pipe = e->pipeline && mem_kind == SGX_MEM_DEVICE && rb == 16 && geo.waves >= WC_GEOM_BASE &&
                      e->diag == 0 && e->chain == 0;
    auto &W = e->ws[pipe ? (e->ws_next ^= 1) : 0];
    hipStream_t sh = pipe ? e->s_hist : st;
    if (pipe && W.used) HIP_TRY(hipStreamWaitEvent(sh, W.used, 0));  // its last reader (K4) is done
    SGX_TRY(W.offs.ensure((size_t)len * 4));
    // one work block, zeroed by ONE memset (each fill / copy between kernels costs ~5-10 µs):
    // [counts u32 x R*G][ticket u32 | pad][look-back status u64 x tiles]
    // [partition offsets u32 x (R+1) | error] -- the error word sits right after the
    // offsets so one copy lands both on the host
    const size_t counts_bytes = ((size_t)len * 4 + 15) & ~(size_t)15;
    const size_t status_bytes = ((size_t)(16 + tiles * 8) + 15) & ~(size_t)15;
    const size_t work_bytes = counts_bytes + status_bytes + (((size_t)(R + 2) * 4 + 15) & ~(size_t)15);
    SGX_TRY(W.status.ensure(work_bytes));
    uint32_t *counts = (uint32_t *)W.status.p;
    uint32_t *ticket = (uint32_t *)((char *)W.status.p + counts_bytes);
    uint64_t *status = (uint64_t *)((char *)ticket + 16);
    uint32_t *part_off_dev = (uint32_t *)((char *)ticket + status_bytes);
    uint32_t *err = part_off_dev + R + 1;
    e->last_off_dev = part_off_dev;
    HIP_TRY(hipMemsetAsync(W.status.p, 0, work_bytes, sh));

    // stage events: consecutive stages on one stream share their boundary event (every
    // timing marker between two kernels measured ~5 µs of idle GPU); the pipelined mode's
    // stages sit on two streams and keep their own pairs
    hipEvent_t h0 = e->ev(), h1 = e->ev(), c0 = pipe ? e->ev() : h1, c1 = e->ev(), x0 = pipe ? e->ev() : c1,
               x1 = e->ev();
    HIP_TRY(hipEventRecord(h0, sh));
    if (n > 0) {
        HIP_TRY(launch_hist(in, n, rb, chunk, G, spp, counts, sh, pipe ? 1 : e->hist_variant, true));
    }
    HIP_TRY(hipEventRecord(h1, sh));
    if (c0 != h1) HIP_TRY(hipEventRecord(c0, sh));
    HIP_TRY(launch_scan((const uint32_t *)counts, (uint32_t *)W.offs.p, len, status, ticket, err,
                        part_off_dev, G, R, sh));
    HIP_TRY(hipEventRecord(c1, sh));
    if (pipe) HIP_TRY(hipStreamWaitEvent(st, c1, 0));
    if (x0 != c1) HIP_TRY(hipEventRecord(x0, st));
    PartParams lpp = spp;
    SGX_TRY(e->junk.ensure((size_t)G * JUNK_BYTES_PER_WG));
    lpp.junk = e->junk.p;
    lpp.mbits = e->no_table ? 0u : (uint32_t)geo.mbits;
    if (e->diag > 0) lpp.mbits = e->no_table ? 0u : (uint32_t)scatter_geom16((uint32_t)R, 8, 16).mbits;
    const int cw = e->chain / 100, ci = e->chain % 100;
    const ScatterGeom cg = (e->chain > 0 && rb == 16) ? scatter_geom16((uint32_t)R, cw, ci) : ScatterGeom{0, 0, 0, 0, 0};
    if (n > 0 && cg.items > 0 && n < (1ll << 30)) {
        // chained K4: tiles in ticket order, per-partition decoupled look-back across tiles
        int mb = e->no_table ? 0 : cg.mbits;
        while (mb > 0 && scatter16_chain_lds((uint32_t)R, cw, ci, mb) > 160 * 1024) --mb;
        PartParams cpp = spp;
        cpp.mbits = (uint32_t)mb;
        const int ctile = cw * ci * 64;
        const int64_t ntiles = (n + ctile - 1) / ctile;
        const size_t sbytes = 16 + (size_t)ntiles * (size_t)R * 4;
        SGX_TRY(e->chain_buf.ensure(sbytes));
        HIP_TRY(hipMemsetAsync(e->chain_buf.p, 0, sbytes, st));
        int occ = (int)((160 * 1024) / scatter16_chain_lds((uint32_t)R, cw, ci, mb));
        if (occ > 32 / cw) occ = 32 / cw;
        if (occ < 1) occ = 1;
        HIP_TRY(launch_scatter_chain(in, out, n, cpp, (const uint32_t *)part_off_dev,
                                     (uint32_t *)((char *)e->chain_buf.p + 16), (uint32_t *)e->chain_buf.p,
                                     err, cw, ci, e->num_cus * occ, st));
    } else if (n > 0) {
        if (e->diag > 0 && rb == 16 && kind == SGX_PART_HASH)  // measurement-only ablation
            HIP_TRY(launch_scatter_diag(e->diag, in, out, n, chunk, G, lpp, (const uint32_t *)W.offs.p, err, st));
        else
            HIP_TRY(launch_scatter(in, out, n, rb, chunk, G, lpp, (const uint32_t *)W.offs.p, geo, err, st));
    }
    HIP_TRY(hipEventRecord(x1, st));
    // (R+1) offsets then the error word, one copy
    if (host_off) HIP_TRY(hipMemcpyAsync(host_off, part_off_dev, (size_t)(R + 2) * 4, hipMemcpyDeviceToHost, st));
    if (err_slot) HIP_TRY(hipMemcpyAsync(err_slot, err, 4, hipMemcpyDeviceToDevice, st));
    if (pipe) {
        if (!W.used) HIP_TRY(hipEventCreateWithFlags(&W.used, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(W.used, st));
    }
    if (stats) {
        record_stage(e, SGX_STAGE_HIST, h0, h1);
        record_stage(e, SGX_STAGE_SCAN, c0, c1);
        record_stage(e, SGX_STAGE_SCATTER, x0, x1);
    } else {
        for (hipEvent_t v : {h0, h1, c1, x1}) e->ev_free.push_back(v);
        if (pipe) for (hipEvent_t v : {c0, x0}) e->ev_free.push_back(v);
    }
    return SGX_OK;
}

// Kryo framing of the partition-contiguous 16 B records just written (sgx_serde.hip), on
// the compute stream behind the scatter; byte offsets land in m.ser_off (pinned).
static int serialize_kryo(sgx_engine *e, Shuffle &s, MapOut &m) {
    hipStream_t st = e->s_comp;
    const int64_t n = m.nrec;
    const int64_t tiles = kryo_ser16_tiles(n);
    const size_t offb = (size_t)(s.R + 1) * 8;
    SGX_TRY(m.ser.ensure((size_t)(20 * n + 16)));
    SGX_TRY(m.ser_work.ensure(offb + (size_t)kryo_work_bytes(tiles)));
    SGX_TRY(m.ser_off.ensure(offb));
    int64_t *off_dev = (int64_t *)m.ser_work.p;
    uint64_t *work = (uint64_t *)((char *)m.ser_work.p + offb);
    if (n == 0) HIP_TRY(hipMemsetAsync(off_dev, 0, offb, st));  // no tile writes them
    hipEvent_t k0 = e->ev(), k1 = e->ev();
    HIP_TRY(hipEventRecord(k0, st));
    HIP_TRY(launch_kryo_ser16(m.data.p, n, m.ser.p, e->last_off_dev, s.R, off_dev, work, st));
    HIP_TRY(hipEventRecord(k1, st));
    record_stage(e, SGX_STAGE_SERIALIZE, k0, k1);
    HIP_TRY(hipMemcpyAsync(m.ser_off.p, off_dev, offb, hipMemcpyDeviceToHost, st));  // (R+1) byte offsets
    return SGX_OK;
}

extern "C" int sgx_set_serializer(sgx_engine *e, int32_t shuffle_id, int32_t serializer) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    Shuffle &s = it->second;
    if (serializer != SGX_SER_FIXED && serializer != SGX_SER_KRYO)
        return fail(SGX_ERR_INVALID, "unknown serializer %d", serializer);
    if (!s.maps.empty()) return fail(SGX_ERR_STATE, "shuffle %d already has map outputs", shuffle_id);
    if (serializer == SGX_SER_KRYO && (s.rb != 16 || s.kind == SGX_PART_RANGE_BYTES10))
        return fail(SGX_ERR_UNSUPPORTED, "Kryo framing is for (Long, Long) 16 B records, not %d B", s.rb);
    s.ser = serializer;
    return SGX_OK;
}

extern "C" int sgx_set_compression(sgx_engine *e, int32_t shuffle_id, int32_t codec, int32_t block_size) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    Shuffle &s = it->second;
    if (codec != SGX_CODEC_NONE && codec != SGX_CODEC_LZ4) return fail(SGX_ERR_INVALID, "unknown codec %d", codec);
    if (!s.maps.empty()) return fail(SGX_ERR_STATE, "shuffle %d already has map outputs", shuffle_id);
    if (codec == SGX_CODEC_LZ4) {
        if (s.ser != SGX_SER_KRYO)
            return fail(SGX_ERR_UNSUPPORTED, "LZ4 compression is published over the Kryo stream (sgx_set_serializer first)");
        if (block_size < 64 || block_size > sgx::lz4_max_block())
            return fail(SGX_ERR_UNSUPPORTED, "LZ4 block size %d outside [64, %d]", block_size, sgx::lz4_max_block());
    }
    s.lz4_block = codec == SGX_CODEC_LZ4 ? block_size : 0;
    return SGX_OK;
}

extern "C" int sgx_write_map(sgx_engine *e, int32_t shuffle_id, int64_t map_id, const void *records,
                             int64_t n, int32_t rb, int32_t mem_kind, int64_t *out_lengths) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    Shuffle &s = it->second;
    if (rb != s.rb) return fail(SGX_ERR_INVALID, "record_bytes %d != registered %d", rb, s.rb);
    if (n < 0 || n >= (int64_t)UINT32_MAX) return fail(SGX_ERR_INVALID, "nrecords %lld out of range", (long long)n);
    if (n > 0 && !records) return fail(SGX_ERR_INVALID, "records is NULL");
    if (mem_kind != SGX_MEM_HOST && mem_kind != SGX_MEM_DEVICE)
        return fail(SGX_ERR_INVALID, "unknown mem_kind %d", mem_kind);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t st = e->s_comp;

    std::unique_ptr<MapOut> &slot = s.maps[map_id];
    if (!slot) slot.reset(new MapOut());
    MapOut &m = *slot;
    // A re-attempt of the same map replaces the previous output (the in-HBM analogue of the
    // index commit; the file commit keeps "first valid attempt wins", sgx_write_index).
    if (m.done) HIP_TRY(hipEventSynchronize(m.done));
    // ... and must not overwrite the previous output while an exchange still sends it
    if (m.read_done) HIP_TRY(hipStreamWaitEvent(st, m.read_done, 0));
    m.ready = false;
    if (s.ser != SGX_SER_KRYO) m.ser.release();
    m.nrec = n;
    m.bytes = n * rb;
    SGX_TRY(m.data.ensure((size_t)m.bytes));
    SGX_TRY(m.part_off.ensure((size_t)(s.R + 2) * 4));
    if (!m.done) HIP_TRY(hipEventCreateWithFlags(&m.done, hipEventDisableTiming));

    const void *in = records;
    if (mem_kind == SGX_MEM_HOST && n > 0) {
        SGX_TRY(e->input_stage.ensure((size_t)m.bytes));
        HIP_TRY(hipMemcpyAsync(e->input_stage.p, records, (size_t)m.bytes, hipMemcpyHostToDevice, st));
        in = e->input_stage.p;
    }

    SGX_TRY(partition_pass(e, in, m.data.p, n, rb, s.pp, s.R, s.kind, s.nb, mem_kind, (uint32_t *)m.part_off.p,
                           nullptr, true));
    if (s.ser == SGX_SER_KRYO) SGX_TRY(serialize_kryo(e, s, m));
    HIP_TRY(hipEventRecord(m.done, st));
    if (out_lengths) {
        SGX_TRY(finish_lengths(e, s, m));
        std::memcpy(out_lengths, m.lengths.data(), sizeof(int64_t) * (size_t)s.R);
    }
    return SGX_OK;
}

static int find_map(sgx_engine *e, int32_t shuffle_id, int64_t map_id, Shuffle **ps, MapOut **pm) {
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    auto mt = it->second.maps.find(map_id);
    if (mt == it->second.maps.end())
        return fail(SGX_ERR_NOT_FOUND, "map %lld of shuffle %d was not written", (long long)map_id, shuffle_id);
    *ps = &it->second;
    *pm = mt->second.get();
    return SGX_OK;
}

extern "C" int sgx_map_lengths(sgx_engine *e, int32_t shuffle_id, int64_t map_id, int64_t *out) {
    if (!e || !out) return fail(SGX_ERR_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(e->mu);
    Shuffle *s;
    MapOut *m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    SGX_TRY(finish_lengths(e, *s, *m));
    std::memcpy(out, m->lengths.data(), sizeof(int64_t) * (size_t)s->R);
    return SGX_OK;
}

extern "C" int sgx_map_data(sgx_engine *e, int32_t shuffle_id, int64_t map_id, void **ptr, int64_t *bytes) {
    if (!e || !ptr || !bytes) return fail(SGX_ERR_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(e->mu);
    Shuffle *s;
    MapOut *m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    SGX_TRY(finish_lengths(e, *s, *m));
    *ptr = const_cast<void *>(m->view());
    *bytes = m->out_bytes;
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// IndexShuffleBlockResolver: index + data files (IndexShuffleBlockResolver.scala:56-262)
// ------------------------------------------------------------------------------------
static bool read_file(const char *path, std::vector<uint8_t> &out) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    out.clear();
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + k);
    fclose(f);
    return true;
}

static int64_t file_size(const char *path) {
    struct stat st;
    if (stat(path, &st) != 0) return -1;
    return (int64_t)st.st_size;
}

static int64_t load_be64(const uint8_t *p) {
    uint64_t u = 0;
    for (int i = 0; i < 8; ++i) u = (u << 8) | p[i];
    return (int64_t)u;
}

// checkIndexAndDataFile (:110-149): lengths if index and data agree, else false.
static bool check_index_and_data(const char *index_path, const char *data_path, int32_t blocks,
                                 std::vector<int64_t> &lengths) {
    const int64_t isz = file_size(index_path);
    if (isz != ((int64_t)blocks + 1) * 8) return false;
    std::vector<uint8_t> idx;
    if (!read_file(index_path, idx) || (int64_t)idx.size() != isz) return false;
    int64_t off = load_be64(idx.data());
    if (off != 0) return false;
    lengths.assign((size_t)blocks, 0);
    int64_t sum = 0;
    for (int32_t i = 0; i < blocks; ++i) {
        const int64_t nx = load_be64(idx.data() + 8 * (size_t)(i + 1));
        lengths[(size_t)i] = nx - off;
        sum += nx - off;
        off = nx;
    }
    const int64_t dsz = file_size(data_path);
    return dsz >= 0 && dsz == sum;
}

extern "C" int sgx_check_index_and_data(const char *index_path, const char *data_path, int32_t blocks,
                                        int64_t *out_lengths) {
    if (!index_path || !data_path || blocks < 0) return fail(SGX_ERR_INVALID, "bad arguments");
    std::vector<int64_t> l;
    if (!check_index_and_data(index_path, data_path, blocks, l))
        return fail(SGX_ERR_NOT_FOUND, "index %s and data %s do not match for %d blocks", index_path, data_path,
                    blocks);
    if (out_lengths) std::memcpy(out_lengths, l.data(), sizeof(int64_t) * l.size());
    return SGX_OK;
}

extern "C" int sgx_index_block_range(const char *index_path, int32_t start, int32_t end, int64_t *off,
                                     int64_t *len) {
    if (!index_path || !off || !len || start < 0 || end < start)
        return fail(SGX_ERR_INVALID, "bad arguments");
    FILE *f = fopen(index_path, "rb");
    if (!f) return fail(SGX_ERR_IO, "cannot open index %s: %s", index_path, strerror(errno));
    uint8_t a[8], b[8];
    bool ok = fseek(f, (long)start * 8, SEEK_SET) == 0 && fread(a, 1, 8, f) == 8 &&
              fseek(f, (long)end * 8, SEEK_SET) == 0 && fread(b, 1, 8, f) == 8;
    // SPARK-22982 position check: after reading end's long we must sit at end*8+8.
    const bool pos_ok = ok && ftell(f) == (long)end * 8 + 8;
    fclose(f);
    if (!ok) return fail(SGX_ERR_IO, "index %s too short for reduce range [%d, %d)", index_path, start, end);
    if (!pos_ok) return fail(SGX_ERR_IO, "SPARK-22982: incorrect channel position after index file reads");
    *off = load_be64(a);
    *len = load_be64(b) - *off;
    return SGX_OK;
}

static int write_all(const char *path, const void *data, size_t n) {
    int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return fail(SGX_ERR_IO, "cannot create %s: %s", path, strerror(errno));
    const char *p = (const char *)data;
    while (n > 0) {
        ssize_t k = write(fd, p, n);
        if (k < 0) {
            if (errno == EINTR) continue;
            close(fd);
            return fail(SGX_ERR_IO, "write %s: %s", path, strerror(errno));
        }
        p += k;
        n -= (size_t)k;
    }
    if (close(fd) != 0) return fail(SGX_ERR_IO, "close %s: %s", path, strerror(errno));
    return SGX_OK;
}

extern "C" int sgx_write_index(sgx_engine *e, int32_t shuffle_id, int64_t map_id, const char *index_path,
                               const char *data_path, int64_t *out_lengths) {
    if (!e || !index_path || !data_path) return fail(SGX_ERR_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(e->mu);
    Shuffle *s;
    MapOut *m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    SGX_TRY(finish_lengths(e, *s, *m));
    HIP_TRY(hipSetDevice(e->device));
    const std::string data_tmp = std::string(data_path) + ".sgx.tmp";
    const std::string index_tmp = std::string(index_path) + ".sgx.tmp";
    // map output -> data tmp (dataTmp of writeIndexFileAndCommit)
    {
        std::vector<uint8_t> host((size_t)m->out_bytes);
        if (m->out_bytes) HIP_TRY(hipMemcpy(host.data(), m->view(), (size_t)m->out_bytes, hipMemcpyDeviceToHost));
        SGX_TRY(write_all(data_tmp.c_str(), host.data(), host.size()));
    }
    std::vector<int64_t> existing;
    if (check_index_and_data(index_path, data_path, s->R, existing)) {
        // another attempt already committed: use its lengths, drop our data
        unlink(data_tmp.c_str());
        if (out_lengths) std::memcpy(out_lengths, existing.data(), sizeof(int64_t) * existing.size());
        return SGX_OK;
    }
    std::vector<uint8_t> idx((size_t)(s->R + 1) * 8);
    int64_t off = 0;
    for (int32_t i = 0; i <= s->R; ++i) {
        if (i > 0) off += m->lengths[(size_t)i - 1];
        uint64_t u = (uint64_t)off;
        for (int b = 7; b >= 0; --b) { idx[(size_t)i * 8 + (size_t)b] = (uint8_t)(u & 0xFF); u >>= 8; }
    }
    int rc = write_all(index_tmp.c_str(), idx.data(), idx.size());
    if (rc) { unlink(data_tmp.c_str()); return rc; }
    unlink(index_path);
    unlink(data_path);
    if (rename(index_tmp.c_str(), index_path) != 0) {
        unlink(index_tmp.c_str());
        unlink(data_tmp.c_str());
        return fail(SGX_ERR_IO, "fail to rename file %s to %s", index_tmp.c_str(), index_path);
    }
    if (rename(data_tmp.c_str(), data_path) != 0) {
        unlink(data_tmp.c_str());
        return fail(SGX_ERR_IO, "fail to rename file %s to %s", data_tmp.c_str(), data_path);
    }
    if (out_lengths) std::memcpy(out_lengths, m->lengths.data(), sizeof(int64_t) * (size_t)s->R);
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// exchange planning (pure host)
// ------------------------------------------------------------------------------------
extern "C" int32_t sgx_reducer_owner(int32_t r, int32_t R, int32_t P) {
    return (int32_t)(((int64_t)r * P) / R);
}

static void my_reducers(int32_t R, int32_t P, int32_t rank, int32_t *r0, int32_t *r1) {
    // owner(r) = floor(r*P/R) is monotone: [r0, r1) = { r : owner(r) == rank }
    int32_t lo = (int32_t)(((int64_t)rank * R + P - 1) / P);
    int32_t hi = (int32_t)(((int64_t)(rank + 1) * R + P - 1) / P);
    *r0 = std::min(lo, R);
    *r1 = std::min(hi, R);
}

extern "C" int sgx_plan_exchange(const int64_t *L, int32_t P, int32_t R, int32_t rank, int64_t item_bytes,
                                 int64_t *send_counts, int64_t *send_displs, int64_t *recv_counts,
                                 int64_t *recv_displs, int64_t *items, int64_t *n_items) {
    if (!L || P < 1 || R < 1 || rank < 0 || rank >= P || !send_counts || !send_displs || !recv_counts ||
        !recv_displs || !n_items)
        return fail(SGX_ERR_INVALID, "sgx_plan_exchange: bad arguments");
    const int64_t *mine = L + (int64_t)rank * R;
    for (int32_t j = 0; j < P; ++j) send_counts[j] = 0;
    for (int32_t r = 0; r < R; ++r) send_counts[sgx_reducer_owner(r, R, P)] += mine[r];
    int64_t run = 0;
    for (int32_t j = 0; j < P; ++j) { send_displs[j] = run; run += send_counts[j]; }
    int32_t r0, r1;
    my_reducers(R, P, rank, &r0, &r1);
    run = 0;
    for (int32_t sidx = 0; sidx < P; ++sidx) {
        int64_t c = 0;
        for (int32_t r = r0; r < r1; ++r) c += L[(int64_t)sidx * R + r];
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
    if (items && cnt > cap) return fail(SGX_ERR_INVALID, "item capacity %lld < %lld", (long long)cap, (long long)cnt);
    return SGX_OK;
}

extern "C" int sgx_copy_items(sgx_engine *e, const void *src, void *dst, const int64_t *items,
                              int64_t n_items, int32_t align) {
    if (!e || n_items < 0 || (n_items > 0 && (!items || !src || !dst)) || (align != 4 && align != 16))
        return fail(SGX_ERR_INVALID, "sgx_copy_items: bad arguments");
    for (int64_t i = 0; i < n_items; ++i)
        if (items[3 * i] % align || items[3 * i + 1] % align || items[3 * i + 2] % align || items[3 * i + 2] < 0)
            return fail(SGX_ERR_INVALID, "sgx_copy_items: item %lld not %d-byte aligned", (long long)i, align);
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    if (n_items == 0) return SGX_OK;
    DevBuf d;
    SGX_TRY(d.ensure((size_t)n_items * 24));
    HIP_TRY(hipMemcpyAsync(d.p, items, (size_t)n_items * 24, hipMemcpyHostToDevice, e->s_comp));
    HIP_TRY(launch_copy_items(src, dst, (const int64_t *)d.p, n_items, align, e->s_comp));
    HIP_TRY(hipStreamSynchronize(e->s_comp));
    d.release();
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// RCCL exchange
// ------------------------------------------------------------------------------------
extern "C" int sgx_get_unique_id(uint8_t out_id[128]) {
    if (!out_id) return fail(SGX_ERR_INVALID, "NULL id");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(out_id, id.internal, 128);
    return SGX_OK;
}

extern "C" int sgx_comm_init(sgx_engine *e, int32_t nranks, int32_t rank, const uint8_t id[128]) {
    if (!e || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(SGX_ERR_INVALID, "bad arguments");
    std::lock_guard<std::mutex> lk(e->mu);
    if (e->comm) return fail(SGX_ERR_STATE, "communicator already initialised");
    HIP_TRY(hipSetDevice(e->device));
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, 128);
    NCCL_TRY(ncclCommInitRank(&e->comm, nranks, uid, rank));
    e->nranks = nranks;
    e->rank = rank;
    return SGX_OK;
}

extern "C" int sgx_comm_size(sgx_engine *e, int32_t *nranks, int32_t *rank) {
    if (!e || !nranks || !rank) return fail(SGX_ERR_INVALID, "NULL argument");
    *nranks = e->nranks;
    *rank = e->rank;
    return SGX_OK;
}

static constexpr int64_t ITEM_BYTES = 64 * 1024;

extern "C" int sgx_exchange(sgx_engine *e, int32_t shuffle_id, int64_t map_id) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    Shuffle *s;
    MapOut *m;
    SGX_TRY(find_map(e, shuffle_id, map_id, &s, &m));
    HIP_TRY(hipSetDevice(e->device));
    SGX_TRY(finish_lengths(e, *s, *m));
    const int32_t P = e->nranks, R = s->R;
    std::unique_ptr<Round> rd(new Round());
    rd->map_ids.assign((size_t)P, 0);
    rd->lens.assign((size_t)P * R, 0);
    my_reducers(R, P, e->rank, &rd->r0, &rd->r1);
    const int32_t nmine = rd->r1 - rd->r0;
    HIP_TRY(hipEventCreateWithFlags(&rd->done, hipEventDisableTiming));
    if (P == 1 && !e->comm) {
        rd->map_ids[0] = map_id;
        std::memcpy(rd->lens.data(), m->lengths.data(), sizeof(int64_t) * (size_t)R);
        rd->block_off.assign((size_t)nmine, 0);
        int64_t off = 0;
        for (int32_t r = 0; r < R; ++r) { rd->block_off[(size_t)r] = off; off += m->lengths[(size_t)r]; }
        rd->alias = m->view();
        HIP_TRY(hipEventRecord(rd->done, e->s_comp));
        for (auto it = s->rounds.begin(); it != s->rounds.end(); ++it)
            if ((*it)->map_ids == rd->map_ids) { free_round(**it); s->rounds.erase(it); break; }
        s->rounds.push_back(std::move(rd));
        return SGX_OK;
    }
    if (!e->comm) return fail(SGX_ERR_STATE, "sgx_comm_init was not called (world of %d ranks)", P);
    hipStream_t st = e->s_comm;
    // (1) counts exchange: all-gather {map_id, lengths[R]}
    const size_t row = (size_t)R + 1;
    SGX_TRY(e->ag_host.ensure(row * 8 * (size_t)(P + 1)));
    int64_t *agh = (int64_t *)e->ag_host.p;
    agh[0] = map_id;
    std::memcpy(agh + 1, m->lengths.data(), sizeof(int64_t) * (size_t)R);
    SGX_TRY(e->ag_send.ensure(row * 8));
    SGX_TRY(e->ag_recv.ensure(row * 8 * (size_t)P));
    hipEvent_t a0 = e->ev(), a1 = e->ev(), a2 = e->ev(), a3 = e->ev();
    HIP_TRY(hipEventRecord(a0, st));
    HIP_TRY(hipMemcpyAsync(e->ag_send.p, agh, row * 8, hipMemcpyHostToDevice, st));
    NCCL_TRY(ncclAllGather(e->ag_send.p, e->ag_recv.p, row, ncclInt64, e->comm, st));
    HIP_TRY(hipMemcpyAsync(agh + row, e->ag_recv.p, row * 8 * (size_t)P, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(a1, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (int32_t j = 0; j < P; ++j) {
        rd->map_ids[(size_t)j] = agh[row * (size_t)(j + 1)];
        std::memcpy(&rd->lens[(size_t)j * R], agh + row * (size_t)(j + 1) + 1, sizeof(int64_t) * (size_t)R);
    }
    // (2) plan: send/recv counts and displacements (no copy list: blocks stay where they land)
    std::vector<int64_t> sc(P), sd(P), rc(P), rdp(P);
    int64_t nitems = 0;
    SGX_TRY(sgx_plan_exchange(rd->lens.data(), P, R, e->rank, 0, sc.data(), sd.data(), rc.data(), rdp.data(),
                              nullptr, &nitems));
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
    // its HBM once every reader of it has finished.
    for (auto it = s->rounds.begin(); it != s->rounds.end(); ++it) {
        if ((*it)->map_ids == rd->map_ids) {
            if ((*it)->done) HIP_TRY(hipEventSynchronize((*it)->done));
            std::swap(rd->data, (*it)->data);
            free_round(**it);
            s->rounds.erase(it);
            break;
        }
    }
    // (3) all-to-all of the partition-contiguous map output (already destination-grouped,
    //     reducer r lives on rank floor(r*P/R)): no pack step before, no regroup after
    SGX_TRY(rd->data.ensure((size_t)total_recv));
    HIP_TRY(hipStreamWaitEvent(st, m->done, 0));
    std::vector<size_t> scz(P), sdz(P), rcz(P), rdz(P);
    for (int32_t j = 0; j < P; ++j) {
        scz[(size_t)j] = (size_t)sc[(size_t)j];
        sdz[(size_t)j] = (size_t)sd[(size_t)j];
        rcz[(size_t)j] = (size_t)rc[(size_t)j];
        rdz[(size_t)j] = (size_t)rdp[(size_t)j];
    }
    HIP_TRY(hipEventRecord(a2, st));
    NCCL_TRY(ncclAllToAllv(m->view(), scz.data(), sdz.data(), rd->data.p, rcz.data(), rdz.data(), ncclUint8,
                           e->comm, st));
    HIP_TRY(hipEventRecord(a3, st));
    HIP_TRY(hipEventRecord(rd->done, st));
    if (!m->read_done) HIP_TRY(hipEventCreateWithFlags(&m->read_done, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(m->read_done, st));
    record_stage(e, SGX_STAGE_ALLGATHER, a0, a1);
    record_stage(e, SGX_STAGE_ALLTOALL, a2, a3);
    s->rounds.push_back(std::move(rd));
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// fetchBlocksByBlockIds
// ------------------------------------------------------------------------------------
// fetchBlocksByBlockIds body (caller holds e->mu).  `sync`: wait for the copy before
// returning (the public call); the reduce side chains its sort behind it on s_comp instead.
static int fetch_locked(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, const int32_t *reduce_ids,
                        int64_t n, void *dst, int64_t dst_cap, int32_t dst_mem_kind, int64_t *out_lengths,
                        bool sync) {
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    Shuffle &s = it->second;
    HIP_TRY(hipSetDevice(e->device));
    struct Src { const void *p; int64_t len; hipEvent_t ready; };
    std::vector<Src> srcs((size_t)n);
    int64_t total = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t mid = map_ids[i];
        const int32_t r = reduce_ids[i];
        if (r < 0 || r >= s.R) return fail(SGX_ERR_INVALID, "reduceId %d out of range [0, %d)", r, s.R);
        bool found = false;
        // received blocks (newest round first)
        for (auto rt = s.rounds.rbegin(); rt != s.rounds.rend() && !found; ++rt) {
            Round &rd = **rt;
            if (r < rd.r0 || r >= rd.r1) continue;
            for (size_t j = 0; j < rd.map_ids.size(); ++j) {
                if (rd.map_ids[j] != mid) continue;
                const int32_t nmine = rd.r1 - rd.r0;
                srcs[(size_t)i] = Src{(const char *)rd.base() + rd.block_off[j * (size_t)nmine + (size_t)(r - rd.r0)],
                                      rd.lens[j * (size_t)s.R + (size_t)r], rd.done};
                found = true;
                break;
            }
        }
        if (!found) {
            auto mt = s.maps.find(mid);
            if (mt != s.maps.end()) {
                MapOut &m = *mt->second;
                SGX_TRY(finish_lengths(e, s, m));
                int64_t off = 0;
                for (int32_t q = 0; q < r; ++q) off += m.lengths[(size_t)q];
                srcs[(size_t)i] = Src{(const char *)m.view() + off, m.lengths[(size_t)r], m.done};
                found = true;
            }
        }
        if (!found)
            return fail(SGX_ERR_NOT_FOUND, "shuffle_%d_%lld_%d is not registered", shuffle_id, (long long)mid, r);
        out_lengths[i] = srcs[(size_t)i].len;
        total += srcs[(size_t)i].len;
    }
    if (total > dst_cap)
        return fail(SGX_ERR_INVALID, "destination capacity %lld < %lld bytes", (long long)dst_cap, (long long)total);
    if (total > 0 && !dst) return fail(SGX_ERR_INVALID, "dst is NULL");
    if (total == 0) return SGX_OK;
    hipStream_t st = e->s_comp;
    // every source must be complete: wait on each distinct producer event once
    std::vector<hipEvent_t> waited;
    for (int64_t i = 0; i < n; ++i) {
        hipEvent_t ev = srcs[(size_t)i].ready;
        if (ev && std::find(waited.begin(), waited.end(), ev) == waited.end()) {
            HIP_TRY(hipStreamWaitEvent(st, ev, 0));
            waited.push_back(ev);
        }
    }
    // one gather launch: {src, dst, bytes} pieces of <= 64 KiB, back to back in request
    // order (the reader asks reducer-major, map-minor: the canonical per-reducer sequence)
    const bool dev_dst = dst_mem_kind == SGX_MEM_DEVICE;
    char *gdst = (char *)dst;
    if (!dev_dst) {
        SGX_TRY(e->gather_stage.ensure((size_t)total));
        gdst = (char *)e->gather_stage.p;
    }
    int64_t npieces = 0;
    for (int64_t i = 0; i < n; ++i) npieces += (srcs[(size_t)i].len + ITEM_BYTES - 1) / ITEM_BYTES;
    SGX_TRY(e->gather_items.ensure((size_t)npieces * 24));
    SGX_TRY(e->items_dev.ensure((size_t)npieces * 24));
    int64_t *gi = (int64_t *)e->gather_items.p, k = 0, off = 0;
    bool al16 = ((uintptr_t)gdst & 15) == 0, al4 = ((uintptr_t)gdst & 3) == 0;
    for (int64_t i = 0; i < n; ++i) {
        const char *sp = (const char *)srcs[(size_t)i].p;
        for (int64_t done = 0; done < srcs[(size_t)i].len; done += ITEM_BYTES, ++k) {
            const int64_t b = std::min<int64_t>(ITEM_BYTES, srcs[(size_t)i].len - done);
            gi[3 * k] = (int64_t)(uintptr_t)(sp + done);
            gi[3 * k + 1] = (int64_t)(uintptr_t)(gdst + off + done);
            gi[3 * k + 2] = b;
            const uintptr_t bits = (uintptr_t)(sp + done) | (uintptr_t)(off + done) | (uintptr_t)b;
            al16 = al16 && (bits & 15) == 0;
            al4 = al4 && (bits & 3) == 0;
        }
        off += srcs[(size_t)i].len;
    }
    hipEvent_t g0 = e->ev(), g1 = e->ev();
    HIP_TRY(hipEventRecord(g0, st));
    HIP_TRY(hipMemcpyAsync(e->items_dev.p, gi, (size_t)npieces * 24, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_gather_items((const int64_t *)e->items_dev.p, npieces, al16 ? 16 : al4 ? 4 : 1, st));
    HIP_TRY(hipEventRecord(g1, st));
    record_stage(e, SGX_STAGE_REGROUP, g0, g1);
    if (!dev_dst) HIP_TRY(hipMemcpyAsync(dst, gdst, (size_t)total, hipMemcpyDeviceToHost, st));
    if (sync) HIP_TRY(hipStreamSynchronize(st));
    return SGX_OK;
}

extern "C" int sgx_fetch_blocks(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids,
                                const int32_t *reduce_ids, int64_t n, void *dst, int64_t dst_cap,
                                int32_t dst_mem_kind, int64_t *out_lengths) {
    if (!e || (n > 0 && (!map_ids || !reduce_ids || !out_lengths)))
        return fail(SGX_ERR_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(e->mu);
    return fetch_locked(e, shuffle_id, map_ids, reduce_ids, n, dst, dst_cap, dst_mem_kind, out_lengths, true);
}

// ------------------------------------------------------------------------------------
// Reduce side after the fetch (UcxShuffleReader.scala:137-191): stable sort by key per
// reducer, then groupByKey / reduceByKey on (Long, Long) records
// ------------------------------------------------------------------------------------
// Gather the canonical blocks of reducers [r0, r1) x maps into e->sort_buf[0] as records
// (a Kryo shuffle's stream is decoded on the GPU on the way); sort_buf[1] is sized to match.
// *nrec = records; asynchronous on s_comp except for a Kryo shuffle's record count.
static int records_locked(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps, int32_t r0,
                          int32_t r1, int64_t *nrec) {
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    Shuffle &s = it->second;
    if (r0 < 0 || r1 > s.R || r0 > r1)
        return fail(SGX_ERR_INVALID, "partition range [%d, %d) outside [0, %d)", r0, r1, s.R);
    if (nmaps < 0 || (nmaps > 0 && !map_ids)) return fail(SGX_ERR_INVALID, "bad map list");
    const int rb = s.rb;
    const int64_t nreq = (int64_t)(r1 - r0) * nmaps;
    std::vector<int64_t> mids((size_t)nreq), lens((size_t)nreq);
    std::vector<int32_t> rids((size_t)nreq);
    for (int32_t r = r0; r < r1; ++r)
        for (int64_t j = 0; j < nmaps; ++j) {
            mids[(size_t)((r - r0) * nmaps + j)] = map_ids[j];
            rids[(size_t)((r - r0) * nmaps + j)] = r;
        }
    // size query (fails with SGX_ERR_INVALID on capacity, after filling the lengths)
    int rc = fetch_locked(e, shuffle_id, mids.data(), rids.data(), nreq, nullptr, 0, SGX_MEM_DEVICE, lens.data(), false);
    if (rc != SGX_OK && rc != SGX_ERR_INVALID) return rc;
    int64_t total = 0;
    for (int64_t L : lens) total += L;
    hipStream_t st = e->s_comp;
    if (s.ser == SGX_SER_KRYO) {
        // the fetched Kryo stream (blocks back to back are one valid stream) -> records
        *nrec = 0;
        if (s.lz4_block > 0 && total > 0) {
            // a compressed shuffle: fetch the LZ4 frames, decompress them into the Kryo input
            // (LZ4BlockInputStream, same stream, so no host round trip between the two)
            DevBuf comp;
            DevBufScope gc{comp};
            SGX_TRY(comp.ensure((size_t)total));
            SGX_TRY(fetch_locked(e, shuffle_id, mids.data(), rids.data(), nreq, comp.p, total, SGX_MEM_DEVICE,
                                 lens.data(), false));
            int64_t dec = 0;
            SGX_TRY(lz4_unframe_impl(e, comp.p, total, &e->kryo_in, nullptr, 0, &dec));
            total = dec;
        }
        const int64_t cap = total / 4;  // a record takes >= 4 bytes
        SGX_TRY(e->sort_buf[0].ensure((size_t)cap * 16));
        if (total == 0) return SGX_OK;
        if (s.lz4_block == 0) {
            SGX_TRY(e->kryo_in.ensure((size_t)total + 64));
            SGX_TRY(fetch_locked(e, shuffle_id, mids.data(), rids.data(), nreq, e->kryo_in.p, total, SGX_MEM_DEVICE,
                                 lens.data(), false));
        }
        const int64_t tiles = kryo_deser16_tiles(total);
        SGX_TRY(e->kryo_work.ensure(24 + (size_t)kryo_work_bytes(tiles)));
        HIP_TRY(hipMemsetAsync(e->kryo_work.p, 0, 24, st));  // error word, record count
        uint32_t *tick = (uint32_t *)e->kryo_work.p;
        int64_t *cnt_dev = (int64_t *)((char *)e->kryo_work.p + 16);
        uint64_t *status = (uint64_t *)((char *)e->kryo_work.p + 24);
        hipEvent_t k0 = e->ev(), k1 = e->ev();
        HIP_TRY(hipEventRecord(k0, st));
        HIP_TRY(launch_kryo_deser16(e->kryo_in.p, total, e->sort_buf[0].p, cap, status, tick, cnt_dev, st));
        HIP_TRY(hipEventRecord(k1, st));
        record_stage(e, SGX_STAGE_DESERIALIZE, k0, k1);
        uint32_t herr[4];
        int64_t hcnt = 0;
        HIP_TRY(hipMemcpyAsync(herr, tick, 16, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(&hcnt, cnt_dev, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (herr[1] & 1u) return fail(SGX_ERR_TIMEOUT, "Kryo decoder look-back spin gave up");
        if (herr[1] & 2u) return fail(SGX_ERR_INVALID, "fetched blocks are not a Kryo stream of (Long, Long) pairs");
        if (hcnt < 0 || hcnt > cap) return fail(SGX_ERR_HIP, "internal error: Kryo record count %lld", (long long)hcnt);
        if (hcnt >= (int64_t)INT32_MAX) return fail(SGX_ERR_INVALID, "%lld records exceed one read", (long long)hcnt);
        *nrec = hcnt;
        SGX_TRY(e->sort_buf[1].ensure((size_t)hcnt * 16));
        return SGX_OK;
    }
    const int64_t n = total / rb;
    if (n >= (int64_t)INT32_MAX) return fail(SGX_ERR_INVALID, "%lld records exceed one sorted read", (long long)n);
    *nrec = n;
    SGX_TRY(e->sort_buf[0].ensure((size_t)total));
    SGX_TRY(e->sort_buf[1].ensure((size_t)total));
    if (n == 0) return SGX_OK;
    SGX_TRY(fetch_locked(e, shuffle_id, mids.data(), rids.data(), nreq, e->sort_buf[0].p, total, SGX_MEM_DEVICE,
                         lens.data(), false));
    return SGX_OK;
}

// Fetch the canonical blocks of reducers [r0, r1) x maps into e->sort_buf[0] and sort them
// stably by key within each reducer.  On return (asynchronous on s_comp) *sorted points at
// the device buffer holding the result and *nrec its record count.
static int sort_locked(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps, int32_t r0,
                       int32_t r1, const void **sorted, int64_t *nrec) {
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    Shuffle &s = it->second;
    const int rb = s.rb;
    if (rb != 16 && rb != 100)
        return fail(SGX_ERR_UNSUPPORTED, "sorted read needs 16 B (Long, Long) or 100 B TeraSort records, not %d B", rb);
    int64_t n = 0;
    SGX_TRY(records_locked(e, shuffle_id, map_ids, nmaps, r0, r1, &n));
    *nrec = n;
    *sorted = e->sort_buf[0].p;
    if (n == 0) return SGX_OK;
    hipStream_t st = e->s_comp;
    constexpr int MAXP = 12;
    SGX_TRY(e->sort_err.ensure(MAXP * 4));
    HIP_TRY(hipMemsetAsync(e->sort_err.p, 0, MAXP * 4, st));
    uint32_t *errs = (uint32_t *)e->sort_err.p;
    hipEvent_t t0 = e->ev(), t1 = e->ev();
    HIP_TRY(hipEventRecord(t0, st));
    // LSD digit passes, least significant byte first: i64 keys (bytes 0..7 of the record,
    // sign flip on the top byte), or TeraSort's 10-byte big-endian keys (bytes 9..0).  One
    // read of the keys histograms every digit; a digit with a single non-empty bucket is
    // the identity permutation and is skipped.
    const int ndig = rb == 16 ? 8 : 10;
    SGX_TRY(e->digit_hist.ensure((size_t)ndig * 256 * 4));
    HIP_TRY(launch_digit_hist(e->sort_buf[0].p, n, rb, (uint32_t *)e->digit_hist.p, e->num_cus, st));
    std::vector<uint32_t> dh((size_t)ndig * 256);
    HIP_TRY(hipMemcpyAsync(dh.data(), e->digit_hist.p, dh.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    int cur = 0, np = 0;
    for (int d = 0; d < ndig; ++d) {
        const int byte = rb == 16 ? d : 9 - d;  // digit d of the LSD order
        bool trivial = false;
        for (int b = 0; b < 256; ++b)
            if (dh[(size_t)byte * 256 + (size_t)b] == (uint32_t)n) trivial = true;
        if (trivial && e->sort_skip) continue;
        ++np;
        PartParams dp{};
        dp.kind = KIND_DIGIT;
        dp.R = DIGIT_R;
        dp.nbits = 8;
        dp.dshift = rb == 16 ? 8u * (uint32_t)d : 8u * (uint32_t)(9 - d);
        dp.dflip = (rb == 16 && d == 7) ? 0x80u : 0u;
        SGX_TRY(partition_pass(e, e->sort_buf[cur].p, e->sort_buf[cur ^ 1].p, n, rb, dp, (int32_t)DIGIT_R,
                               KIND_DIGIT, 0, SGX_MEM_DEVICE, nullptr, errs + np - 1, false));
        cur ^= 1;
    }
    // records back into reducer order: the shuffle's own partitioner, stable (an ascending
    // RangePartitioner's partition order is already key order)
    const bool range_asc = s.kind != SGX_PART_HASH && s.asc;
    if (!range_asc && s.R > 1) {
        SGX_TRY(partition_pass(e, e->sort_buf[cur].p, e->sort_buf[cur ^ 1].p, n, rb, s.pp, s.R, s.kind, s.nb,
                               SGX_MEM_DEVICE, nullptr, errs + np, false));
        cur ^= 1;
        ++np;
    }
    HIP_TRY(hipEventRecord(t1, st));
    record_stage(e, SGX_STAGE_SORT, t0, t1);
    uint32_t herr[MAXP];
    HIP_TRY(hipMemcpyAsync(herr, e->sort_err.p, MAXP * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (int i = 0; i < np; ++i) {
        if (herr[i] & 1u) return fail(SGX_ERR_TIMEOUT, "sort pass %d: scan look-back spin gave up", i);
        if (herr[i] & 2u) return fail(SGX_ERR_HIP, "sort pass %d: a scatter destination was out of range", i);
    }
    *sorted = e->sort_buf[cur].p;
    return SGX_OK;
}

static int copy_out(sgx_engine *e, void *dst, const void *src, int64_t bytes, int32_t mem_kind) {
    if (bytes <= 0) return SGX_OK;
    HIP_TRY(hipMemcpyAsync(dst, src, (size_t)bytes,
                           mem_kind == SGX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, e->s_comp));
    return SGX_OK;
}

extern "C" int sgx_read_sorted(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                               int32_t start_partition, int32_t end_partition, void *dst, int64_t dst_cap,
                               int32_t dst_mem_kind, int64_t *out_bytes) {
    if (!e || !out_bytes) return fail(SGX_ERR_INVALID, "NULL argument");
    if (dst_mem_kind != SGX_MEM_HOST && dst_mem_kind != SGX_MEM_DEVICE)
        return fail(SGX_ERR_INVALID, "unknown mem_kind %d", dst_mem_kind);
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    const int rb = it->second.rb;
    if (!dst && dst_cap == 0 && it->second.ser == SGX_SER_KRYO) {  // size query: decoded records
        int64_t n = 0;
        SGX_TRY(records_locked(e, shuffle_id, map_ids, nmaps, start_partition, end_partition, &n));
        *out_bytes = n * rb;
        return SGX_OK;
    }
    if (!dst && dst_cap == 0) {  // size query: lengths only
        const int64_t nreq = (int64_t)std::max(0, end_partition - start_partition) * std::max<int64_t>(0, nmaps);
        if (start_partition < 0 || end_partition > it->second.R || start_partition > end_partition || nmaps < 0 ||
            (nmaps > 0 && !map_ids))
            return fail(SGX_ERR_INVALID, "bad partition range or map list");
        std::vector<int64_t> mids((size_t)nreq), lens((size_t)nreq);
        std::vector<int32_t> rids((size_t)nreq);
        for (int64_t q = 0; q < nreq; ++q) {
            mids[(size_t)q] = map_ids[q % nmaps];
            rids[(size_t)q] = start_partition + (int32_t)(q / nmaps);
        }
        int rc = fetch_locked(e, shuffle_id, mids.data(), rids.data(), nreq, nullptr, 0, SGX_MEM_DEVICE, lens.data(), false);
        if (rc != SGX_OK && rc != SGX_ERR_INVALID) return rc;
        int64_t total = 0;
        for (int64_t L : lens) total += L;
        *out_bytes = total;
        return SGX_OK;
    }
    const void *sorted = nullptr;
    int64_t n = 0;
    SGX_TRY(sort_locked(e, shuffle_id, map_ids, nmaps, start_partition, end_partition, &sorted, &n));
    *out_bytes = n * rb;
    if (n * rb > dst_cap) return fail(SGX_ERR_INVALID, "destination capacity %lld < %lld bytes", (long long)dst_cap,
                                      (long long)(n * rb));
    if (n > 0 && !dst) return fail(SGX_ERR_INVALID, "dst is NULL");
    SGX_TRY(copy_out(e, dst, sorted, n * rb, dst_mem_kind));
    HIP_TRY(hipStreamSynchronize(e->s_comp));
    return SGX_OK;
}

extern "C" int sgx_read_records(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                                int32_t start_partition, int32_t end_partition, void *dst, int64_t dst_cap,
                                int32_t dst_mem_kind, int64_t *out_bytes) {
    if (!e || !out_bytes) return fail(SGX_ERR_INVALID, "NULL argument");
    if (dst_mem_kind != SGX_MEM_HOST && dst_mem_kind != SGX_MEM_DEVICE)
        return fail(SGX_ERR_INVALID, "unknown mem_kind %d", dst_mem_kind);
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    const int rb = it->second.rb;
    int64_t n = 0;
    SGX_TRY(records_locked(e, shuffle_id, map_ids, nmaps, start_partition, end_partition, &n));
    *out_bytes = n * rb;
    if (!dst && dst_cap == 0) return SGX_OK;  // size query
    if (n * rb > dst_cap) return fail(SGX_ERR_INVALID, "destination capacity %lld < %lld bytes", (long long)dst_cap,
                                      (long long)(n * rb));
    if (n > 0 && !dst) return fail(SGX_ERR_INVALID, "dst is NULL");
    SGX_TRY(copy_out(e, dst, e->sort_buf[0].p, n * rb, dst_mem_kind));
    HIP_TRY(hipStreamSynchronize(e->s_comp));
    return SGX_OK;
}

extern "C" int sgx_read_grouped(sgx_engine *e, int32_t shuffle_id, const int64_t *map_ids, int64_t nmaps,
                                int32_t start_partition, int32_t end_partition, int32_t agg, int64_t *keys,
                                int64_t *group_starts, int64_t *values, int64_t cap_groups, int64_t cap_values,
                                int32_t mem_kind, int64_t *out_groups, int64_t *out_values) {
    if (!e || !out_groups || !out_values) return fail(SGX_ERR_INVALID, "NULL argument");
    if (agg != SGX_AGG_GROUP && agg != SGX_AGG_SUM) return fail(SGX_ERR_INVALID, "unknown aggregation %d", agg);
    if (mem_kind != SGX_MEM_HOST && mem_kind != SGX_MEM_DEVICE)
        return fail(SGX_ERR_INVALID, "unknown mem_kind %d", mem_kind);
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    auto it = e->shuffles.find(shuffle_id);
    if (it == e->shuffles.end()) return fail(SGX_ERR_STATE, "shuffle %d is not registered", shuffle_id);
    if (it->second.rb != 16)
        return fail(SGX_ERR_UNSUPPORTED, "grouped read needs 16 B (Long, Long) records, not %d B", it->second.rb);
    const void *sorted = nullptr;
    int64_t n = 0;
    SGX_TRY(sort_locked(e, shuffle_id, map_ids, nmaps, start_partition, end_partition, &sorted, &n));
    hipStream_t st = e->s_comp;
    // group ids: flags of key changes, exclusive scan (K3 with one partition: offs[i] is the
    // group of record i minus its flag; part_off[1] the group count)
    const int64_t tiles = scan_tiles(n);
    SGX_TRY(e->grp_flags.ensure((size_t)std::max<int64_t>(n, 1) * 4));
    SGX_TRY(e->grp_offs.ensure((size_t)std::max<int64_t>(n, 1) * 4));
    SGX_TRY(e->grp_status.ensure((size_t)(16 + tiles * 8 + 16)));
    uint32_t *ticket_err = (uint32_t *)e->grp_status.p;
    uint32_t *gcount = (uint32_t *)((char *)e->grp_status.p + 16 + tiles * 8);  // [0, total]
    int64_t ngroups = 0;
    hipEvent_t t0 = e->ev(), t1 = e->ev();
    HIP_TRY(hipEventRecord(t0, st));
    if (n > 0) {
        HIP_TRY(hipMemsetAsync(e->grp_status.p, 0, (size_t)(16 + tiles * 8 + 16), st));
        HIP_TRY(launch_group_flags(sorted, n, (uint32_t *)e->grp_flags.p, st));
        HIP_TRY(launch_scan((const uint32_t *)e->grp_flags.p, (uint32_t *)e->grp_offs.p, n,
                            (uint64_t *)((char *)e->grp_status.p + 16), ticket_err, ticket_err + 1, gcount, (int)n,
                            1, st));
        uint32_t h[2] = {0, 0}, terr[2] = {0, 0};
        HIP_TRY(hipMemcpyAsync(h, gcount, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(terr, ticket_err, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (terr[1] & 1u) return fail(SGX_ERR_TIMEOUT, "group scan look-back spin gave up");
        ngroups = h[1];
    }
    const int64_t nvals = agg == SGX_AGG_GROUP ? n : ngroups;
    *out_groups = ngroups;
    *out_values = nvals;
    if (!keys && cap_groups == 0 && cap_values == 0) {
        (void)hipEventRecord(t1, st);
        record_stage(e, SGX_STAGE_GROUP, t0, t1);
        return SGX_OK;  // size query
    }
    if (ngroups > cap_groups || nvals > cap_values)
        return fail(SGX_ERR_INVALID, "capacity (%lld groups, %lld values) < (%lld, %lld)", (long long)cap_groups,
                    (long long)cap_values, (long long)ngroups, (long long)nvals);
    if (n == 0) return SGX_OK;
    if (!keys || !values || (agg == SGX_AGG_GROUP && !group_starts))
        return fail(SGX_ERR_INVALID, "NULL output array");
    SGX_TRY(e->grp_out.ensure((size_t)(ngroups * 16 + nvals * 8)));
    int64_t *dkeys = (int64_t *)e->grp_out.p, *dstarts = dkeys + ngroups, *dvals = dstarts + ngroups;
    HIP_TRY(launch_group_emit(sorted, n, (const uint32_t *)e->grp_flags.p, (const uint32_t *)e->grp_offs.p, dkeys,
                              dstarts, agg == SGX_AGG_GROUP ? dvals : nullptr, st));
    if (agg == SGX_AGG_SUM) {
        SGX_TRY(e->grp_prefix.ensure((size_t)(n + prefix64_blocks(n)) * 8));
        uint64_t *P = (uint64_t *)e->grp_prefix.p, *bsum = P + n;
        HIP_TRY(launch_group_sums(sorted, n, dstarts, ngroups, bsum, P, dvals, st));
    }
    HIP_TRY(hipEventRecord(t1, st));
    record_stage(e, SGX_STAGE_GROUP, t0, t1);
    SGX_TRY(copy_out(e, keys, dkeys, ngroups * 8, mem_kind));
    if (group_starts) SGX_TRY(copy_out(e, group_starts, dstarts, ngroups * 8, mem_kind));
    SGX_TRY(copy_out(e, values, dvals, nvals * 8, mem_kind));
    HIP_TRY(hipStreamSynchronize(st));
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// progress / sync / stats
// ------------------------------------------------------------------------------------
extern "C" int sgx_progress(sgx_engine *e) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    hipError_t a = hipStreamQuery(e->s_comp), b = hipStreamQuery(e->s_comm);
    if ((a != hipSuccess && a != hipErrorNotReady) || (b != hipSuccess && b != hipErrorNotReady))
        return fail(SGX_ERR_HIP, "stream error: %s / %s", hipGetErrorString(a), hipGetErrorString(b));
    return (a == hipSuccess && b == hipSuccess) ? 1 : 0;
}

extern "C" int sgx_sync(sgx_engine *e) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->s_comp));
    HIP_TRY(hipStreamSynchronize(e->s_comm));
    HIP_TRY(hipStreamSynchronize(e->s_hist));
    for (auto &kv : e->shuffles)
        for (auto &m : kv.second.maps) SGX_TRY(finish_lengths(e, kv.second, *m.second));
    return SGX_OK;
}

extern "C" int sgx_stats_reset(sgx_engine *e) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    e->resolve_stats();
    for (int i = 0; i < SGX_NUM_STAGES; ++i) { e->stage_ms[i] = 0; e->stage_n[i] = 0; }
    return SGX_OK;
}

extern "C" int sgx_stats_get(sgx_engine *e, double *ms, int64_t *cnt) {
    if (!e || !ms || !cnt) return fail(SGX_ERR_INVALID, "NULL argument");
    std::lock_guard<std::mutex> lk(e->mu);
    e->resolve_stats();
    for (int i = 0; i < SGX_NUM_STAGES; ++i) { ms[i] = e->stage_ms[i]; cnt[i] = e->stage_n[i]; }
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// generators and memory helpers
// ------------------------------------------------------------------------------------
extern "C" int sgx_gen_uniform16(sgx_engine *e, void *dst, int64_t n, uint64_t seed, int64_t vbase) {
    if (!e || (n > 0 && !dst)) return fail(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    if (n > 0) HIP_TRY(launch_gen_uniform16(dst, n, seed, vbase, e->s_comp));
    HIP_TRY(hipStreamSynchronize(e->s_comp));
    return SGX_OK;
}

extern "C" int sgx_gen_zipf16(sgx_engine *e, void *dst, int64_t n, uint64_t seed, int64_t vbase,
                              const double *cdf_host, int64_t K) {
    if (!e || (n > 0 && !dst) || !cdf_host || K < 1) return fail(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    DevBuf cdf;
    SGX_TRY(cdf.ensure((size_t)K * 8));
    HIP_TRY(hipMemcpy(cdf.p, cdf_host, (size_t)K * 8, hipMemcpyHostToDevice));
    if (n > 0) HIP_TRY(launch_gen_zipf16(dst, n, seed, vbase, (const double *)cdf.p, K, e->s_comp));
    HIP_TRY(hipStreamSynchronize(e->s_comp));
    cdf.release();
    return SGX_OK;
}

extern "C" int sgx_gen_terasort100(sgx_engine *e, void *dst, int64_t n, uint64_t seed, int64_t ibase) {
    if (!e || (n > 0 && !dst)) return fail(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    if (n > 0) HIP_TRY(launch_gen_terasort100(dst, n, seed, ibase, e->s_comp));
    HIP_TRY(hipStreamSynchronize(e->s_comp));
    return SGX_OK;
}

extern "C" int sgx_device_alloc(sgx_engine *e, int64_t bytes, void **out) {
    if (!e || !out || bytes < 0) return fail(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    hipError_t er = hipMalloc(out, (size_t)(bytes ? bytes : 16));
    if (er != hipSuccess) return fail(SGX_ERR_NOMEM, "hipMalloc(%lld): %s", (long long)bytes, hipGetErrorString(er));
    return SGX_OK;
}

extern "C" int sgx_device_free(sgx_engine *e, void *p) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    HIP_TRY(hipSetDevice(e->device));
    if (p) HIP_TRY(hipFree(p));
    return SGX_OK;
}

extern "C" int sgx_memcpy(sgx_engine *e, void *dst, const void *src, int64_t bytes) {
    if (!e || bytes < 0) return fail(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    if (bytes > 0) HIP_TRY(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDefault));
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// RangePartitioner bounds from the data: sketch (GPU reservoir sampling) + determineBounds
// (Spark 3.0.1 RangePartitioner, spark-core; restated, see include/sgx.h)
// ------------------------------------------------------------------------------------
namespace {

// scala.util.hashing.MurmurHash3 (Scala 2.12): bytesHash(data, seed), arraySeed = 0x3c074a61
inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t mm3_mix_last(uint32_t h, uint32_t k) {
    k *= 0xcc9e2d51u;
    k = rotl32(k, 15);
    k *= 0x1b873593u;
    return h ^ k;
}
inline uint32_t mm3_mix(uint32_t h, uint32_t k) {
    h = mm3_mix_last(h, k);
    h = rotl32(h, 13);
    return h * 5u + 0xe6546b64u;
}
inline uint32_t mm3_avalanche(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
uint32_t mm3_bytes_hash(const uint8_t *d, int len, uint32_t seed) {
    uint32_t h = seed;
    int i = 0, rem = len;
    while (rem >= 4) {
        const uint32_t k = (uint32_t)d[i] | ((uint32_t)d[i + 1] << 8) | ((uint32_t)d[i + 2] << 16) |
                           ((uint32_t)d[i + 3] << 24);
        h = mm3_mix(h, k);
        i += 4;
        rem -= 4;
    }
    uint32_t k = 0;
    if (rem == 3) k ^= (uint32_t)d[i + 2] << 16;
    if (rem >= 2) k ^= (uint32_t)d[i + 1] << 8;
    if (rem >= 1) {
        k ^= (uint32_t)d[i];
        h = mm3_mix_last(h, k);
    }
    return mm3_avalanche(h ^ (uint32_t)len);
}

// org.apache.spark.util.random.XORShiftRandom.hashSeed: MurmurHash3 of the big-endian bytes
uint64_t xorshift_hash_seed(int64_t seed) {
    uint8_t b[8];
    for (int i = 0; i < 8; ++i) b[i] = (uint8_t)((uint64_t)seed >> (56 - 8 * i));
    const uint32_t lo = mm3_bytes_hash(b, 8, 0x3c074a61u);
    const uint32_t hi = mm3_bytes_hash(b, 8, lo);
    return ((uint64_t)hi << 32) | (uint64_t)lo;
}

// scala.util.hashing.byteswap32
int32_t byteswap32(int32_t v) {
    uint32_t hc = (uint32_t)v * 0x9e3775cdu;
    hc = __builtin_bswap32(hc);
    return (int32_t)(hc * 0x9e3775cdu);
}

// column form of M^(2^t), t = 0..47, M = one XORShiftRandom step
std::vector<uint64_t> xorshift_jump_table() {
    auto step = [](uint64_t s) {
        s ^= s << 21;
        s ^= s >> 35;
        s ^= s << 4;
        return s;
    };
    auto apply = [](const uint64_t *cols, uint64_t v) {
        uint64_t r = 0;
        for (int b = 0; b < 64; ++b)
            if ((v >> b) & 1ull) r ^= cols[b];
        return r;
    };
    std::vector<uint64_t> t(48 * 64);
    for (int b = 0; b < 64; ++b) t[(size_t)b] = step(1ull << b);
    for (int lvl = 1; lvl < 48; ++lvl)
        for (int b = 0; b < 64; ++b)
            t[(size_t)lvl * 64 + (size_t)b] = apply(&t[(size_t)(lvl - 1) * 64], apply(&t[(size_t)(lvl - 1) * 64], 1ull << b));
    return t;
}

struct Cand {
    std::array<uint8_t, 10> k10;
    int64_t k64;
    float w;
};

}  // namespace

extern "C" int sgx_range_bounds(sgx_engine *e, const void *const *batches, const int64_t *nrecords, int32_t nbatches,
                                int32_t rb, int32_t mem_kind, int32_t num_partitions, int32_t rdd_id,
                                int32_t sample_points_per_partition, void *out_bounds, int32_t *out_nbounds) {
    if (!e || !out_nbounds || (nbatches > 0 && (!batches || !nrecords))) return fail(SGX_ERR_INVALID, "NULL argument");
    if (rb != 16 && rb != 100) return fail(SGX_ERR_UNSUPPORTED, "range bounds need 16 B or 100 B records, not %d", rb);
    if (mem_kind != SGX_MEM_HOST && mem_kind != SGX_MEM_DEVICE) return fail(SGX_ERR_INVALID, "unknown mem_kind");
    if (num_partitions < 1 || nbatches < 0 || sample_points_per_partition < 1)
        return fail(SGX_ERR_INVALID, "bad partition / batch / sample counts");
    *out_nbounds = 0;
    if (num_partitions <= 1 || nbatches == 0) return SGX_OK;  // rangeBounds = Array.empty
    std::lock_guard<std::mutex> lk(e->mu);
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t st = e->s_comp;
    const int kb = rb == 16 ? 8 : 10;
    // sampleSize capped at 1M; over-sample 3x per partition (RangePartitioner rangeBounds)
    const double sample_size = std::min((double)sample_points_per_partition * num_partitions, 1e6);
    const int64_t k = (int64_t)std::ceil(3.0 * sample_size / nbatches);
    if (e->jump_dev.p == nullptr) {
        const std::vector<uint64_t> jt = xorshift_jump_table();
        SGX_TRY(e->jump_dev.ensure(jt.size() * 8));
        HIP_TRY(hipMemcpy(e->jump_dev.p, jt.data(), jt.size() * 8, hipMemcpyHostToDevice));
    }
    SGX_TRY(e->sample_winner.ensure((size_t)k * 8));
    SGX_TRY(e->sample_keys.ensure((size_t)k * (size_t)kb));
    std::vector<std::vector<uint8_t>> samples((size_t)nbatches);
    int64_t num_items = 0;
    for (int32_t i = 0; i < nbatches; ++i) {
        const int64_t n = nrecords[i];
        if (n < 0) return fail(SGX_ERR_INVALID, "batch %d: %lld records", i, (long long)n);
        num_items += n;
        const int64_t kk = std::min(n, k);
        samples[(size_t)i].resize((size_t)(kk * kb));
        if (kk == 0) continue;
        const void *src = batches[i];
        if (mem_kind == SGX_MEM_HOST) {
            SGX_TRY(e->input_stage.ensure((size_t)(n * rb)));
            HIP_TRY(hipMemcpyAsync(e->input_stage.p, src, (size_t)(n * rb), hipMemcpyHostToDevice, st));
            src = e->input_stage.p;
        }
        const int32_t seed = byteswap32((int32_t)((uint32_t)i ^ ((uint32_t)rdd_id << 16)));
        const uint64_t s0 = xorshift_hash_seed((int64_t)seed);  // Int seed widened to Long
        HIP_TRY(launch_reservoir(src, n, rb, kb, k, s0, (const uint64_t *)e->jump_dev.p,
                                 (long long *)e->sample_winner.p, e->sample_keys.p, st));
        HIP_TRY(hipMemcpyAsync(samples[(size_t)i].data(), e->sample_keys.p, (size_t)(kk * kb), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    if (num_items == 0) return SGX_OK;
    // candidates weighted by 1 / sampling probability; imbalanced partitions would be
    // re-sampled by Spark (PartitionPruningRDD.sample): not reproduced here
    const double fraction = std::min(sample_size / (double)std::max<int64_t>(num_items, 1), 1.0);
    std::vector<Cand> cand;
    for (int32_t i = 0; i < nbatches; ++i) {
        const int64_t n = nrecords[i];
        const int64_t len = (int64_t)samples[(size_t)i].size() / kb;
        if (fraction * (double)n > (double)k)
            return fail(SGX_ERR_UNSUPPORTED, "partition %d is imbalanced (%lld records): Spark re-samples it", i,
                        (long long)n);
        if (len == 0) continue;
        const float w = (float)((double)n / (double)len);
        for (int64_t j = 0; j < len; ++j) {
            Cand c{};
            const uint8_t *p = samples[(size_t)i].data() + j * kb;
            if (kb == 8) {
                int64_t v;
                std::memcpy(&v, p, 8);
                c.k64 = v;
            } else {
                std::memcpy(c.k10.data(), p, 10);
            }
            c.w = w;
            cand.push_back(c);
        }
    }
    // determineBounds(candidates, min(partitions, candidates.size)): stable sort by key,
    // weights summed in sorted order, a bound each time the cumulative weight reaches the
    // next step, duplicates skipped
    auto lt = [kb](const Cand &a, const Cand &b) {
        return kb == 8 ? a.k64 < b.k64 : std::memcmp(a.k10.data(), b.k10.data(), 10) < 0;
    };
    std::stable_sort(cand.begin(), cand.end(), lt);
    const int32_t parts = (int32_t)std::min<int64_t>(num_partitions, (int64_t)cand.size());
    double sum_w = 0.0;
    for (const Cand &c : cand) sum_w += (double)c.w;
    const double step = sum_w / parts;
    double cum = 0.0, target = step;
    int32_t j = 0;
    const Cand *prev = nullptr;
    for (size_t i = 0; i < cand.size() && j < parts - 1; ++i) {
        cum += (double)cand[i].w;
        if (cum >= target) {
            if (!prev || lt(*prev, cand[i])) {
                if (out_bounds) {
                    if (kb == 8) std::memcpy((char *)out_bounds + (size_t)j * 8, &cand[i].k64, 8);
                    else std::memcpy((char *)out_bounds + (size_t)j * 10, cand[i].k10.data(), 10);
                }
                target += step;
                ++j;
                prev = &cand[i];
            }
        }
    }
    *out_nbounds = j;
    return SGX_OK;
}

// ------------------------------------------------------------------------------------
// LZ4BlockOutputStream framing of partition streams (spark.shuffle.compress=true, lz4)
// ------------------------------------------------------------------------------------
// caller holds e->mu; alloc_dst: allocate the destination (exact size) instead of dst_dev
static int lz4_frame_impl(sgx_engine *e, const void *stream_dev, const int64_t *part_offsets,
                          int32_t num_partitions, int32_t block_size, DevBuf *alloc_dst, void *dst_dev,
                          int64_t dst_cap, int64_t *out_lengths) {
    if (!e || !part_offsets || !out_lengths || num_partitions < 1)
        return fail(SGX_ERR_INVALID, "sgx_lz4_frame_partitions: bad arguments");
    if (block_size < 64 || block_size > sgx::lz4_max_block())
        return fail(SGX_ERR_UNSUPPORTED, "LZ4 block size %d outside [64, %d]", block_size, sgx::lz4_max_block());
    const int R = num_partitions;
    std::vector<int64_t> blocks;  // {src offset, length} per block
    std::vector<int32_t> first(R + 1);
    for (int r = 0; r < R; ++r) {
        first[r] = (int32_t)(blocks.size() / 2);
        int64_t a = part_offsets[r], b = part_offsets[r + 1];
        if (b < a || a < 0) return fail(SGX_ERR_INVALID, "partition offsets decrease at %d", r);
        for (int64_t p = a; p < b; p += block_size) {
            blocks.push_back(p);
            blocks.push_back(std::min<int64_t>(block_size, b - p));
        }
    }
    const int64_t nb = (int64_t)blocks.size() / 2;
    first[R] = (int32_t)nb;
    if (nb > 0 && !stream_dev) return fail(SGX_ERR_INVALID, "stream is NULL");
    // lz4-java: level = max(0, 32 - nlz(blockSize - 1) - COMPRESSION_LEVEL_BASE (10))
    const int level = std::max(0, 32 - __builtin_clz((unsigned)(block_size - 1)) - 10);
    const int64_t slot = ((int64_t)21 + block_size + block_size / 255 + 16 + 15) / 16 * 16;
    HIP_TRY(hipSetDevice(e->device));
    DevBuf d_blocks, d_slots, d_sizes, d_offs;
    DevBufScope g1{d_blocks}, g2{d_slots}, g3{d_sizes}, g4{d_offs};
    std::vector<int32_t> sizes(nb);
    if (nb > 0) {
        SGX_TRY(d_blocks.ensure((size_t)nb * 16));
        SGX_TRY(d_slots.ensure((size_t)(nb * slot)));
        SGX_TRY(d_sizes.ensure((size_t)nb * 4));
        HIP_TRY(hipMemcpyAsync(d_blocks.p, blocks.data(), (size_t)nb * 16, hipMemcpyHostToDevice, e->s_comp));
        HIP_TRY(sgx::launch_lz4_blocks((const uint8_t *)stream_dev, (const int64_t *)d_blocks.p, nb, level,
                                       (uint8_t *)d_slots.p, slot, (int32_t *)d_sizes.p, e->s_comp));
        HIP_TRY(hipMemcpyAsync(sizes.data(), d_sizes.p, (size_t)nb * 4, hipMemcpyDeviceToHost, e->s_comp));
        HIP_TRY(hipStreamSynchronize(e->s_comp));
    }
    // frame offsets (blocks of a partition back to back, then its end mark)
    std::vector<int64_t> offs((size_t)nb + R);  // nb frame offsets | end-mark offsets
    int64_t total = 0, nends = 0;
    for (int r = 0; r < R; ++r) {
        int64_t start = total;
        for (int32_t b = first[r]; b < first[r + 1]; ++b) {
            if (sizes[b] < 21 || sizes[b] > slot) return fail(SGX_ERR_HIP, "LZ4 block %d: bad frame size %d", b, sizes[b]);
            offs[b] = total;
            total += sizes[b];
        }
        if (first[r + 1] > first[r]) {
            offs[nb + nends++] = total;
            total += 21;
        }
        out_lengths[r] = total - start;
    }
    if (alloc_dst) {
        SGX_TRY(alloc_dst->ensure((size_t)total));
        dst_dev = alloc_dst->p;
        dst_cap = total;
    }
    if (!dst_dev) return SGX_OK;
    if (total > dst_cap)
        return fail(SGX_ERR_INVALID, "LZ4 frames need %lld bytes, destination holds %lld", (long long)total,
                    (long long)dst_cap);
    if (nb > 0) {
        SGX_TRY(d_offs.ensure((size_t)(nb + nends) * 8));
        HIP_TRY(hipMemcpyAsync(d_offs.p, offs.data(), (size_t)(nb + nends) * 8, hipMemcpyHostToDevice, e->s_comp));
        HIP_TRY(sgx::launch_lz4_gather((const uint8_t *)d_slots.p, slot, (const int32_t *)d_sizes.p,
                                       (const int64_t *)d_offs.p, nb, (const int64_t *)d_offs.p + nb, nends, level,
                                       (uint8_t *)dst_dev, e->s_comp));
        HIP_TRY(hipStreamSynchronize(e->s_comp));
    }
    return SGX_OK;
}

extern "C" int sgx_lz4_frame_partitions(sgx_engine *e, const void *stream_dev, const int64_t *part_offsets,
                                        int32_t num_partitions, int32_t block_size, void *dst_dev,
                                        int64_t dst_cap, int64_t *out_lengths) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    return lz4_frame_impl(e, stream_dev, part_offsets, num_partitions, block_size, nullptr, dst_dev, dst_cap,
                          out_lengths);
}

// LZ4BlockInputStream on the reduce side: decompress fetched LZ4-framed partition streams
extern "C" int sgx_lz4_unframe(sgx_engine *e, const void *framed_dev, int64_t framed_bytes, void *dst_dev,
                               int64_t dst_cap, int64_t *out_bytes) {
    if (!e) return fail(SGX_ERR_INVALID, "engine is NULL");
    std::lock_guard<std::mutex> lk(e->mu);
    return lz4_unframe_impl(e, framed_dev, framed_bytes, nullptr, dst_dev, dst_cap, out_bytes);
}

// caller holds e->mu; alloc_dst: size (decompressed + 64 B of decoder padding) and use it
static int lz4_unframe_impl(sgx_engine *e, const void *framed_dev, int64_t framed_bytes, DevBuf *alloc_dst,
                            void *dst_dev, int64_t dst_cap, int64_t *out_bytes) {
    if (!e || !out_bytes || framed_bytes < 0 || (framed_bytes > 0 && !framed_dev))
        return fail(SGX_ERR_INVALID, "sgx_lz4_unframe: bad arguments");
    *out_bytes = 0;
    if (framed_bytes == 0) return SGX_OK;
    HIP_TRY(hipSetDevice(e->device));
    // one walk normally suffices: room for a frame per 512 B of input (frames of full 32 KiB
    // blocks are ~64x sparser); a denser stream (tiny partitions) is walked again with room
    // for every frame
    int64_t cap = framed_bytes / 512 + 4096;
    DevBuf d_info, d_desc;
    DevBufScope g1{d_info}, g2{d_desc};
    SGX_TRY(d_info.ensure(64));
    int64_t info[5];
    for (int pass = 0; pass < 2; ++pass) {
        SGX_TRY(d_desc.ensure((size_t)cap * 16));
        HIP_TRY(hipMemsetAsync(d_info.p, 0, 64, e->s_comp));
        HIP_TRY(sgx::launch_lz4_walk((const uint8_t *)framed_dev, framed_bytes, (int64_t *)d_desc.p, cap,
                                     (int64_t *)d_info.p, e->s_comp));
        HIP_TRY(hipMemcpyAsync(info, d_info.p, 40, hipMemcpyDeviceToHost, e->s_comp));
        HIP_TRY(hipStreamSynchronize(e->s_comp));
        if (info[2] != 0 || info[0] <= cap || (!dst_dev && !alloc_dst)) break;
        cap = info[0];
    }
    static const char *why[] = {"", "truncated header", "bad magic", "unknown compression method",
                                "malformed end mark", "bad block lengths"};
    if (info[2] != 0)
        return fail(SGX_ERR_INVALID, "LZ4 stream: %s at byte %lld", why[info[2] < 6 ? info[2] : 0],
                    (long long)info[3]);
    const int64_t nframes = info[0];
    *out_bytes = info[1];
    if (alloc_dst) {
        SGX_TRY(alloc_dst->ensure((size_t)info[1] + 64));
        dst_dev = alloc_dst->p;
        dst_cap = info[1];
    }
    if (!dst_dev) return SGX_OK;
    if (info[1] > dst_cap)
        return fail(SGX_ERR_INVALID, "LZ4 stream decodes to %lld bytes, destination holds %lld",
                    (long long)info[1], (long long)dst_cap);
    if (nframes == 0) return SGX_OK;
    HIP_TRY(sgx::launch_lz4_decode((const uint8_t *)framed_dev, (const int64_t *)d_desc.p, nframes,
                                   (uint8_t *)dst_dev, (uint32_t *)((int64_t *)d_info.p + 4), e->s_comp));
    uint32_t derr = 0;
    HIP_TRY(hipMemcpyAsync(&derr, (int64_t *)d_info.p + 4, 4, hipMemcpyDeviceToHost, e->s_comp));
    HIP_TRY(hipStreamSynchronize(e->s_comp));
    if (derr & 1u) return fail(SGX_ERR_INVALID, "LZ4 stream: corrupt compressed block");
    if (derr & 2u) return fail(SGX_ERR_INVALID, "LZ4 stream: block checksum mismatch");
    return SGX_OK;
}
