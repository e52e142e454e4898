// sgx_engine.h — the engine's internal state, shared by the C-ABI translation units
// (sgx_engine.cpp, sgx_map.cpp, sgx_exchange.cpp, sgx_read.cpp, sgx_lz4_host.cpp,
// sgx_range.cpp).  Not part of the public ABI (include/sgx.h).
//
// Threading model (SURVEY §8(b) "Threading"; the reference routes each calling thread to its
// own UCX worker, UcxShuffleTransport.scala:277-296): every calling thread gets its own
// context -- a HIP stream plus private scratch buffers -- so concurrent map tasks of one
// executor run their kernels side by side on the GPU and never share a work buffer.  Shared
// state is guarded by short-lived locks, never held across a device wait of another thread:
//   reg_mu     the shuffle registry and the context table
//   Shuffle::mu   a shuffle's map / round containers
//   MapOut::mu    one map output (its writer, its lengths)
//   comm_mu    the exchange: collectives are issued by one thread at a time, in call order,
//              on the engine's exchange stream (RCCL needs the same order on every rank)
//   stats_mu   stage timing events
// Lock order: reg_mu -> Shuffle::mu -> MapOut::mu; comm_mu before Shuffle::mu.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <map>
#include <memory>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/sgx.h"
#include "sgx_internal.h"

#include <rocprofiler-sdk-roctx/roctx.h>

namespace sgx {
// roctx range around a C-ABI call (SURVEY §5 tracing): `rocprofv3 --marker-trace` shows the
// engine's calls beside the kernels they launch; a no-op when no tool is attached.
struct TraceRange {
    explicit TraceRange(const char *name) { roctxRangePushA(name); }
    ~TraceRange() { roctxRangePop(); }
    TraceRange(const TraceRange &) = delete;
    TraceRange &operator=(const TraceRange &) = delete;
};


#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return ::sgx::fail_msg(SGX_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                                   __FILE__, __LINE__);                                        \
    } while (0)
#define NCCL_TRY(expr)                                                                         \
    do {                                                                                       \
        ncclResult_t _r = (expr);                                                              \
        if (_r != ncclSuccess)                                                                 \
            return ::sgx::fail_msg(SGX_ERR_COMM, "%s failed: %s", #expr, ncclGetErrorString(_r)); \
    } while (0)
#define SGX_TRY(expr)                                                                          \
    do {                                                                                       \
        int _c = (expr);                                                                       \
        if (_c != SGX_OK) return _c;                                                           \
    } while (0)

// ------------------------------------------------------------------------------------
// buffers
// ------------------------------------------------------------------------------------
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    // grow-only: keeps the allocation when it is large enough
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return SGX_OK;
        release();
        size_t want = bytes ? bytes : 16;
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return fail_msg(SGX_ERR_NOMEM, "hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
        }
        cap = want;
        return SGX_OK;
    }
    void swap(DevBuf &o) {
        std::swap(p, o.p);
        std::swap(cap, o.cap);
    }
};

// memcpy over a few threads (sgx_engine.cpp): sgx_map_append's pinned staging of host batches
void host_copy_parallel(char *dst, const char *src, size_t bytes);

struct HostPinned {
    void *p = nullptr;
    size_t cap = 0;
    HostPinned() = default;
    HostPinned(const HostPinned &) = delete;
    HostPinned &operator=(const HostPinned &) = delete;
    ~HostPinned() { release(); }
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
            return fail_msg(SGX_ERR_NOMEM, "hipHostMalloc(%zu) failed: %s", want, hipGetErrorString(e));
        }
        cap = want;
        return SGX_OK;
    }
};

struct Event {  // a lazily created, timing-disabled event
    hipEvent_t ev = nullptr;
    Event() = default;
    Event(const Event &) = delete;
    Event &operator=(const Event &) = delete;
    ~Event() {
        if (ev) (void)hipEventDestroy(ev);
    }
    hipError_t record(hipStream_t st) {
        if (!ev) {
            hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        return hipEventRecord(ev, st);
    }
    hipError_t wait_host() const { return ev ? hipEventSynchronize(ev) : hipSuccess; }
};

// ------------------------------------------------------------------------------------
// registry
// ------------------------------------------------------------------------------------
// One partition-contiguous batch of records of a streaming map output (a "spill": the
// reference's writer receives unbounded partition streams, NvkvShuffleMapOutputWriter.scala:
// 106-113, 228-246; Spark merges spills in spill order).
struct Spill {
    DevBuf data;                   // published bytes of this batch, partition-contiguous
                                   // (deferred: the batch's records as appended, engine copy)
    std::vector<int64_t> lengths;  // [R] published bytes per partition
    int64_t nrec = 0;
    const void *src = nullptr;     // deferred: the batch's records (in the map's landing
                                   // area, or the caller's SGX_MEM_DEVICE_RETAINED buffer)
    bool landed = false;           // deferred: copied into the map's landing area
};

struct MapOut {
    std::mutex mu;             // serialises the writer(s) and the length finisher of this map
    bool written = false;      // a write was enqueued successfully
    DevBuf data;               // partition-contiguous records (engine-owned HBM)
    int64_t nrec = 0;
    HostPinned part_off;       // (R+1) u32 record offsets + 1 u32 error word, landed async
    std::vector<int64_t> lengths;  // published bytes per partition (valid once `ready`)
    bool ready = false;
    Event done;                // recorded on the writer's stream after the last producer kernel
    Event read_done;           // recorded on the exchange stream after an all-to-all read it
    // serializer KRYO: the published bytes are the Kryo stream of the records
    DevBuf ser;                // Kryo-framed partition-contiguous bytes (capacity 20 n + 16)
    DevBuf ser_work;           // device (R+1) i64 byte offsets | tile prefixes | tile sums
    HostPinned ser_off;        // (nseg+1) i64 byte offsets, landed async
    // SGX_WRITER_UNSAFE, compressed, several spills: the Kryo stream is cut into nseg = R x
    // spills segments (partition-major, spill-minor), each framed as its own LZ4 stream
    int32_t seg_spills = 1;    // spills per partition segment list (1 = one segment per partition)
    DevBuf seg_off;            // device (R x seg_spills + 1) u32 record offsets of the segments
    int64_t out_bytes = 0;     // published bytes
    DevBuf comp;               // LZ4-framed partition streams (sgx_set_compression), once `ready`
    bool comp_valid = false;   // `comp` holds this write's frames (false until finish_lengths)
    // streaming writes (sgx_map_begin / _append / _commit): the batches so far
    bool open = false;
    std::vector<std::unique_ptr<Spill>> spills;
    // deferred (sgx_map.cpp deferred_ok): the batches are kept as appended and the commit
    // partitions all of them in one pass through a chunk table
    bool deferred = false;
    HostPinned chunk_host;     // [2G] i64 {byte offset from the first batch, records} | [S] i32 first chunk per batch
    DevBuf chunk_dev;
    // deferred: the landing area of copied batches, packed back to back in append order into
    // large segments, so a run of batches is one region of the commit's chunk table (the
    // chunk count stays ~one per CU whatever the number of batches)
    std::vector<std::unique_ptr<DevBuf>> landing;
    size_t land_used = 0;      // bytes used in landing.back()
    // Single-pass padded output (sgx_map.cpp padded_pass): `data` holds one
    // line-aligned sub-bin per (partition, chunk) stream with unwritten gaps between them;
    // frag = device [fstart][foff][cnt] u32 x R*G: a stream's first record in `data`, its
    // position in the contiguous layout, its record count.  pad_try: this write ran the
    // padded kernels (the layout is decided when its lengths land: padded, or -- a sub-bin
    // overflowed -- rewritten contiguous by the fallback).  Consumers that need contiguous
    // bytes (view(): exchange sends, map data, index files) use `dense`, built once by
    // materialize(); fetches gather the fragments directly.
    bool pad_try = false;
    bool padded = false;       // valid once `ready`
    bool rec_padded = false;   // the records were written padded (a Kryo map: SGX_LAYOUT_SERIALIZED_PADDED)
    int32_t frag_G = 0;
    DevBuf frag;
    DevBuf dense;
    bool dense_valid = false;
    const void *view() const {
        return comp_valid ? comp.p : (ser.p && ser_valid ? ser.p : (padded ? (dense_valid ? dense.p : nullptr) : data.p));
    }
    bool ser_valid = false;    // `ser` holds this write's Kryo stream
    bool exchanged = false;    // an exchange round carried this write (sgx_exchange skips it)
    ~MapOut() {
        (void)read_done.wait_host();  // an all-to-all may still read `data`
        (void)done.wait_host();
    }
};

// One exchange round: every rank pushed the maps it contributed (any number, 0 included);
// this rank holds its reducers' blocks of all of them.  The receive buffer is laid out
// [source rank][that rank's maps, in its order][my reducers]: every (map, reducer) block is
// contiguous in it, so blocks are served from it directly and the per-reducer canonical
// order (reducer, then map) is produced by the fetch that asks for it (one gather launch),
// not by an extra pass over every received byte.
struct Round {
    std::vector<int64_t> map_ids;        // [M] every map of the round, source-rank-major
    std::vector<int32_t> src;            // [M] the rank that pushed it
    std::vector<int64_t> lens;           // [M][R] bytes
    std::vector<int64_t> block_off;      // [M][nmine] byte offset in `data` (or in alias[j])
    int32_t r0 = 0, r1 = 0;              // my reducers [r0, r1)
    DevBuf data;                          // receive buffer
    // the receive buffer's IPC handle (the direct peer gather), taken once per allocation: it
    // moves with `data` when a re-run round reuses the buffer, so peers keep their mapping
    hipIpcMemHandle_t ipc{};
    bool ipc_valid = false;
    uint64_t ipc_gen = 0;  // this rank's serial of the allocation: peers key their mappings on it
    // P == 1 without a communicator: the map outputs themselves ([M], block_off inside each)
    std::vector<std::shared_ptr<MapOut>> alias;
    // sgx_import_blocks: blocks a reader fetched from elsewhere (0 = an exchange round)
    int64_t import_id = 0;
    Event done;
    const char *block_ptr(size_t j, int32_t r) const {
        const size_t nmine = (size_t)(r1 - r0);
        const char *b = alias.empty() ? (const char *)data.p : (const char *)alias[j]->view();
        return b + block_off[j * nmine + (size_t)(r - r0)];
    }
    ~Round() { (void)done.wait_host(); }
};

struct Shuffle {
    std::mutex mu;                // maps / rounds containers
    int32_t id = 0;
    int32_t R = 0, kind = 0, nb = 0, asc = 1, rb = 16;
    int32_t ser = SGX_SER_FIXED;  // dep.serializer (sgx_set_serializer)
    int32_t lz4_block = 0;        // spark.shuffle.compress with lz4 (sgx_set_compression): block size
    int32_t combine = -1;         // map-side combine aggregation (sgx_set_map_side_combine), -1 = none
    int32_t writer = SGX_WRITER_SORT;  // the map writer of the shuffle's handle (sgx_set_map_writer)
    std::atomic<int32_t> placement{SGX_PLACE_EVEN};  // reducer placement of exchange rounds
    // the reducer ranges of every rank, bounds[P + 1], fixed by the shuffle's first exchange
    // round (empty before): a reducer's blocks from every round land on the same rank
    std::vector<int32_t> place_bounds;
    DevBuf bounds;                // the bounds, then (dir_ok) their top-bits directory at dir_off
    bool dir_ok = false;
    size_t dir_off = 0;
    PartParams pp{};
    std::map<int64_t, std::shared_ptr<MapOut>> maps;
    std::vector<std::shared_ptr<Round>> rounds;
    int64_t next_import = 1;      // sgx_import_blocks ids
    // a padded write of this shuffle overflowed its sub-bins (keys not spread like the
    // sample): its later maps take the two-pass path directly
    std::atomic<bool> pad_failed{false};
    bool configurable() {  // serializer / codec / combine may change until the first write
        std::lock_guard<std::mutex> lk(mu);
        return maps.empty();
    }
};

// ------------------------------------------------------------------------------------
// per-thread context: a HIP stream and private scratch
// ------------------------------------------------------------------------------------
struct Ctx {
    hipStream_t st = nullptr;
    uint64_t ops = 0;  // API calls made with this context (sgx_engine::ctx)
    // The last reduce-side result computed on this context: a size query (NULL destination)
    // leaves it here and the filling call that follows it directly on the same thread, with
    // the same arguments and no mutation of the engine in between, reuses it instead of
    // fetching / decoding / sorting / grouping again.
    struct ReadCache {
        uint64_t ops = ~0ull, epoch = 0;
        int32_t sid = -1, kind = -1, agg = -1, r0 = 0, r1 = 0;
        std::vector<int64_t> maps;
        int64_t n = 0, ng = 0;
        const void *sorted = nullptr;
        int64_t *keys = nullptr, *starts = nullptr, *vals = nullptr;
    } rc;
    // map side: [counts][ticket | look-back status][partition offsets | error] + offs[R][G]
    DevBuf offs, work;
    DevBuf split_work, split_tmp;  // R > 1024: the two-level split scatter's scratch and level-1 output
    DevBuf input_stage;
    // host batches of a streaming map: two pinned staging buffers, each reused once its last
    // copy to HBM has run (the caller's buffer is free as soon as it is copied into one)
    HostPinned host_stage[2];
    Event host_up[2];
    int host_slot = 0;
    // pre-aggregation records of the last read on this thread (sgx_last_read_records)
    int64_t last_read_records = 0;
    const uint32_t *last_off_dev = nullptr;  // device (R+1) record offsets of the last partition pass
    // The padded write's tail (its scan, the guarded two-pass fallback, the offsets' copy to the
    // host) runs on a second stream so that the next write's kernels do not queue behind it;
    // its work block and offsets alternate between two slots, a slot reused only once the tail
    // that last read it has run (pad_done)
    hipStream_t st_tail = nullptr;
    DevBuf pad_work[2], pad_offs[2];
    // The padded split's front (sample, hot cut, capacities, cursors) runs on a third stream:
    // it reads only its own map's input, so it overlaps the previous write's level 2; its
    // scratch alternates with the slots (split_pad[slot]), and level 1 waits for pre_done[slot]
    hipStream_t st_pre = nullptr;
    DevBuf split_pad[2];
    Event pre_done[2], pre_in;
    // 16 B padded writes: the sample's block per slot ([est][K4 flags][layout]), how many of its
    // leading bytes the slot's last tail left zeroed (its next sample needs them zero), and the
    // event behind that reset (the next write on the slot waits for it, not for the whole tail)
    DevBuf pad_crit[2];
    size_t pad_crit_zeroed[2] = {0, 0};
    Event pad_free[2];
    Event pad_done[2];
    int pad_slot = 0, tail_slot = -1;
    // Host records into input_stage on stream `s`, behind the last padded-write tail: its
    // guarded fallback still reads its map's input, which may be this buffer (a growth waits
    // for that tail on the host, since the old allocation is freed).
    int stage_input(const void *src, size_t bytes, hipStream_t s, const void **out) {
        const hipEvent_t tail = tail_slot >= 0 ? pad_done[tail_slot].ev : nullptr;
        if (tail && bytes > input_stage.cap) HIP_TRY(hipEventSynchronize(tail));
        SGX_TRY(input_stage.ensure(bytes));
        if (tail) HIP_TRY(hipStreamWaitEvent(s, tail, 0));
        HIP_TRY(hipMemcpyAsync(input_stage.p, src, bytes, hipMemcpyHostToDevice, s));
        *out = input_stage.p;
        return SGX_OK;
    }
    // reduce side and map-side combine
    DevBuf kryo_in, kryo_work, sort_buf[2], sort_err, grp_status, grp_out;
    DevBuf digit_hist, items_dev, gather_stage, fetch_tmp, comb_buf;
    // records of each partition in c.sort_buf[0] after the last fixed-codec gather (canonical
    // reducer-major order: the partitions are contiguous), empty when unknown (Kryo reads)
    std::vector<int64_t> gather_part_recs;
    DevBuf seg_work;  // the segmented window pass: [desc][ndesc | seg_end][counts][offsets]
    HostPinned seg_desc_host;
    HostPinned gather_items;
    HostPinned seg_host;  // (partition, spill) segment offsets of an UnsafeShuffleWriter commit
    // LZ4 framing / unframing scratch (grow-only)
    DevBuf lz4_blocks, lz4_slots, lz4_sizes, lz4_offs, lz4_info, lz4_desc;
    HostPinned lz4_host;  // pinned staging of the block list / frame sizes / frame offsets
    // RangePartitioner.sketch
    DevBuf sample_winner, sample_keys, cdf;
    ~Ctx() {
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
        if (st_tail) {
            (void)hipStreamSynchronize(st_tail);
            (void)hipStreamDestroy(st_tail);
        }
        if (st_pre) {
            (void)hipStreamSynchronize(st_pre);
            (void)hipStreamDestroy(st_pre);
        }
    }
};

struct PendingStage {
    int stage;
    hipEvent_t a, b;
};

struct PoolState;  // sgx_pool.cpp

}  // namespace sgx

struct sgx_engine {
    // bumped by every call that changes what a read could return (maps, rounds, shuffle
    // properties): a cached read result is valid only for the epoch it was computed in
    std::atomic<uint64_t> epoch{0};
    void mutated() { epoch.fetch_add(1, std::memory_order_relaxed); }
    int device = 0;
    int num_cus = 256;
    int G = 256;
    bool G_forced = false;
    int sc_waves = 0, sc_items = 0;  // K4 geometry override (sgx_config)
    int hist_mode = 0;               // sgx_config.hist_mode
    int rank_mode = 0;               // sgx_config.rank_mode
    int flags = 0;                   // sgx_config.flags
    // consecutive padded writes of a thread alternate between two streams (sgx_set_overlap_writes)
    std::atomic<bool> overlap_writes{true};
    bool lds_order_ok = true;        // engine-start check (sgx_create; sgx_lds_order_ok)
    int64_t pad_min = 1 << 20;       // smallest map written padded (SGX_FLAG_PAD_ANY_SIZE: 1)
    int64_t comm_timeout_ms = 300000;

    std::mutex reg_mu;
    std::map<int32_t, std::shared_ptr<sgx::Shuffle>> shuffles;
    std::unordered_map<std::thread::id, std::unique_ptr<sgx::Ctx>> ctxs;

    // exchange
    std::mutex comm_mu;
    hipStream_t s_comm = nullptr;
    ncclComm_t comm = nullptr;
    bool host_comm = false;
    sgx_host_comm hc{};
    bool comm_broken = false;
    int32_t nranks = 1, rank = 0;
    sgx::DevBuf ag_send, ag_recv;
    sgx::HostPinned ag_host, x_send, x_recv;
    // RCCL exchange of a rank holding many small maps: its pieces packed per destination
    sgx::DevBuf x_pack, x_items_dev;
    sgx::HostPinned x_items;
    // the direct peer gather: its descriptors' upload (reused by the next round once done),
    // peers' receive buffers still mapped by a round whose gather may be running (closed once
    // the round's event has passed), and the RCCL completion barrier's word
    sgx::Event x_items_up;
    // peers' receive buffers mapped by the direct peer gather, by handle: kept open across
    // rounds (a re-run round reuses its buffer, so its handle comes back); closed once unused
    // for a few rounds and the last gather into it has finished
    struct PeerMap {
        void *ptr = nullptr;
        uint64_t last_round = 0;
        hipEvent_t done = nullptr;  // behind the last round's gather that wrote into it
    };
    std::map<std::string, PeerMap> p2p_cache;  // key: rank, allocation serial, handle bytes
    uint64_t p2p_rounds = 0, p2p_gen = 0;
    // the direct peer gather failed to map a peer's buffer on some rank: every later round
    // moves contiguous pieces (RCCL send / recv, host all-to-all) and maps are written two-pass
    std::atomic<bool> p2p_off{false};
    sgx::DevBuf p2p_word;
    sgx::DevBuf jump_dev;  // XORShiftRandom jump table (built once, read-only after)
    std::mutex jump_mu;
    std::shared_ptr<sgx::PoolState> pool;  // MemoryPool (sgx_pool.cpp), created on first use

    // stats
    std::mutex stats_mu;
    std::vector<hipEvent_t> ev_free;
    std::vector<sgx::PendingStage> pending;
    double stage_ms[SGX_NUM_STAGES] = {0};
    int64_t stage_n[SGX_NUM_STAGES] = {0};
    // exchange bytes: [0] sent to other ranks, [1] kept by this rank, [2] rounds (sgx_exchange_bytes)
    int64_t x_bytes[3] = {0, 0, 0};

    // the calling thread's context (created on first use); nullptr + last_error on failure
    sgx::Ctx *ctx();
    hipEvent_t ev();
    void record_stage(int stage, hipEvent_t a, hipEvent_t b);
    void release_events(std::initializer_list<hipEvent_t> evs);
    void resolve_stats();
    std::shared_ptr<sgx::Shuffle> find_shuffle(int32_t shuffle_id);
};

namespace sgx {

// ---- shared internals (defined across the engine's translation units) ----
// SGX_FLAG_DEBUG_SYNC: synchronise `st` and report a device error naming `what`.
int debug_sync(sgx_engine *e, hipStream_t st, const char *what);
PartParams make_part_params(const Shuffle &s);
// A streaming map's batches as the map side's chunks (sgx_map_commit of deferred batches):
// chunk g = chunks[2g+1] records at byte chunks[2g] from the pass's input pointer, every
// chunk inside one batch, at most `chunk` records (a multiple of the K4 tile).
struct ChunkTable {
    const int64_t *dev = nullptr;
    int64_t chunk = 0;
    int G = 0;
    std::vector<int64_t> len;  // host copy of the chunks' record counts
};
// One stable partition pass (K1+K2 hist -> K3 scan -> K4 scatter) on the context's stream;
// with a chunk table its chunks replace the contiguous input's.
int partition_pass(sgx_engine *e, Ctx &c, const void *in, void *out, int64_t n, int rb, const PartParams &spp,
                   int32_t R, int32_t kind, uint32_t *host_off, uint32_t *err_slot, bool stats,
                   const ChunkTable *ct = nullptr);
// Lengths / published bytes of a written map (waits for its kernels).  Caller holds m.mu.
int finish_lengths(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m);
// A padded map's contiguous copy (m.dense, once; m.done is recorded behind it), so that
// view() is valid.  No-op for other maps.  Caller holds m.mu and ran finish_lengths.
int materialize(sgx_engine *e, Ctx &c, Shuffle &s, MapOut &m);
// Look up a map output (shared pointer: stays alive while used).
int find_map(sgx_engine *e, int32_t shuffle_id, int64_t map_id, std::shared_ptr<Shuffle> *ps,
             std::shared_ptr<MapOut> *pm);
// Gather blocks into dst (request order) on the context's stream; see sgx_read.cpp.  `keep`
// receives references to every source so it outlives an asynchronous gather.
int fetch_impl(sgx_engine *e, Ctx &c, Shuffle &s, const int64_t *map_ids, const int32_t *reduce_ids, int64_t n,
               void *dst, int64_t dst_cap, int32_t dst_mem_kind, int64_t *out_lengths, bool sync,
               std::vector<std::shared_ptr<void>> *keep);
// Group n key-sorted (Long, Long) records (device) by key, synchronously: *ngroups, and
// device arrays in the context's grp_out: keys[G], starts[G] (may be NULL), vals[G] sums
// (SGX_AGG_SUM) or vals[n] every value (SGX_AGG_GROUP).
int group_records(sgx_engine *e, Ctx &c, const void *sorted, int64_t n, int32_t agg, int64_t *ngroups,
                  int64_t **keys, int64_t **starts, int64_t **vals);
// Stable sort of n 16 B / 100 B records in c.sort_buf[0] by key, then by the shuffle's
// partitioner (when `by_partition`): *sorted = the buffer holding the result.
// nparts: partitions present in the records (a read's reducer range; 0 = all R), which sizes
// the bucket path's key window.  final_dst (device, n records, 16 B-aligned, not a sort buffer):
// the bucket path's last pass writes there directly -- *sorted == final_dst tells the caller
// no copy is left to do.
int sort_records(sgx_engine *e, Ctx &c, const Shuffle &s, int64_t n, bool by_partition, const void **sorted,
                 int32_t nparts = 0, void *final_dst = nullptr);
// LZ4 framing / unframing on the context's stream (sgx_lz4_host.cpp).
int lz4_frame_impl(sgx_engine *e, Ctx &c, const void *stream_dev, const int64_t *part_offsets, int32_t R,
                   int32_t block_size, DevBuf *alloc_dst, void *dst_dev, int64_t dst_cap, int64_t *out_lengths);
int lz4_unframe_impl(sgx_engine *e, Ctx &c, const void *framed_dev, int64_t framed_bytes, DevBuf *alloc_dst,
                     void *dst_dev, int64_t dst_cap, int64_t *out_bytes, const int64_t *stream_lens = nullptr,
                     int64_t nstreams = 0);
// Wait for the exchange stream with RCCL async-error polling and the engine's timeout.
int comm_wait(sgx_engine *e);

}  // namespace sgx
