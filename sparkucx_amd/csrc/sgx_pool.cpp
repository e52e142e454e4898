// sgx_pool.cpp — the MemoryPool of the fetch contract (memory/MemoryPool.scala:22-147): the
// BufferAllocator (ShuffleTransport.scala:113) that hands out the MemoryBlocks fetched blocks
// land in, returned to the pool by MemoryBlock.close().  The reference pools UCX-registered
// host memory in power-of-two size classes from spark.shuffle.ucx.memory.minBufferSize
// (4 KiB) with per-class free stacks (:34-110) and optional preallocation (:141-147).  Here
// the same classes hold pinned host memory (hipHostMalloc: DMA-able by the GPU, what a
// host-side fetch destination needs) or HBM (device destinations for the GPU reader).
#include "sgx_engine.h"

#include <algorithm>

using namespace sgx;

namespace sgx {
struct PoolState {
    std::mutex mu;
    struct Entry {
        int kind;
        int cls;
    };
    std::unordered_map<void *, Entry> out;       // handed-out blocks
    std::vector<void *> free_[2][48];            // [mem kind][size class]
    int64_t allocated = 0, idle = 0;             // bytes
    ~PoolState() {
        for (int k = 0; k < 2; ++k)
            for (auto &v : free_[k])
                for (void *p : v) (void)(k == SGX_MEM_HOST ? hipHostFree(p) : hipFree(p));
        for (auto &kv : out) (void)(kv.second.kind == SGX_MEM_HOST ? hipHostFree(kv.first) : hipFree(kv.first));
    }
};
}  // namespace sgx

static constexpr int64_t kMinBuffer = 4096;  // spark.shuffle.ucx.memory.minBufferSize default

static int size_class(int64_t size) {  // smallest c with (kMinBuffer << c) >= size
    int c = 0;
    while ((kMinBuffer << c) < size) ++c;
    return c;
}

static PoolState &pool(sgx_engine *e) {
    std::lock_guard<std::mutex> lk(e->reg_mu);
    if (!e->pool) e->pool.reset(new PoolState());
    return *e->pool;
}

static int pool_alloc(int kind, int64_t bytes, void **p) {
    const hipError_t r = kind == SGX_MEM_HOST ? hipHostMalloc(p, (size_t)bytes, hipHostMallocDefault)
                                              : hipMalloc(p, (size_t)bytes);
    if (r != hipSuccess) return fail_msg(SGX_ERR_NOMEM, "pool allocation of %lld bytes: %s", (long long)bytes,
                                         hipGetErrorString(r));
    return SGX_OK;
}

extern "C" int sgx_pool_get(sgx_engine *e, int64_t size, int32_t mem_kind, void **out_ptr, int64_t *out_cap) {
    if (!e || !out_ptr || !out_cap || size < 0 || size > ((int64_t)1 << 40) ||
        (mem_kind != SGX_MEM_HOST && mem_kind != SGX_MEM_DEVICE))
        return fail_msg(SGX_ERR_INVALID, "sgx_pool_get: bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    PoolState &ps = pool(e);
    const int c = size_class(size);
    const int64_t cap = kMinBuffer << c;
    void *p = nullptr;
    {
        std::lock_guard<std::mutex> lk(ps.mu);
        auto &fl = ps.free_[mem_kind][c];
        if (!fl.empty()) {
            p = fl.back();
            fl.pop_back();
            ps.idle -= cap;
        }
    }
    if (!p) {
        SGX_TRY(pool_alloc(mem_kind, cap, &p));
        std::lock_guard<std::mutex> lk(ps.mu);
        ps.allocated += cap;
    }
    std::lock_guard<std::mutex> lk(ps.mu);
    ps.out[p] = PoolState::Entry{mem_kind, c};
    *out_ptr = p;
    *out_cap = cap;
    return SGX_OK;
}

extern "C" int sgx_pool_put(sgx_engine *e, void *ptr) {
    if (!e || !ptr) return fail_msg(SGX_ERR_INVALID, "sgx_pool_put: bad arguments");
    PoolState &ps = pool(e);
    std::lock_guard<std::mutex> lk(ps.mu);
    auto it = ps.out.find(ptr);
    if (it == ps.out.end()) return fail_msg(SGX_ERR_INVALID, "sgx_pool_put: %p was not handed out by this pool", ptr);
    ps.free_[it->second.kind][it->second.cls].push_back(ptr);
    ps.idle += kMinBuffer << it->second.cls;
    ps.out.erase(it);
    return SGX_OK;
}

extern "C" int sgx_pool_preallocate(sgx_engine *e, int64_t size, int32_t count, int32_t mem_kind) {
    if (!e || size < 0 || size > ((int64_t)1 << 40) || count < 0 || (mem_kind != SGX_MEM_HOST && mem_kind != SGX_MEM_DEVICE))
        return fail_msg(SGX_ERR_INVALID, "sgx_pool_preallocate: bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    PoolState &ps = pool(e);
    const int c = size_class(size);
    const int64_t cap = kMinBuffer << c;
    for (int32_t i = 0; i < count; ++i) {
        void *p = nullptr;
        SGX_TRY(pool_alloc(mem_kind, cap, &p));
        std::lock_guard<std::mutex> lk(ps.mu);
        ps.free_[mem_kind][c].push_back(p);
        ps.allocated += cap;
        ps.idle += cap;
    }
    return SGX_OK;
}

extern "C" int sgx_pool_stats(sgx_engine *e, int64_t *out_allocated, int64_t *out_idle) {
    if (!e || !out_allocated || !out_idle) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    PoolState &ps = pool(e);
    std::lock_guard<std::mutex> lk(ps.mu);
    *out_allocated = ps.allocated;
    *out_idle = ps.idle;
    return SGX_OK;
}
