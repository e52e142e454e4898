// Probe: a kernel bumps a 64-bit signal-memory counter (one system-scope atomic per
// workgroup, at its start); a second stream waits on the counter with hipStreamWaitValue64
// before its own kernel.  Prints the order the two kernels ran in (timestamps) and whether the
// waiting kernel started only after every workgroup of the first had started.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_long(unsigned long long *started, unsigned long long *t_first, int spin) {
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(started, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (blockIdx.x == 0) *t_first = wall_clock64();
    }
    unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < (unsigned long long)spin) {}
}

__global__ void k_after(const unsigned long long *started, unsigned long long *seen, unsigned long long *t) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        *seen = __hip_atomic_load(started, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        *t = wall_clock64();
    }
}

int main() {
    int ok = 0;
    CK(hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, 0));
    printf("CanUseStreamWaitValue %d\n", ok);
    unsigned long long *sig = nullptr, *out = nullptr;
    CK(hipExtMallocWithFlags((void **)&sig, 8, hipMallocSignalMemory));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(sig, 0, 8));
    CK(hipMemset(out, 0, 64));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    for (int rep = 0; rep < 3; ++rep) {
        const unsigned long long target = 256ull * (rep + 1);
        CK(hipStreamWaitValue64(b, sig, target, hipStreamWaitValueGte, ~0ull));
        hipLaunchKernelGGL(k_after, dim3(1), dim3(64), 0, b, sig, out + 1, out + 2);
        hipLaunchKernelGGL(k_long, dim3(256), dim3(64), 0, a, sig, out, 100000);  // ~1 ms at 100 MHz
        CK(hipStreamSynchronize(b));
        CK(hipStreamSynchronize(a));
        unsigned long long h[3];
        CK(hipMemcpy(h, out, 24, hipMemcpyDeviceToHost));
        printf("rep %d: counter seen %llu (target %llu), k_after - k_long start = %lld ticks\n", rep, h[1], target,
               (long long)(h[2] - h[0]));
    }
    printf("done\n");
    return 0;
}
