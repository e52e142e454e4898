// Probe: which hipMalloc'd buffers hipIpcGetMemHandle accepts (sizes, reuse after hipFree).
#include <hip/hip_runtime.h>
#include <cstdio>
int main() {
    const size_t sizes[] = {16, 4096, 65536, 1 << 20, 2 << 20, 3 << 20, 64 << 20, 1ull << 30};
    for (int cyc = 0; cyc < 3; ++cyc)
        for (size_t sz : sizes) {
            void *p = nullptr;
            hipError_t e = hipMalloc(&p, sz);
            hipIpcMemHandle_t h;
            hipError_t e2 = e == hipSuccess ? hipIpcGetMemHandle(&h, p) : e;
            printf("cycle %d size %zu: malloc %s ipc %s ptr %p\n", cyc, sz, hipGetErrorString(e), hipGetErrorString(e2), p);
            if (cyc < 2) (void)hipFree(p);
        }
    // a buffer allocated, freed, and a different size allocated
    void *a, *b;
    hipMalloc(&a, 100 << 20); hipFree(a); hipMalloc(&b, 50 << 20);
    hipIpcMemHandle_t h;
    printf("realloc smaller: %s\n", hipGetErrorString(hipIpcGetMemHandle(&h, b)));
    return 0;
}
