// Probe (measurement tool, not product code): does one wave64 ds_add_rtn_u32 hand out the
// old values of same-address lanes in lane order?  Every wave runs many rounds; each round
// picks, per lane, one of K counters (K small => heavy same-address contention), issues a
// single atomicAdd(+1) and checks that for every pair of lanes l < m hitting the same
// counter, old[l] < old[m].  Prints the number of violations found.
//
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/mb_order tools/mb_lds_atomic_order.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <bool PACKED>
__global__ __launch_bounds__(512) void k(unsigned long long *viol, unsigned long long *checked, int rounds, int K) {
    __shared__ uint32_t cnt[8][1024];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned long long v = 0, c = 0;
    for (int i = threadIdx.x; i < 8 * 1024; i += 512) (&cnt[0][0])[i] = 0;
    __syncthreads();
    for (int r = 0; r < rounds; ++r) {
        const uint32_t h = mix((uint32_t)(blockIdx.x * 1000003u + w * 7919u + r * 104729u) ^ (lane * 0x9E3779B9u));
        const int kk = K > 0 ? K : 1 + (mix(blockIdx.x * 31u + w + r) & 63);
        const uint32_t p = h % (uint32_t)kk;
        uint32_t old;
        if (PACKED) {
            const uint32_t sh = (p & 1u) << 4;
            old = (atomicAdd(&cnt[w][p >> 1], 1u << sh) >> sh) & 0xFFFFu;
        } else {
            old = atomicAdd(&cnt[w][p], 1u);
        }
        // check: lanes with the same p must have old values increasing with lane id
        for (int m = 0; m < 64; ++m) {
            const uint32_t pm = __shfl(p, m, 64);
            const uint32_t om = __shfl(old, m, 64);
            if (pm == p && m < lane) { ++c; if (!(om < old)) ++v; }
        }
        if ((r & 255) == 255) {  // reset counters (keep u16 halves far from overflow)
            __syncthreads();
            for (int i = threadIdx.x; i < 8 * 1024; i += 512) (&cnt[0][0])[i] = 0;
            __syncthreads();
        }
    }
    atomicAdd(viol, v);
    atomicAdd(checked, c);
}

int main() {
    unsigned long long *d;
    hipMalloc(&d, 16);
    for (int packed = 0; packed < 2; ++packed)
        for (int K : {1, 2, 4, 16, 64, 512, 0}) {
            hipMemset(d, 0, 16);
            if (packed) k<true><<<2048, 512>>>(d, d + 1, 1024, K);
            else k<false><<<2048, 512>>>(d, d + 1, 1024, K);
            unsigned long long h[2];
            hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
            printf("{\"packed\": %d, \"K\": %d, \"violations\": %llu, \"pairs_checked\": %llu}\n", packed, K, h[0], h[1]);
        }
    return 0;
}
