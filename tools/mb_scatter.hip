// Memory-only floor for K4's store pattern (measurement tool, not product code).
//
// N 16 B records, G chunks (one workgroup each), R partitions.  Tile t of chunk g holds
// TILE records already "sorted": slot s belongs to partition p = s / RUN (RUN = TILE / R)
// and goes to out[p * (N/R) + g * (N/R/G) + t * RUN + s % RUN] -- exactly where a uniform
// hash shuffle sends it.  No LDS, no ranking: coalesced loads, arithmetic destinations.
//
//   mode 0: coalesced copy (out[i] = in[i])
//   mode 1: the scatter pattern above (every run starts on a 128 B line)
//   mode 2: same runs, each (chunk, partition) stream shifted by 0..7 records: runs straddle
//           lines the way real cursors do (a line is finished by the next tile's run)
//   mode 3: shift 0 or 4 records: runs start on 64 B but not always on 128 B
//   mode 4: INTERLEAVED tiles: workgroup g's t-th tile is global tile t*G + g, and within a
//           partition the runs of consecutive global tiles are adjacent (one stream per
//           partition, shifted 0..7 records): a line straddling two runs is finished by the
//           neighbouring workgroup at about the same time, on another XCD
//   mode 5: as 4, XCD-aware: the 32 workgroups of one XCD (g % 8) take 32 consecutive global
//           tiles, so both halves of a straddling line meet in the same L2
//   mode 6: as 5 with every stream line-aligned (row locality of adjacent runs, no halves)
//
// build: hipcc -O3 --offload-arch=gfx950 -o /tmp/mb_scatter tools/mb_scatter.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int WAVES, int ITEMS, int MODE>
__global__ __launch_bounds__(WAVES * 64) void k(const uint4 *__restrict__ in, uint4 *__restrict__ out,
                                                long n, long chunk, int R, int G) {
    constexpr int T = WAVES * 64, TILE = T * ITEMS;
    const int g = blockIdx.x;
    const long begin = (long)g * chunk, end = begin + chunk;
    const long per_part = n / R, per_chunk = per_part / G;
    const int run = TILE / R;
    for (long tb = begin; tb < end; tb += TILE) {
        uint4 r[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) r[j] = in[tb + j * T + threadIdx.x];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const int s = j * T + threadIdx.x;
            long d;
            if (MODE == 0) d = tb + s;
            else if (MODE >= 4) {
                const long t = (tb - begin) / TILE;
                const int p = s / run;
                const long gt = MODE == 4 ? t * G + g : t * G + (long)(g % 8) * (G / 8) + g / 8;
                d = (long)p * per_part + gt * run + s % run;
                if (MODE != 6) d += (p * 13) & 7;
            } else {
                const long t = (tb - begin) / TILE;
                const int p = s / run;
                d = (long)p * per_part + (long)g * per_chunk + t * run + s % run;
                if (MODE == 2) d += (g * 7 + p * 13) & 7;
                if (MODE == 3) d += ((g * 7 + p * 13) & 1) * 4;
            }
            out[d] = r[j];
        }
    }
}

template <int W, int I, int M>
float timeit(const uint4 *in, uint4 *out, long n, int R, int G, int reps) {
    const long chunk = n / G;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int i = 0; i < reps + 2; ++i) {
        CK(hipEventRecord(a));
        k<W, I, M><<<G, W * 64>>>(in, out, n, chunk, R, G);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (i >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
    const long n = 1L << 28;
    uint4 *in, *out;
    CK(hipMalloc(&in, n * 16));
    CK(hipMalloc(&out, (n + 64) * 16));
    CK(hipMemset(in, 1, n * 16));
    CK(hipMemset(out, 0, n * 16));
    const double gb = 32.0 * n / 1e9;
    auto rep = [&](const char *name, int R, int G, float ms) {
        printf("{\"kernel\": \"%s\", \"R\": %d, \"G\": %d, \"ms\": %.4f, \"GBs\": %.1f}\n", name, R, G, ms, gb / ms * 1e3);
    };
    for (int G : {256, 512, 2048}) {
        rep("copy_8x16", 0, G, timeit<8, 16, 0>(in, out, n, 1, G, 10));
        rep("scatter_8x16_aligned128", 1024, G, timeit<8, 16, 1>(in, out, n, 1024, G, 10));
        rep("scatter_8x16_unaligned", 1024, G, timeit<8, 16, 2>(in, out, n, 1024, G, 10));
        rep("scatter_8x16_aligned64", 1024, G, timeit<8, 16, 3>(in, out, n, 1024, G, 10));
        rep("scatter_8x16_unaligned_R512", 512, G, timeit<8, 16, 2>(in, out, n, 512, G, 10));
        rep("scatter_8x16_unaligned_R4096", 4096, G, timeit<8, 16, 2>(in, out, n, 4096, G, 10));
        rep("interleaved_unaligned", 1024, G, timeit<8, 16, 4>(in, out, n, 1024, G, 10));
        rep("interleaved_xcd_unaligned", 1024, G, timeit<8, 16, 5>(in, out, n, 1024, G, 10));
        rep("interleaved_xcd_aligned", 1024, G, timeit<8, 16, 6>(in, out, n, 1024, G, 10));
        rep("interleaved_xcd_unaligned_R4096", 4096, G, timeit<8, 16, 5>(in, out, n, 4096, G, 10));
    }
    return 0;
}
