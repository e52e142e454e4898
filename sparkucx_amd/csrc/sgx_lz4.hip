// Spark shuffle compression on the GPU: every partition stream of a map output framed as
// lz4-java's LZ4BlockOutputStream writes it (spark.shuffle.compress=true, codec lz4, the
// Spark 3.0.1 defaults; SerializerManager.wrapStream per partition in
// ShufflePartitionPairsWriter.open).  Byte-identical to liblz4 1.9.x LZ4_compress_default
// per 32 KiB block + XXH32 (seed 0x9747b28c, masked to 28 bits) + the 21-byte block headers and
// the end mark; see oracle/lz4_oracle.c for the restated algorithm and DESIGN.md §13.
//
// Three kernels:
//   k_lz4_blocks    one WAVE per block: the block's 8192-entry u16 hash table lives in LDS
//                   (16 KiB: 10 blocks per CU; the input is read through L1), and the wave
//                   runs LZ4_compress_default's greedy search 64 iterations at a time
//                   (lz4_compress_wave: the skip schedule fixes the probed positions,
//                   same-hash conflicts inside a batch are resolved by ballots), so a block
//                   costs ~1/64 of the serial chain where it searches, and its match counts,
//                   catch-ups and literal copies are lane-parallel.  The payload goes to a
//                   fixed-size slot; the frame size to sizes[b].
//   k_xxh32_blocks  XXH32 of every block, one lane per block.
//   k_lz4_gather    one workgroup per block writes the header and copies the payload (the
//                   slot, or the stream itself for a RAW block) to the frame's final offset
//                   (offsets scanned on the host from sizes), and writes the partition end marks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sgx_internal.h"

namespace sgx {
namespace {

constexpr int kMinMatch = 4;
constexpr int kLastLiterals = 5;
constexpr int kMfLimit = 12;
constexpr int kHashLog = 13;                       // byU16 table: LZ4_HASHLOG + 1
constexpr int kTable = 1 << kHashLog;              // 8192 u16 entries
constexpr int kMaxBlock = 32768;                   // largest block (lz4-java's 32 KiB blockSize)
constexpr int kLanes = 1;                          // one block per workgroup (one wave):
                                                   // 16 KiB LDS -> 10 workgroups per CU
constexpr int kHeader = 21;
// A/B switch: the search's table candidate loads before the same-hash ballots resolve, a
// lower peer's bytes then come from its probe by lane shuffle (1), or the candidate loads
// after them (0)
#ifndef SGX_LZ4_PEER_SHFL
#define SGX_LZ4_PEER_SHFL 1
#endif
// Diagnostic build only (-DSGX_LZ4_STAMPS, tools/lz4_stamps.py): per-phase s_memtime sums of
// lz4_compress_batch, read through sgx_diag_lz4_stamps.  Never in libsgx.so; the stamps' waits
// (lgkmcnt(0), and vmcnt(0) where a phase is a memory wait) change the run: read the SHARES.
#ifdef SGX_LZ4_STAMPS
__device__ unsigned long long g_lz4_stamps[16];
__device__ __forceinline__ uint64_t lz4_stamp_now() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define LZ4_STAMP(i)                          \
    do {                                      \
        const uint64_t t_ = lz4_stamp_now();  \
        st_acc[i] += t_ - st_last;            \
        st_last = t_;                         \
    } while (0)
#define LZ4_STAMP_VM(i)                                           \
    do {                                                          \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          \
        LZ4_STAMP(i);                                             \
    } while (0)
#else
#define LZ4_STAMP(i) \
    do {             \
    } while (0)
#define LZ4_STAMP_VM(i) \
    do {                \
    } while (0)
#endif
// lz4_compress_batch (several sequences per batch, 1) or lz4_compress_wave (0)
#ifndef SGX_LZ4_BATCH
#define SGX_LZ4_BATCH 1
#endif

// unaligned little-endian 32-bit read from the LDS staging buffer: the two aligned dwords
// around it + one v_alignbyte (instead of four ds_read_u8); the buffer is padded by 8 bytes
__device__ __forceinline__ uint32_t lds32(const uint8_t *p) {
    // pointer arithmetic (no int-to-pointer cast) keeps the LDS address space visible to the
    // compiler: ds_read, not flat loads that would also wait on the pending HBM stores
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *w = (const uint32_t *)(p - sh);
    return __builtin_amdgcn_alignbyte(w[1], w[0], sh);
}
// unaligned little-endian 32-bit read of global bytes p[0..3]: one global_load_dword (gfx950
// serves unaligned dword loads; nothing outside p[0..3] is read)
__device__ __forceinline__ uint32_t g32(const uint8_t *p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
// The compressor's view of its block: bytes [0, n) read as one unaligned little-endian dword
// (u32) or one byte (u8) through L1.  (Staging the whole block in LDS first -- 48 KiB per
// block with the table, 3 blocks per CU instead of 10 -- measured 1.7x slower on C1's Kryo
// stream: DESIGN §13.)
struct GlobalSrc {
    const uint8_t *p;
    __device__ __forceinline__ uint32_t u32(int i) const { return g32(p + i); }
    __device__ __forceinline__ uint32_t u8(int i) const { return p[i]; }
    // bytes [i, i + 4 * N) as N little-endian dwords: one unaligned global_load_dwordxN
    template <int N>
    __device__ __forceinline__ void words(int i, uint32_t (&w)[N]) const { __builtin_memcpy(w, p + i, 4 * N); }
};
__device__ __forceinline__ uint32_t hash4(uint32_t seq) { return (seq * 2654435761u) >> (32 - kHashLog); }
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// XXH32 (seed 0x9747b28c, LZ4BlockOutputStream's) of the LDS bytes [base + sh, base + sh +
// len), base 16 B-aligned, sh < 4: whole stripes from a rolling window of ds_read_b128 (one
// per stripe, realigned with v_alignbyte), four stripes in flight per step.  The buffer is
// readable 16 B past the data.
__device__ uint32_t xxh32_lds_window(const uint8_t *base, int sh, int len, uint32_t seed) {
    const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                   P5 = 374761393u;
    const uint4 *q = (const uint4 *)base;
    const uint32_t s8 = (uint32_t)sh;
    uint32_t h;
    int i = 0;
    if (len >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        const int ns = len >> 4;
        uint4 prev = q[0];
        int k = 0;
        auto step = [&](const uint4 &nx) {
            const uint32_t a0 = __builtin_amdgcn_alignbyte(prev.y, prev.x, s8);
            const uint32_t a1 = __builtin_amdgcn_alignbyte(prev.z, prev.y, s8);
            const uint32_t a2 = __builtin_amdgcn_alignbyte(prev.w, prev.z, s8);
            const uint32_t a3 = __builtin_amdgcn_alignbyte(nx.x, prev.w, s8);
            v1 = rotl(v1 + a0 * P2, 13) * P1;
            v2 = rotl(v2 + a1 * P2, 13) * P1;
            v3 = rotl(v3 + a2 * P2, 13) * P1;
            v4 = rotl(v4 + a3 * P2, 13) * P1;
            prev = nx;
        };
        for (; k + 4 <= ns; k += 4) {
            uint4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = q[k + 1 + u];
#pragma unroll
            for (int u = 0; u < 4; ++u) step(x[u]);
        }
        for (; k < ns; ++k) step(q[k + 1]);
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        i = ns << 4;
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    const uint8_t *p = base + sh;
    for (; i + 4 <= len; i += 4) h = rotl(h + lds32(p + i) * P3, 17) * P4;
    for (; i < len; ++i) h = rotl(h + (uint32_t)p[i] * P5, 11) * P1;
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

// Skip schedule of LZ4_compress_default's search: iteration 0 steps 1, iteration i >= 1
// steps (63 + i) >> 6.  skip_dist(m) = total distance of iterations [0, m): with
// G(x) = sum_{j<=x} floor(j / 64) = 32 q (q - 1) + q (r + 1) (q = x / 64, r = x % 64),
// skip_dist(m) = 1 + G(62 + m) for m >= 1.
__device__ __forceinline__ int skip_dist(int m) {
    const int x = 62 + m, q = x >> 6, r = x & 63;
    return (1 + 32 * q * (q - 1) + q * (r + 1)) & -(int)(m != 0);  // (a mask, not a branch)
}
__device__ __forceinline__ int first_clear(uint64_t m) { return m == ~0ull ? 64 : (int)__builtin_ctzll(~m); }
__device__ __forceinline__ int lane_value(int v, int l) { return __builtin_amdgcn_readlane(v, l); }

// LZ4_compress_default of src[0, n) (n < 65547) into out[0, cap), run by ONE WAVE: returns
// the compressed size in every lane, or -1 if the output would pass `cap`
// (LZ4_compressBound(n) <= cap by construction: a guard against corrupt input, never a path
// of correct runs).  `src` is the block in global memory (read through L1: the search
// touches a few hundred bytes around the cursor at a time), `table` (zeroed:
// LZ4_initStream) the wave's 16 KiB LDS slice -- the only LDS a block needs, so 10 blocks
// are in flight per CU; output bytes go straight to HBM.
//
// Bit-exact with the serial algorithm (oracle/lz4_oracle.c, pinned to liblz4) because it
// executes the same iterations, 64 at a time where the serial code has no data dependence
// it cannot resolve in the wave:
//  * the match search: from a search start the probed positions follow from the skip
//    schedule alone (step 1, then (63 + i) >> 6 at iteration i), so lane k takes iteration
//    it + k: its position (a wave prefix sum of the steps), its hash, the table entry as of
//    the batch start -- overridden by the latest lower lane with the same hash (whose write
//    the serial code would have made first) -- and the 4-byte comparison.  The first lane
//    that matches (or whose next position passes mflimit) ends the search; the table then
//    receives, per hash, the position of the last lane before it, as the serial writes
//    would have left it.
//  * LZ4_count: 64 4-byte comparisons per round, the first differing byte from a ballot.
//  * the backward catch-up: 64 byte comparisons per round.
//  * literal and length-run bytes: lane-parallel stores.
// The wave is latency-bound, so loads whose addresses are known early go out
// together: the catch-up's and LZ4_count's first rounds (the catch-up never moves the match
// end), a _next_match candidate's 4-byte test and its first count round, and the next
// search's first 64 sequences with the _next_match test.  (Loading each search batch's
// successor with the batch measured 2-3% slower: DESIGN §13.)  Only loads move; every table
// access and every decision stays in the serial order.
// LZ4_count's end: the first a' >= a with src[a'] != src[a' + d0], or mlimit.  (d, full) is
// the first round's comparison at a + 4 * lane, issued by the caller.
template <typename Src>
__device__ __forceinline__ int lz4_count_end(const Src &src, int a, int d0, int mlimit, uint32_t d, bool full) {
    const int lane = (int)(threadIdx.x & 63);
    for (;;) {
        const uint64_t dm = __ballot(d != 0);
        if (dm) {
            const int k = (int)__builtin_ctzll(dm);
            return a + 4 * k + ((int)__builtin_ctz((uint32_t)lane_value((int)d, k)) >> 3);
        }
        const int nfull = __popcll(__ballot(full));
        a += 4 * nfull;
        if (nfull < 64) {  // < 4 bytes before matchlimit: byte-wise
            while (a < mlimit && src.u8(a) == src.u8(a + d0)) ++a;
            return a;
        }
        const int al = a + 4 * lane;
        full = al + 4 <= mlimit;
        d = full ? src.u32(al) ^ src.u32(al + d0) : 0u;
    }
}

// A search lane's bytes: s0, s4, s8 = the dwords at pos, pos + 4, pos + 8 and pb = the byte
// at pos - 1 -- the sequence it hashes, plus what a hit needs to settle the common match
// without another round trip: the first LZ4_count comparison (s4 against the candidate's
// second dword), the first catch-up comparison (pb against the byte before the candidate) and
// the next position's sequences (_next_match's ip - 2 and ip, inside bytes [pos + 2, pos + 11)
// when the match ends in that first dword).  Valid lanes have pos + 12 <= n (pos < mflimit).
struct Probe {
    uint32_t s0, s4, s8, pb;
};
template <typename Src>
__device__ __forceinline__ Probe search_probe(const Src &src, int start, int it, int n) {
    const int lane = (int)(threadIdx.x & 63);
    const int pos = min(start + skip_dist(it + lane), n - 12);  // (invalid lanes: any bytes)
    Probe pr;
    if (start >= 4) {  // uniform: bytes [pos - 4, pos + 12) in one load
        uint32_t w[4];
        src.words(pos - 4, w);
        pr = Probe{w[1], w[2], w[3], w[0] >> 24};
    } else {  // the block's first positions
        uint32_t w[3];
        src.words(pos, w);
        pr = Probe{w[0], w[1], w[2], src.u8(max(pos - 1, 0))};
    }
    return pr;
}

template <typename Src>
__device__ __forceinline__ int lz4_compress_wave(const Src &src, int n, uint16_t *table, uint8_t *out, int cap) {
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t below = (1ull << lane) - 1ull;
    int anchor = 0, op = 0;
    if (n >= kMfLimit + 1) {
        const int lim = n - kMfLimit + 1;      // mflimit_plus_one
        const int mlimit = n - kLastLiterals;  // matchlimit
        if (lane == 0) table[hash4(src.u32(0))] = 0;
        int ip = 1;
        Probe pr0 = search_probe(src, ip, 0, n);
        // _next_match's two sequences when the search's match settled inside its probe bytes
        bool have_next = false;
        uint32_t nx_s2 = 0, nx_s0 = 0;
        for (;;) {
            // ---- match search from ip (step 1, search counter 64)
            const int start = ip;
            int it = 0, match = 0;
            bool found = false;
            Probe pr = pr0;
            // the hit lane's bytes (Probe) and its candidate's: dword at match + 4, the byte
            // before match (cbok: read; a candidate below 4 leaves the catch-up to the loop)
            uint32_t hs0 = 0, hs4 = 0, hs8 = 0, hpb = 0, hc4 = 0, hcb = 0;
            bool hcbok = false;
            for (;;) {
                const int pos = start + skip_dist(it + lane);
                const int nxt = pos + max((it + lane + 63) >> 6, 1);  // the position after this one
                const bool valid = nxt <= lim;
                // past the first batch a search tends to run on: the next batch's sequences
                // load with this one's
                Probe prn{0, 0, 0, 0};
                if (it > 0) prn = search_probe(src, start, it + 64, n);
                const uint32_t seq = pr.s0;
                const uint32_t h = hash4(seq);
#if SGX_LZ4_PEER_SHFL
                const int tcand = table[h];
                // the table candidate's bytes [cand - 4, cand + 8) load as soon as the entry
                // arrives (tcand < pos <= n - 12 for a valid lane), before the ballots below
                // resolve: a lane with a lower peer takes the peer's probe bytes instead
                const int tc = min(tcand, n - 12), tb0 = max(tc - 4, 0), tsh = tc - tb0;
                uint32_t cw[3];
                src.words(tb0, cw);
                // lanes probing the same hash: those whose ballot bits agree with ours on all
                // hash bits (diff: the lanes that differ on some bit)
                uint32_t diff_lo = 0, diff_hi = 0;
#pragma unroll
                for (int bt = 0; bt < kHashLog; ++bt) {
                    const uint32_t sx = (uint32_t)((int32_t)(h << (31 - bt)) >> 31);  // 0 or ~0
                    const uint64_t m = __ballot(sx != 0);
                    diff_lo |= (uint32_t)m ^ sx;
                    diff_hi |= (uint32_t)(m >> 32) ^ sx;
                }
                const uint64_t peers = ~(((uint64_t)diff_hi << 32) | diff_lo);
                const uint64_t lower = peers & below;
                // the latest lower lane with our hash: its position is the entry the serial code
                // would read, and its probe holds that position's bytes
                // (a valid lane's candidate is in the block: a lower peer of a valid lane is valid)
                const int peer = lower ? 63 - (int)__builtin_clzll(lower) : lane;
                const uint32_t ps0 = (uint32_t)__shfl((int)pr.s0, peer), ps4 = (uint32_t)__shfl((int)pr.s4, peer),
                               ppb = (uint32_t)__shfl((int)pr.pb, peer);
                const int cand = lower ? start + skip_dist(it + peer) : tcand;
                const uint32_t c0 = lower ? ps0 : tsh == 4 ? cw[1] : __builtin_amdgcn_alignbyte(cw[1], cw[0], (uint32_t)tsh);
                const uint32_t c4 = lower ? ps4 : tsh == 4 ? cw[2] : __builtin_amdgcn_alignbyte(cw[2], cw[1], (uint32_t)tsh);
                const uint32_t cbyte = lower ? ppb : cw[0] >> 24;
                const bool cbok = lower || tsh == 4;  // the byte before the candidate was read
#else
                int cand = table[h];
                uint32_t diff_lo = 0, diff_hi = 0;
#pragma unroll
                for (int bt = 0; bt < kHashLog; ++bt) {
                    const uint32_t sx = (uint32_t)((int32_t)(h << (31 - bt)) >> 31);  // 0 or ~0
                    const uint64_t m = __ballot(sx != 0);
                    diff_lo |= (uint32_t)m ^ sx;
                    diff_hi |= (uint32_t)(m >> 32) ^ sx;
                }
                const uint64_t peers = ~(((uint64_t)diff_hi << 32) | diff_lo);
                const uint64_t lower = peers & below;
                if (lower) cand = start + skip_dist(it + 63 - (int)__builtin_clzll(lower));
                const int tc = min(cand, n - 12), tb0 = max(tc - 4, 0), tsh = tc - tb0;
                uint32_t cw[3];
                src.words(tb0, cw);
                const uint32_t c0 = tsh == 4 ? cw[1] : __builtin_amdgcn_alignbyte(cw[1], cw[0], (uint32_t)tsh);
                const uint32_t c4 = tsh == 4 ? cw[2] : __builtin_amdgcn_alignbyte(cw[2], cw[1], (uint32_t)tsh);
                const uint32_t cbyte = cw[0] >> 24;
                const bool cbok = tsh == 4;
#endif
                const bool hit = c0 == seq && valid;
                const uint64_t vm = __ballot(valid), hm = __ballot(hit);
                const int kinv = first_clear(vm);
                const int khit = hm ? (int)__builtin_ctzll(hm) : 64;
                // iterations [0, kend) of this batch ran: each writes table[h] = pos
                const int kend = khit < kinv ? khit + 1 : kinv;
                const uint64_t ran = kend >= 64 ? ~0ull : (1ull << kend) - 1ull;
                if ((ran >> lane) & 1ull) {
                    if (((peers & ran) >> lane) == 1ull) table[h] = (uint16_t)pos;  // last writer of h
                }
                if (khit < kinv) {
                    found = true;
                    ip = start + skip_dist(it + khit);
                    match = lane_value(cand, khit);
                    hs0 = (uint32_t)lane_value((int)pr.s0, khit);
                    hs4 = (uint32_t)lane_value((int)pr.s4, khit);
                    hs8 = (uint32_t)lane_value((int)pr.s8, khit);
                    hpb = (uint32_t)lane_value((int)pr.pb, khit);
                    hc4 = (uint32_t)lane_value((int)c4, khit);
                    hcb = (uint32_t)lane_value((int)cbyte, khit);
                    hcbok = (__ballot(cbok) >> khit) & 1ull;
                    break;
                }
                if (kinv < 64) break;  // next position past mflimit: no match in this block
                pr = it == 0 ? search_probe(src, start, 64, n) : prn;
                it += 64;
            }
            if (!found) break;
            // ---- catch up backwards, and LZ4_count from ip + 4.  The common match settles from
            // the probe bytes: no catch-up (the bytes before ip and match differ, or ip is the
            // anchor) and an end inside the first counted dword; then _next_match's sequences
            // at the end come from the same bytes.  Otherwise the catch-up and the count's
            // first round load together (the bytes the catch-up adds before ip match, so the
            // match end does not move).
            int aend;
            {
                const int d0 = match - ip, a0 = ip + kMinMatch;
                const bool no_back = ip - 1 < anchor || match < 1 || (hcbok && hpb != hcb);
                const bool short_end = a0 + 4 <= mlimit && hs4 != hc4;
                if (no_back && short_end) {
                    aend = a0 + ((int)__builtin_ctz(hs4 ^ hc4) >> 3);
                    const uint32_t k = (uint32_t)(aend - ip);  // 4..7: ip + 2 .. ip + 10 are probe bytes
                    nx_s0 = k == 4 ? hs4 : __builtin_amdgcn_alignbyte(hs8, hs4, k - 4);
                    nx_s2 = k - 2 < 4 ? __builtin_amdgcn_alignbyte(hs4, hs0, k - 2)
                                      : __builtin_amdgcn_alignbyte(hs8, hs4, k - 6);
                    have_next = true;
                } else {
                    const int al = a0 + 4 * lane;
                    const bool full = al + 4 <= mlimit;
                    const uint32_t d = full ? src.u32(al) ^ src.u32(al + d0) : 0u;
                    if (!no_back) {
                        for (;;) {
                            const int a = ip - 1 - lane, b = match - 1 - lane;
                            const bool eq = (src.u8(max(a, 0)) == src.u8(max(b, 0))) && a >= anchor && b >= 0;  // (loads unconditional)
                            const int back = first_clear(__ballot(eq));
                            ip -= back;
                            match -= back;
                            if (back < 64) break;
                        }
                    }
                    aend = lz4_count_end(src, a0, d0, mlimit, d, full);
                }
            }
            // ---- literals
            const int lit = ip - anchor;
            if (op + 1 + lit / 255 + 1 + lit + 2 + 1 > cap) return -1;
            // the output only grows: once token + literals + offset reach n the block is RAW
            // (lz4-java keeps a block whose compressed size is >= its length uncompressed), and
            // its payload is never read (k_lz4_gather copies RAW blocks from the stream)
            if (op + 1 + lit + 2 >= n) return n;
            int token = op++;
            uint32_t tk;
            if (lit >= 15) {
                const int nrun = (lit - 15) / 255;  // 255-bytes, then the remainder
                for (int j = lane; j <= nrun; j += 64) out[op + j] = j < nrun ? (uint8_t)255 : (uint8_t)((lit - 15) % 255);
                op += nrun + 1;
                tk = 15u << 4;
            } else {
                tk = (uint32_t)lit << 4;
            }
            for (int j = lane; j < lit; j += 64) out[op + j] = (uint8_t)src.u8(anchor + j);
            op += lit;
            for (;;) {  // _next_match
                const uint32_t off = (uint32_t)(ip - match);
                if (lane == 0) {
                    out[op] = (uint8_t)off;
                    out[op + 1] = (uint8_t)(off >> 8);
                }
                op += 2;
                // LZ4_count from ip + 4 / match + 4 up to matchlimit (for the search's match:
                // counted above with the catch-up)
                uint32_t mc = (uint32_t)(aend - (ip + kMinMatch));
                if (op + (int)(mc / 255) + 1 + 3 > cap) return -1;  // run bytes + the next token, offset
                ip = aend;
                if (mc >= 15) {
                    tk += 15;
                    mc -= 15;
                    const int nrun = (int)(mc / 255);
                    for (int j = lane; j <= nrun; j += 64) out[op + j] = j < nrun ? (uint8_t)255 : (uint8_t)(mc % 255);
                    op += nrun + 1;
                } else {
                    tk += mc;
                }
                if (lane == 0) out[token] = (uint8_t)tk;
                anchor = ip;
                if (ip >= lim) goto last_literals;
                // the next search's first sequences load with this test's (unused on a hit)
                pr0 = search_probe(src, ip + 1, 0, n);
                uint32_t s2, s0;
                if (have_next) {
                    s2 = nx_s2;
                    s0 = nx_s0;
                    have_next = false;
                } else {
                    s2 = src.u32(ip - 2);
                    s0 = src.u32(ip);
                }
                if (lane == 0) table[hash4(s2)] = (uint16_t)(ip - 2);
                __builtin_amdgcn_wave_barrier();  // the write above, then the read below
                const uint32_t h = hash4(s0);
                const int m2 = table[h];
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) table[h] = (uint16_t)ip;
                // a candidate's LZ4_count round loads with its test (m2 < ip: in bounds)
                const int d0 = m2 - ip, al = ip + kMinMatch + 4 * lane;
                const bool full = al + 4 <= mlimit;
                const uint32_t d = full ? src.u32(al) ^ src.u32(al + d0) : 0u;
                if (src.u32(m2) != s0) break;
                match = m2;
                token = op++;
                tk = 0;
                aend = lz4_count_end(src, ip + kMinMatch, d0, mlimit, d, full);  // no catch-up: ip is the anchor
            }
            ++ip;
        }
    }
last_literals:
    {
        const int last = n - anchor;
        if (op + 1 + last / 255 + 1 + last > cap) return -1;
        const int fin = op + 1 + (last >= 15 ? (last - 15) / 255 + 1 : 0) + last;
        if (fin >= n) return fin;  // RAW: nothing to write (see the literal run above)
        if (last >= 15) {
            const int nrun = (last - 15) / 255;
            if (lane == 0) out[op] = 15u << 4;
            for (int j = lane; j <= nrun; j += 64) out[op + 1 + j] = j < nrun ? (uint8_t)255 : (uint8_t)((last - 15) % 255);
            op += nrun + 2;
        } else {
            if (lane == 0) out[op] = (uint8_t)(last << 4);
            ++op;
        }
        for (int j = lane; j < last; j += 64) out[op + j] = (uint8_t)src.u8(anchor + j);
        op += last;
    }
    return op;
}

// LZ4_compress_default of src[0, n) again, with several sequences per batch (round 4,
// SGX_LZ4_BATCH).  A batch whose lanes probe consecutive positions (the first 64 iterations
// of a search: step 1) keeps going after a match that ends inside it: the match's end ip,
// `_next_match`'s ip - 2 and ip, and the next search's positions ip + 1, ip + 2, ... are all
// lanes of the same batch, already loaded and hashed.  The serial table state a lane must see
// follows from a mask W of the batch's lanes whose positions the serial code has inserted so
// far (every insertion is at a higher position than the last, so "the latest inserted lane
// below me with my hash" is the entry it would read; no such lane: the batch-start entry);
// the table receives W's last writer per hash when the batch ends.  A candidate that is
// another lane comes with that lane's probe bytes (shuffle / readlane); one from the table
// with the bytes the lane loaded at the batch start.  So a C1 Kryo block's short sequences
// cost a few wave instructions each instead of a batch plus one to three memory round trips.
// Matches that end past the batch, and batches of a search's later iterations (steps > 1),
// go the way of lz4_compress_wave.  Same iterations, same table, same bytes.
template <typename Src>
__device__ __forceinline__ int lz4_compress_batch(const Src &src, int n, uint16_t *table, uint8_t *out, int cap) {
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t below = (1ull << lane) - 1ull;
    int anchor = 0, op = 0;
#ifdef SGX_LZ4_STAMPS
    uint64_t st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t st_last = lz4_stamp_now();
#endif
    if (n >= kMfLimit + 1) {
        const int lim = n - kMfLimit + 1;      // mflimit_plus_one
        const int mlimit = n - kLastLiterals;  // matchlimit
        if (lane == 0) table[hash4(src.u32(0))] = 0;
        int start = 1, it = 0;  // the running search: its first position, iterations done
        Probe pr0 = search_probe(src, start, 0, n);
        bool have_next = false;  // _next_match's sequences from a settled match's probe bytes
        uint32_t nx_s2 = 0, nx_s0 = 0;
        for (;;) {  // ---- one batch: iterations [it, it + 64) of the search from `start`
            const int pos = start + skip_dist(it + lane);
            const int nxt = pos + max((it + lane + 63) >> 6, 1);  // the position after this one
            const bool valid = nxt <= lim;
            LZ4_STAMP_VM(0);  // 0: the batch's probe bytes (loaded at the last batch's end or earlier)
            const Probe pr = pr0;
            Probe prn{0, 0, 0, 0};
            if (it > 0) prn = search_probe(src, start, it + 64, n);  // a search past its first batch runs on
            const uint32_t h = hash4(pr.s0);
            const int tcand = table[h];
            // the batch-start entry's bytes [tcand - 4, tcand + 8) (tcand < pos <= n - 12 for a valid lane)
            const int tc = min(tcand, n - 12), tb0 = max(tc - 4, 0), tsh = tc - tb0;
            uint32_t cw[3];
            src.words(tb0, cw);
            LZ4_STAMP(1);  // 1: hash, table read
            uint32_t diff_lo = 0, diff_hi = 0;
#pragma unroll
            for (int bt = 0; bt < kHashLog; ++bt) {
                const uint32_t sx = (uint32_t)((int32_t)(h << (31 - bt)) >> 31);  // 0 or ~0
                const uint64_t m = __ballot(sx != 0);
                diff_lo |= (uint32_t)m ^ sx;
                diff_hi |= (uint32_t)(m >> 32) ^ sx;
            }
            const uint64_t peers = ~(((uint64_t)diff_hi << 32) | diff_lo);  // lanes with our hash
            LZ4_STAMP(2);  // 2: the 13 same-hash ballots
            const uint32_t tc0 = tsh == 4 ? cw[1] : __builtin_amdgcn_alignbyte(cw[1], cw[0], (uint32_t)tsh);
            const uint32_t tc4 = tsh == 4 ? cw[2] : __builtin_amdgcn_alignbyte(cw[2], cw[1], (uint32_t)tsh);
            LZ4_STAMP_VM(3);  // 3: the table candidates' bytes
            const bool consec = it == 0;  // lane j probes start + j
            uint64_t W = 0;               // lanes whose positions the serial code inserted so far
            int lo = 0;                   // the running search's first lane
            bool ended = false;           // no more matches: last literals
            bool fresh = false;           // pr0 already holds the next batch's probe
            int next_start = 0, next_it = 0;
            for (;;) {  // ---- one search inside the batch: lanes [lo, 64)
                const uint64_t run = ~0ull << lo;
                const uint64_t elig = peers & below & (W | run);
                const int pj = elig ? 63 - (int)__builtin_clzll(elig) : lane;
                const uint32_t ps0 = (uint32_t)__shfl((int)pr.s0, pj), ps4 = (uint32_t)__shfl((int)pr.s4, pj),
                               ppb = (uint32_t)__shfl((int)pr.pb, pj);
                const int cand = elig ? start + skip_dist(it + pj) : tcand;
                const uint32_t c0 = elig ? ps0 : tc0, c4 = elig ? ps4 : tc4, cbyte = elig ? ppb : cw[0] >> 24;
                const bool cbok = elig || tsh == 4;  // the byte before the candidate was read
                const bool hit = ((run >> lane) & 1ull) && valid && c0 == pr.s0;
                const uint64_t hm = __ballot(hit), inv = ~__ballot(valid) & run;
                const int kinv = inv ? (int)__builtin_ctzll(inv) : 64;
                const int khit = hm ? (int)__builtin_ctzll(hm) : 64;
                const int kend = khit < kinv ? khit + 1 : kinv;  // iterations [lo, kend) ran
                LZ4_STAMP(4);  // 4: a search in the batch (candidates, shuffles, hit ballots)
                W |= (kend >= 64 ? ~0ull : (1ull << kend) - 1ull) & run;
                if (khit >= kinv) {
                    if (kinv < 64) {  // the next position passes mflimit: no match in this block
                        ended = true;
                    } else {          // the search runs on in the next batch
                        next_start = lo == 0 ? start : start + lo;  // (lo > 0: a consecutive batch)
                        next_it = lo == 0 ? it + 64 : 64 - lo;
                    }
                    break;
                }
                // ---- a match at lane khit
                int ip = lane_value(pos, khit);
                int match = lane_value(cand, khit);
                const uint32_t hs0 = (uint32_t)lane_value((int)pr.s0, khit), hs4 = (uint32_t)lane_value((int)pr.s4, khit),
                               hs8 = (uint32_t)lane_value((int)pr.s8, khit), hpb = (uint32_t)lane_value((int)pr.pb, khit),
                               hc4 = (uint32_t)lane_value((int)c4, khit), hcb = (uint32_t)lane_value((int)cbyte, khit);
                const bool hcbok = (__ballot(cbok) >> khit) & 1ull;
                int aend;
                {  // catch-up and LZ4_count from ip + 4, settled from the probe bytes when possible
                    const int d0 = match - ip, a0 = ip + kMinMatch;
                    const bool no_back = ip - 1 < anchor || match < 1 || (hcbok && hpb != hcb);
                    const bool short_end = a0 + 4 <= mlimit && hs4 != hc4;
                    if (no_back && short_end) {
                        aend = a0 + ((int)__builtin_ctz(hs4 ^ hc4) >> 3);
                        const uint32_t k = (uint32_t)(aend - ip);  // 4..7: ip + 2 .. ip + 10 are probe bytes
                        nx_s0 = k == 4 ? hs4 : __builtin_amdgcn_alignbyte(hs8, hs4, k - 4);
                        nx_s2 = k - 2 < 4 ? __builtin_amdgcn_alignbyte(hs4, hs0, k - 2)
                                          : __builtin_amdgcn_alignbyte(hs8, hs4, k - 6);
                        have_next = true;
                    } else {
                        have_next = false;
                        const int al = a0 + 4 * lane;
                        const bool full = al + 4 <= mlimit;
                        const uint32_t d = full ? src.u32(al) ^ src.u32(al + d0) : 0u;
                        if (!no_back) {
                            for (;;) {
                                const int a = ip - 1 - lane, b = match - 1 - lane;
                                const bool eq = (src.u8(max(a, 0)) == src.u8(max(b, 0))) && a >= anchor && b >= 0;
                                const int back = first_clear(__ballot(eq));
                                ip -= back;
                                match -= back;
                                if (back < 64) break;
                            }
                        }
                        aend = lz4_count_end(src, a0, d0, mlimit, d, full);
                    }
                }
                LZ4_STAMP_VM(5);  // 5: the hit's catch-up and count (fast: readlanes; slow: loads)
                // ---- literals
                const int lit = ip - anchor;
                if (op + 1 + lit / 255 + 1 + lit + 2 + 1 > cap) return -1;
                if (op + 1 + lit + 2 >= n) return n;  // RAW (see lz4_compress_wave)
                int token = op++;
                uint32_t tk;
                if (lit >= 15) {
                    const int nrun = (lit - 15) / 255;
                    for (int j = lane; j <= nrun; j += 64) out[op + j] = j < nrun ? (uint8_t)255 : (uint8_t)((lit - 15) % 255);
                    op += nrun + 1;
                    tk = 15u << 4;
                } else {
                    tk = (uint32_t)lit << 4;
                }
                if (consec && anchor >= start - 1) {
                    // the literals [anchor, ip) are this batch's positions (and lane 0's byte
                    // before them): their bytes come from the probes, not from memory
                    const int sl = anchor + lane - start;
                    const uint32_t v0 = (uint32_t)__shfl((int)pr.s0, max(sl, 0)), vb = (uint32_t)__shfl((int)pr.pb, 0);
                    if (lane < lit) out[op + lane] = (uint8_t)(sl < 0 ? vb : v0);
                } else {
                    for (int j = lane; j < lit; j += 64) out[op + j] = (uint8_t)src.u8(anchor + j);
                }
                op += lit;
                bool cont = false;  // the next search continues inside this batch from lane lo
                for (;;) {          // ---- _next_match
                    const uint32_t off = (uint32_t)(ip - match);
                    if (lane == 0) {
                        out[op] = (uint8_t)off;
                        out[op + 1] = (uint8_t)(off >> 8);
                    }
                    op += 2;
                    uint32_t mc = (uint32_t)(aend - (ip + kMinMatch));
                    if (op + (int)(mc / 255) + 1 + 3 > cap) return -1;
                    ip = aend;
                    if (mc >= 15) {
                        tk += 15;
                        mc -= 15;
                        const int nrun = (int)(mc / 255);
                        for (int j = lane; j <= nrun; j += 64) out[op + j] = j < nrun ? (uint8_t)255 : (uint8_t)(mc % 255);
                        op += nrun + 1;
                    } else {
                        tk += mc;
                    }
                    if (lane == 0) out[token] = (uint8_t)tk;
                    LZ4_STAMP(6);  // 6: the sequence's output bytes (stores issued)
                    anchor = ip;
                    if (ip >= lim) {
                        ended = true;
                        break;
                    }
                    const int a0 = ip - start;  // ip's lane in a consecutive batch
                    if (consec && a0 < 64) {
                        // insert ip - 2; the entry for ip's hash (the latest inserted lane below
                        // a0 with it, else a0's batch-start entry); insert ip
                        have_next = false;
                        W |= 1ull << (a0 - 2);
                        const uint64_t e = peers & below & W;
                        const uint64_t ea = ((uint64_t)(uint32_t)lane_value((int)(uint32_t)(e >> 32), a0) << 32) |
                                            (uint32_t)lane_value((int)(uint32_t)e, a0);
                        int m2;
                        uint32_t m0, m4;
                        if (ea) {
                            const int pl = 63 - (int)__builtin_clzll(ea);
                            m2 = start + pl;
                            m0 = (uint32_t)lane_value((int)pr.s0, pl);
                            m4 = (uint32_t)lane_value((int)pr.s4, pl);
                        } else {
                            m2 = lane_value(tcand, a0);
                            m0 = (uint32_t)lane_value((int)tc0, a0);
                            m4 = (uint32_t)lane_value((int)tc4, a0);
                        }
                        W |= 1ull << a0;
                        const uint32_t s0 = (uint32_t)lane_value((int)pr.s0, a0), s4 = (uint32_t)lane_value((int)pr.s4, a0);
                        LZ4_STAMP(7);  // 7: _next_match's test inside the batch
                        if (m0 != s0) {  // no match at ip: the next search starts at ip + 1
                            lo = a0 + 1;
                            cont = lo < 64;
                            if (!cont) {
                                next_start = ip + 1;
                                next_it = 0;
                            }
                            break;
                        }
                        match = m2;
                        token = op++;
                        tk = 0;
                        const int a = ip + kMinMatch;
                        if (a + 4 <= mlimit && s4 != m4) {
                            aend = a + ((int)__builtin_ctz(s4 ^ m4) >> 3);
                        } else {
                            const int d0 = m2 - ip, al = a + 4 * lane;
                            const bool full = al + 4 <= mlimit;
                            const uint32_t d = full ? src.u32(al) ^ src.u32(al + d0) : 0u;
                            aend = lz4_count_end(src, a, d0, mlimit, d, full);
                        }
                        continue;
                    }
                    // past the batch: its insertions go to the table first, then the serial test
                    if ((W >> lane) & 1ull) {
                        if (((peers & W) >> lane) == 1ull) table[h] = (uint16_t)pos;
                    }
                    W = 0;
                    __builtin_amdgcn_wave_barrier();
                    pr0 = search_probe(src, ip + 1, 0, n);  // the next search's first batch
                    fresh = true;
                    uint32_t s2, s0;
                    if (have_next) {
                        s2 = nx_s2;
                        s0 = nx_s0;
                        have_next = false;
                    } else {
                        s2 = src.u32(ip - 2);
                        s0 = src.u32(ip);
                    }
                    if (lane == 0) table[hash4(s2)] = (uint16_t)(ip - 2);
                    __builtin_amdgcn_wave_barrier();
                    const uint32_t hh = hash4(s0);
                    const int m2 = table[hh];
                    __builtin_amdgcn_wave_barrier();
                    if (lane == 0) table[hh] = (uint16_t)ip;
                    const int d0 = m2 - ip, al = ip + kMinMatch + 4 * lane;
                    const bool full = al + 4 <= mlimit;
                    const uint32_t d = full ? src.u32(al) ^ src.u32(al + d0) : 0u;
                    LZ4_STAMP_VM(8);  // 8: _next_match's test past the batch (table, loads)
                    if (src.u32(m2) != s0) {
                        next_start = ip + 1;
                        next_it = 0;
                        break;
                    }
                    match = m2;
                    token = op++;
                    tk = 0;
                    aend = lz4_count_end(src, ip + kMinMatch, d0, mlimit, d, full);
                }
                if (ended || !cont) break;
            }
            LZ4_STAMP(9);  // 9: (the batch's last search / exits)
            // ---- the batch's insertions: per hash, its last inserted lane
            if ((W >> lane) & 1ull) {
                if (((peers & W) >> lane) == 1ull) table[h] = (uint16_t)pos;
            }
            __builtin_amdgcn_wave_barrier();
            if (ended) break;
            if (!fresh) pr0 = (it > 0 && next_start == start && next_it == it + 64) ? prn : search_probe(src, next_start, next_it, n);
            start = next_start;
            it = next_it;
        }
    }
#ifdef SGX_LZ4_STAMPS
    if (lane == 0) {
        for (int i = 0; i < 10; ++i) atomicAdd(&g_lz4_stamps[i], (unsigned long long)st_acc[i]);
        atomicAdd(&g_lz4_stamps[15], 1ull);
    }
#endif
    {  // last literals
        const int last = n - anchor;
        if (op + 1 + last / 255 + 1 + last > cap) return -1;
        const int fin = op + 1 + (last >= 15 ? (last - 15) / 255 + 1 : 0) + last;
        if (fin >= n) return fin;  // RAW: nothing to write
        if (last >= 15) {
            const int nrun = (last - 15) / 255;
            if (lane == 0) out[op] = 15u << 4;
            for (int j = lane; j <= nrun; j += 64) out[op + 1 + j] = j < nrun ? (uint8_t)255 : (uint8_t)((last - 15) % 255);
            op += nrun + 2;
        } else {
            if (lane == 0) out[op] = (uint8_t)(last << 4);
            ++op;
        }
        for (int j = lane; j < last; j += 64) out[op + j] = (uint8_t)src.u8(anchor + j);
        op += last;
    }
    return op;
}

#ifdef SGX_LZ4_STAMPS
}  // namespace
}  // namespace sgx
extern "C" int sgx_diag_lz4_stamps(unsigned long long *out16, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(sgx::g_lz4_stamps), 16 * 8) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(sgx::g_lz4_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
namespace sgx {
namespace {
#endif
__device__ __forceinline__ void st32le(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

__device__ __forceinline__ void put_header(uint8_t *h, uint8_t token, uint32_t clen, uint32_t olen,
                                           uint32_t check) {
    h[0] = 'L'; h[1] = 'Z'; h[2] = '4'; h[3] = 'B'; h[4] = 'l'; h[5] = 'o'; h[6] = 'c'; h[7] = 'k';
    h[8] = token;
    st32le(h + 9, clen);
    st32le(h + 13, olen);
    st32le(h + 17, check);
}

// blocks[b] = {src byte offset, length}; one wave per block.
// Every global access is checked against stream_len / the slot: a block outside the stream
// or an output past its slot sets err[0] (1 = bad block, 2 = output overflow) and records
// {block, offset, length} in err[1..3] instead of touching memory.
__global__ __launch_bounds__(64) void k_lz4_blocks(const uint8_t *__restrict__ stream, int64_t stream_len,
                                                   const int64_t *__restrict__ blocks, int64_t nblocks,
                                                   int level, uint8_t *__restrict__ slots,
                                                   int64_t slot_bytes, int32_t *__restrict__ sizes,
                                                   int64_t *__restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint16_t s_tab[kTable];
    static_assert(kLanes == 1, "one block per workgroup");
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    if (b >= nblocks) return;  // uniform across the workgroup
    const int64_t boff = blocks[2 * b], blen = blocks[2 * b + 1];
    if (boff < 0 || blen < 0 || blen > kMaxBlock || boff + blen > stream_len) {
        if (lane == 0) {
            err[1] = b;
            err[2] = boff;
            err[3] = blen;
            atomicOr((unsigned long long *)err, 1ull);
        }
        return;
    }
    for (int i = lane; i < kTable / 8; i += 64) ((uint4 *)s_tab)[i] = make_uint4(0u, 0u, 0u, 0u);
    const int n = (int)blen;
    uint8_t *slot = slots + b * slot_bytes;
    __syncthreads();
    const GlobalSrc src{stream + boff};
#if SGX_LZ4_BATCH
    const int sc = lz4_compress_batch(src, n, s_tab, slot + kHeader, (int)(slot_bytes - kHeader));
#else
    const int sc = lz4_compress_wave(src, n, s_tab, slot + kHeader, (int)(slot_bytes - kHeader));
#endif
    if (sc < 0) {
        if (lane == 0) {
            err[1] = b;
            err[2] = boff;
            err[3] = n;
            atomicOr((unsigned long long *)err, 2ull);
        }
        return;
    }
    // a block that did not shrink is RAW: k_lz4_gather copies it from the stream
    if (lane == 0) sizes[b] = kHeader + (sc >= n ? n : sc);
}

// XXH32 (LZ4BlockOutputStream's seed, masked to 28 bits) of every block: one LANE per block,
// so the serial fold (four accumulators over 16 B stripes) runs for 64 blocks per wave
// instruction.  Reads: aligned dwords, realigned per lane with v_alignbyte.
__global__ __launch_bounds__(256) void k_xxh32_blocks(const uint8_t *__restrict__ stream,
                                                      const int64_t *__restrict__ blocks, int64_t nblocks,
                                                      uint32_t *__restrict__ checks) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= nblocks) return;
    const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                   P5 = 374761393u, seed = 0x9747b28cu;
    const uint8_t *p = stream + blocks[2 * b];
    const int len = (int)blocks[2 * b + 1];
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *w = (const uint32_t *)(p - sh);  // aligned dwords; the fold reads whole stripes
    uint32_t h;
    int i = 0;
    if (len >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        const int ns = len >> 4;
        for (int k = 0; k < ns; ++k) {
            // stripe k = bytes [sh + 16k, sh + 16k + 16) of w: dwords 4k .. 4k+3, and 4k+4
            // only when sh > 0 (it then holds the stripe's last bytes: nothing past them is read)
            const uint32_t w0 = w[4 * k], w1 = w[4 * k + 1], w2 = w[4 * k + 2], w3 = w[4 * k + 3];
            const uint32_t w4 = w[4 * k + (sh ? 4 : 3)];
            v1 = rotl(v1 + __builtin_amdgcn_alignbyte(w1, w0, sh) * P2, 13) * P1;
            v2 = rotl(v2 + __builtin_amdgcn_alignbyte(w2, w1, sh) * P2, 13) * P1;
            v3 = rotl(v3 + __builtin_amdgcn_alignbyte(w3, w2, sh) * P2, 13) * P1;
            v4 = rotl(v4 + __builtin_amdgcn_alignbyte(w4, w3, sh) * P2, 13) * P1;
        }
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        i = ns << 4;
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    for (; i + 4 <= len; i += 4) h = rotl(h + g32(p + i) * P3, 17) * P4;
    for (; i < len; ++i) h = rotl(h + (uint32_t)p[i] * P5, 11) * P1;
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    checks[b] = h & 0x0FFFFFFFu;
}

// frame b: its header (method from the size: a RAW block keeps its length) and payload --
// the slot's compressed bytes or, RAW, the block straight from the stream -- to
// dst + frame_off[b]; workgroups past nblocks write end marks at end_off[r] (partitions with
// bytes only).
__global__ __launch_bounds__(256) void k_lz4_gather(const uint8_t *__restrict__ stream,
                                                    const int64_t *__restrict__ blocks,
                                                    const uint8_t *__restrict__ slots, int64_t slot_bytes,
                                                    const int32_t *__restrict__ sizes,
                                                    const uint32_t *__restrict__ checks,
                                                    const int64_t *__restrict__ frame_off, int64_t nblocks,
                                                    const int64_t *__restrict__ end_off, int64_t nends,
                                                    int level, uint8_t *__restrict__ dst) {
    const int64_t b = blockIdx.x;
    if (b < nblocks) {
        const int n = (int)blocks[2 * b + 1];
        const int c = sizes[b] - kHeader;
        const bool raw = c == n;  // compressed payloads are strictly shorter
        const uint8_t *s = raw ? stream + blocks[2 * b] : slots + b * slot_bytes + kHeader;
        uint8_t *d = dst + frame_off[b];
        if (threadIdx.x == 0) put_header(d, (uint8_t)((raw ? 0x10 : 0x20) | level), (uint32_t)c, (uint32_t)n, checks[b]);
        for (int i = threadIdx.x; i < c; i += 256) d[kHeader + i] = s[i];
        return;
    }
    const int64_t e = (b - nblocks) * 256 + threadIdx.x;
    if (e < nends) put_header(dst + end_off[e], (uint8_t)(0x10 | level), 0u, 0u, 0u);
}


// ---------------------------------------------------------------------------------------
// reduce side: LZ4BlockInputStream over fetched bytes (any number of partition streams back
// to back, each ended by its end mark)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t g32le(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// One thread walks the frame headers (each header gives the next one's position: a serial
// pointer chase, ~1 HBM latency per frame) and records desc[k] = {frame offset, output
// offset} for the first desc_cap frames.  info = {frames, output bytes, error code, error
// position}.
__global__ void k_lz4_walk(const uint8_t *__restrict__ in, int64_t nbytes, int64_t *__restrict__ desc,
                           int64_t desc_cap, int64_t *__restrict__ info) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t p = 0, k = 0, out = 0, err = 0;
    while (p < nbytes) {
        if (p + kHeader > nbytes) { err = 1; break; }
        const uint8_t *h = in + p;
        if (h[0] != 'L' || h[1] != 'Z' || h[2] != '4' || h[3] != 'B' || h[4] != 'l' || h[5] != 'o' ||
            h[6] != 'c' || h[7] != 'k') { err = 2; break; }
        const uint32_t tok = h[8], clen = g32le(h + 9), olen = g32le(h + 13), check = g32le(h + 17);
        const uint32_t method = tok & 0xF0u;
        if (method != 0x10u && method != 0x20u) { err = 3; break; }
        if (olen == 0) {  // end mark
            if (clen != 0 || check != 0) { err = 4; break; }
            p += kHeader;
            continue;
        }
        if (olen > (uint32_t)kMaxBlock || clen == 0 || (method == 0x10u && clen != olen) ||
            (method == 0x20u && clen > olen + (olen >> 8) + 32) || p + kHeader + (int64_t)clen > nbytes) {
            err = 5;  // (a compressed block past LZ4_compressBound cannot come from a compressor)
            break;
        }
        if (k < desc_cap) {  // past the capacity the walk only counts (caller re-walks)
            desc[2 * k + 0] = p;
            desc[2 * k + 1] = out;
        }
        ++k;
        out += olen;
        p += kHeader + clen;
    }
    info[0] = k;
    info[1] = out;
    info[2] = err;
    info[3] = p;
}

// Per-stream walk, for callers that know where every LZ4 stream of the buffer starts (the
// reader does: each fetched block is one partition stream): one thread per stream, so the
// pointer chase is as long as the longest stream's frame count instead of the sum of all.
// soff[nstreams + 1]: stream byte offsets.  Pass 0 (WRITE false) writes cnt[s] = {frames,
// output bytes}; pass 1 (WRITE true) reads cnt[s] = {first frame index, output offset} (the
// host's exclusive scan of pass 0) and writes desc[k] = {frame offset, output offset}.
// Malformed input: atomicMin of (byte position << 8 | code) into *err (codes of k_lz4_walk).
template <bool WRITE>
__global__ __launch_bounds__(256) void k_lz4_walk_streams(const uint8_t *__restrict__ in,
                                                          const int64_t *__restrict__ soff, int64_t nstreams,
                                                          int64_t *__restrict__ cnt, int64_t *__restrict__ desc,
                                                          unsigned long long *__restrict__ err) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= nstreams) return;
    const int64_t end = soff[s + 1];
    int64_t p = soff[s], k = 0, out = 0, code = 0;
    if (WRITE) {
        k = cnt[2 * s];
        out = cnt[2 * s + 1];
    }
    while (p < end) {
        if (p + kHeader > end) { code = 1; break; }
        const uint8_t *h = in + p;
        if (g32le(h) != 0x42345a4cu || g32le(h + 4) != 0x6b636f6cu) { code = 2; break; }  // "LZ4B" "lock"
        const uint32_t tok = h[8], clen = g32le(h + 9), olen = g32le(h + 13), check = g32le(h + 17);
        const uint32_t method = tok & 0xF0u;
        if (method != 0x10u && method != 0x20u) { code = 3; break; }
        if (olen == 0) {
            if (clen != 0 || check != 0) { code = 4; break; }
            p += kHeader;
            continue;
        }
        if (olen > (uint32_t)kMaxBlock || clen == 0 || (method == 0x10u && clen != olen) ||
            (method == 0x20u && clen > olen + (olen >> 8) + 32) || p + kHeader + (int64_t)clen > end) {
            code = 5;
            break;
        }
        if (WRITE) {
            desc[2 * k + 0] = p;
            desc[2 * k + 1] = out;
        }
        ++k;
        out += olen;
        p += kHeader + clen;
    }
    if (code) {
        atomicMin(err, ((unsigned long long)p << 8) | (unsigned long long)code);
        return;
    }
    if (!WRITE) {
        cnt[2 * s] = k;
        cnt[2 * s + 1] = out;
    }
}

// LZ4_DECOMPRESS_INPLACE_BUFFER_SIZE(kMaxBlock): a compressed block placed at the end of a
// buffer this long decodes in place -- the output never overtakes the unread input (liblz4's
// in-place margin, (size >> 8) + 32).  One buffer instead of two keeps 4 workgroups per CU.
constexpr int kInplace = kMaxBlock + (kMaxBlock >> 8) + 32;

// One frame per workgroup (one wave).  The payload is staged in LDS by aligned dword loads
// (keeping its misalignment): a RAW block is the output as staged; a compressed one is staged
// at the end of the buffer and decoded in place by the 64 lanes in lockstep -- every lane parses
// the same token bytes (uniform control flow, broadcast LDS reads) and copies its share of each
// sequence's literals and match bytes.  A match byte i reads out[op - off + i mod off]: bytes
// before op, already written even when the match overlaps itself (off < length), so the copy
// is lane-parallel with LZ4_decompress_safe's result.  A literal step reads input at or after
// the bytes it writes (in-place margin), and a wave's LDS operations complete in issue order.
// Bounds are checked as LZ4_decompress_safe does (corrupt input can at worst garble its own
// block, then fails the checksum); XXH32 runs over the LDS output (lane 0), then the wave
// writes the block out with dword stores.  Errors: atomicOr into *err.
__global__ __launch_bounds__(64) void k_lz4_decode(const uint8_t *__restrict__ in,
                                                   const int64_t *__restrict__ desc, int64_t nframes,
                                                   uint8_t *__restrict__ out, uint32_t *__restrict__ err,
                                                   int skip_raw) {
    __shared__ __attribute__((aligned(16))) uint8_t s_buf[kInplace + 48];
    __shared__ int s_bad;
    const int64_t f = blockIdx.x;
    if (f >= nframes) return;
    const int lane = (int)threadIdx.x;
    const uint8_t *h = in + desc[2 * f + 0];  // header fields validated by the walk
    const uint32_t tok = h[8], clen = g32le(h + 9), olen = g32le(h + 13), check = g32le(h + 17);
    const bool raw = (tok & 0xF0u) == 0x10u;
    if (raw && skip_raw) return;  // k_lz4_raw_lanes
    const uint8_t *g = h + kHeader;
    const int sh = (int)((uintptr_t)g & 3u);
    const int n = (int)clen;
    // input position in LDS: RAW at sh (it is the output), compressed at the in-place end
    // (rounded up to the source's byte phase)
    int x = sh;
    if (!raw) {
        const int x0 = (int)olen + ((int)olen >> 8) + 32 - n;
        x = x0 + ((sh - x0) & 3);
    }
    {
        const uint32_t *gw = (const uint32_t *)(g - sh);
        const int full = (sh + n) >> 2;
        uint32_t *sw = (uint32_t *)(s_buf + x - sh);
        for (int i = lane; i < full; i += 64) sw[i] = gw[i];
        if (lane < ((sh + n) & 3)) s_buf[x - sh + full * 4 + lane] = g[full * 4 - sh + lane];
    }
    if (lane == 0) s_bad = 0;
    __syncthreads();
    int bad = 0;
    int ob = sh;  // output position in LDS
    if (!raw) {
        ob = 0;
        const uint8_t *src = s_buf + x;
        uint8_t *o = s_buf;
        uint32_t ip = 0, op = 0;
        for (;;) {  // wave-uniform: every lane reads the same bytes
            if (ip >= clen) { bad = 1; break; }
            const uint32_t t = src[ip++];
            uint32_t lit = t >> 4;
            if (lit == 15) {
                uint32_t b;
                do {
                    if (ip >= clen) { bad = 1; break; }
                    b = src[ip++];
                    lit += b;
                } while (b == 255);
                if (bad) break;
            }
            if (ip + lit > clen || op + lit > olen) { bad = 1; break; }
            for (uint32_t i = lane; i < lit; i += 64) o[op + i] = src[ip + i];
            ip += lit;
            op += lit;
            if (ip == clen) break;  // the last sequence has literals only
            if (ip + 2 > clen) { bad = 1; break; }
            const uint32_t off = (uint32_t)src[ip] | ((uint32_t)src[ip + 1] << 8);
            ip += 2;
            uint32_t ml = (t & 15u) + kMinMatch;
            if ((t & 15u) == 15u) {
                uint32_t b;
                do {
                    if (ip >= clen) { bad = 1; break; }
                    b = src[ip++];
                    ml += b;
                } while (b == 255);
                if (bad) break;
            }
            if (off == 0 || off > op || op + ml > olen) { bad = 1; break; }
            const uint32_t base = op - off;
            if (off >= 64 || off >= ml) {
                // every byte read was written before this loop (off >= ml) or in an earlier
                // step of it (off >= 64)
                for (uint32_t i = lane; i < ml; i += 64) o[op + i] = o[base + i];
            } else {
                const uint32_t stp = 64u % off;
                uint32_t m = (uint32_t)lane % off;
                for (uint32_t i = lane; i < ml; i += 64) {
                    o[op + i] = o[base + m];
                    m += stp;
                    m = m >= off ? m - off : m;
                }
            }
            op += ml;
        }
        if (!bad && op != olen) bad = 1;
    }
    __syncthreads();
    if (lane == 0) {
        if (!bad && (xxh32_lds_window(s_buf, ob, (int)olen, 0x9747b28cu) & 0x0FFFFFFFu) != check) bad = 2;
        s_bad = bad;
    }
    __syncthreads();
    if (s_bad) {
        if (lane == 0) atomicOr(err, (uint32_t)s_bad);
        return;
    }
    // write out: head bytes to a dword boundary, dword stores, tail bytes
    const uint8_t *ls = s_buf + ob;
    uint8_t *d = out + desc[2 * f + 1];
    const int on = (int)olen;
    const int head = min(on, (int)((4u - ((uintptr_t)d & 3u)) & 3u));
    if (lane < head) d[lane] = ls[lane];
    const int nw = (on - head) >> 2;
    uint32_t *dw = (uint32_t *)(d + head);
    for (int i = lane; i < nw; i += 64) dw[i] = lds32(ls + head + 4 * i);
    const int tail0 = head + 4 * nw;
    if (lane < on - tail0) d[tail0 + lane] = ls[tail0 + lane];
}

// Compressed frames, one LANE per frame (when there are enough frames to fill the chip with
// lanes: kLaneDecodeMinFrames).  The sequence stream is a serial chain per frame, so one frame
// per lane makes every wave instruction advance 64 frames, where the wave-per-frame decoder
// above spends ~30 VALU + ~70 SALU instructions of the whole wave per sequence at one wave
// per SIMD (its 33 KB of LDS per frame).  The lane decodes straight into the destination
// (bytes of its own frame only; every write is checked against the frame's output length
// first, as LZ4_decompress_safe does), reading literals from the fetched payload and match
// sources from its own earlier output -- a same-thread store -> load through global memory,
// which the hardware keeps in order.  Copies go 8 bytes at a time: a chunk's 8 loads are
// one 8-byte load before its store (one memory round trip per chunk), which is also what
// makes the self-overlapping copy exact: chunk [i, i + 8) of a match at offset >= 8 reads
// bytes written before it; an offset below 8 writes the match's first p bytes (p the first
// multiple of the offset >= 8) from registers, then copies chunks from p bytes back.  Then
// XXH32 of the frame's output (re-read, L2-resident) against the header.  RAW frames go to
// k_lz4_raw_lanes.  Errors: atomicOr into *err.
// (A variant that kept each lane's last 256 output bytes in an LDS ring, so that no load
// follows the lane's own stores, measured slower: 17.3 / 30.2 ms against 11.9 / 24.6 ms,
// profiles/r02_lz4_decode_lanes_ab.jsonl.)
constexpr int64_t kLaneDecodeMinFrames = 32768;  // below: k_lz4_decode does the compressed frames
constexpr int64_t kRawLaneMinFrames = 2048;      // below: k_lz4_decode does the RAW frames too

__device__ uint32_t xxh32_global(const uint8_t *p, int len, uint32_t seed) {
    const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                   P5 = 374761393u;
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *w = (const uint32_t *)(p - sh);  // aligned dwords, realigned with v_alignbyte
    uint32_t h;
    int i = 0;
    if (len >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        const int ns = len >> 4;
        for (int k = 0; k < ns; ++k) {
            const uint32_t w0 = w[4 * k], w1 = w[4 * k + 1], w2 = w[4 * k + 2], w3 = w[4 * k + 3];
            const uint32_t w4 = w[4 * k + (sh ? 4 : 3)];  // only when it holds stripe bytes
            v1 = rotl(v1 + __builtin_amdgcn_alignbyte(w1, w0, sh) * P2, 13) * P1;
            v2 = rotl(v2 + __builtin_amdgcn_alignbyte(w2, w1, sh) * P2, 13) * P1;
            v3 = rotl(v3 + __builtin_amdgcn_alignbyte(w3, w2, sh) * P2, 13) * P1;
            v4 = rotl(v4 + __builtin_amdgcn_alignbyte(w4, w3, sh) * P2, 13) * P1;
        }
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        i = ns << 4;
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    for (; i + 4 <= len; i += 4) h = rotl(h + g32(p + i) * P3, 17) * P4;
    for (; i < len; ++i) h = rotl(h + (uint32_t)p[i] * P5, 11) * P1;
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

// byte i (< 16) of a 16-byte little-endian register value
__device__ __forceinline__ uint32_t byte_at(const uint4 &x, uint32_t i) {
    const uint32_t w = i < 8u ? (i < 4u ? x.x : x.y) : (i < 12u ? x.z : x.w);
    return (w >> (8u * (i & 3u))) & 0xFFu;
}

// ceil(len / 16) 16-byte chunks (unaligned dwordx4): d[len, ceil16(len)) receives bytes that
// later writes replace before anything reads them; s is >= 16 bytes before d (or elsewhere)
__device__ __forceinline__ void copy16_over(uint8_t *d, const uint8_t *s, uint32_t len) {
    for (uint32_t i = 0; i < len; i += 16) {
        uint4 v;
        __builtin_memcpy(&v, s + i, 16);
        __builtin_memcpy(d + i, &v, 16);
    }
}

// d and s may overlap (a match copy): each 8-byte chunk is read before it is written (one
// unaligned global_load_dwordx2 / global_store_dwordx2 per chunk)
__device__ __forceinline__ void copy8_chunks(uint8_t *d, const uint8_t *s, uint32_t len) {
    uint32_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t v;
        __builtin_memcpy(&v, s + i, 8);
        __builtin_memcpy(d + i, &v, 8);
    }
    if (i + 4 <= len) {
        const uint32_t w = g32(s + i);
        __builtin_memcpy(d + i, &w, 4);
        i += 4;
    }
    for (; i < len; ++i) d[i] = s[i];
}
__global__ __launch_bounds__(64) void k_lz4_decode_lanes(const uint8_t *__restrict__ in,
                                                         const int64_t *__restrict__ desc, int64_t nframes,
                                                         uint8_t *__restrict__ out, uint32_t *__restrict__ err) {
    const int64_t f = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (f >= nframes) return;
    const uint8_t *h = in + desc[2 * f + 0];
    if ((h[8] & 0xF0u) == 0x10u) return;
    const uint32_t clen = g32le(h + 9), olen = g32le(h + 13), check = g32le(h + 17);
    const uint8_t *src = h + kHeader;
    uint8_t *o = out + desc[2 * f + 1];
    uint32_t ip = 0, op = 0, bad = 0;
    for (;;) {
        uint32_t t = 0, off = 0;
        bool fast = false;
        if (ip + 16 <= clen && op + 16 <= olen) {
            // a short sequence head in one 16-byte load: token, literals, offset.  The literals
            // go out as one 16-byte store; its bytes past the literals land in [op + lit,
            // op + 16), inside this frame, where this sequence's match or later sequences write
            // before anything reads them (a match reads only bytes before its own position)
            uint4 x;
            __builtin_memcpy(&x, src + ip, 16);
            t = x.x & 0xFFu;
            const uint32_t lit = t >> 4;
            if (lit <= 13u) {
                fast = true;
                const uint4 y = make_uint4(__builtin_amdgcn_alignbyte(x.y, x.x, 1),
                                           __builtin_amdgcn_alignbyte(x.z, x.y, 1),
                                           __builtin_amdgcn_alignbyte(x.w, x.z, 1), x.w >> 8);
                __builtin_memcpy(o + op, &y, 16);
                off = byte_at(x, 1u + lit) | (byte_at(x, 2u + lit) << 8);
                ip += 3u + lit;
                op += lit;
            }
        }
        if (!fast) {
            if (ip >= clen) { bad = 1; break; }
            t = src[ip++];
            uint32_t lit = t >> 4;
            if (lit == 15) { uint32_t b; do { if (ip >= clen) { bad = 1; break; } b = src[ip++]; lit += b; } while (b == 255); if (bad) break; }
            if (ip + lit > clen || op + lit > olen) { bad = 1; break; }
            const uint32_t lr = (lit + 15u) & ~15u;
            if (ip + lr <= clen && op + lr <= olen) copy16_over(o + op, src + ip, lit);
            else copy8_chunks(o + op, src + ip, lit);
            ip += lit; op += lit;
            if (ip == clen) break;
            if (ip + 2 > clen) { bad = 1; break; }
            off = (uint32_t)src[ip] | ((uint32_t)src[ip + 1] << 8);
            ip += 2;
        }
        uint32_t ml = (t & 15u) + kMinMatch;
        if ((t & 15u) == 15u) { uint32_t b; do { if (ip >= clen) { bad = 1; break; } b = src[ip++]; ml += b; } while (b == 255); if (bad) break; }
        if (off == 0 || off > op || op + ml > olen) { bad = 1; break; }
        if (off >= 16 && op + ((ml + 15u) & ~15u) <= olen) copy16_over(o + op, o + op - off, ml);
        else if (off >= 8) copy8_chunks(o + op, o + op - off, ml);
        else {
            // the match repeats with period off, so also with period p = the first multiple of
            // off >= 8: bytes [0, p) from the period held in registers, the rest as chunks
            // from p bytes back
            const uint32_t p = off * ((8u + off - 1u) / off);
            const uint32_t head = ml < p ? ml : p;
            uint8_t pat[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) pat[k] = (uint32_t)k < off ? o[op - off + k] : (uint8_t)0;
            uint32_t m = 0;
            for (uint32_t i = 0; i < head; ++i) {
                uint8_t v = pat[0];
#pragma unroll
                for (int k = 1; k < 8; ++k) v = (uint32_t)k == m ? pat[k] : v;
                o[op + i] = v;
                m = m + 1 == off ? 0u : m + 1;
            }
            if (ml > p) copy8_chunks(o + op + p, o + op, ml - p);
        }
        op += ml;
    }
    if (!bad && op != olen) bad = 1;
    if (!bad && (xxh32_global(o, (int)olen, 0x9747b28cu) & 0x0FFFFFFFu) != check) bad = 2;
    if (bad) atomicOr(err, bad);
}

// RAW frames of a lane-decoded stream, one per LANE: the payload is copied in 16-byte chunks
// (one unaligned global_load_dwordx4 / global_store_dwordx4 each) and every chunk is also the
// next XXH32 stripe, so the checksum reads nothing twice.  (k_lz4_decode's wave-per-frame
// RAW path stages 32 KB in LDS -- 4 frames per CU -- and runs XXH32 on one lane.)
__global__ __launch_bounds__(64) void k_lz4_raw_lanes(const uint8_t *__restrict__ in,
                                                      const int64_t *__restrict__ desc, int64_t nframes,
                                                      uint8_t *__restrict__ out, uint32_t *__restrict__ err) {
    const int64_t f = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (f >= nframes) return;
    const uint8_t *h = in + desc[2 * f + 0];
    if ((h[8] & 0xF0u) != 0x10u) return;  // compressed: k_lz4_decode_lanes
    const uint32_t olen = g32le(h + 13), check = g32le(h + 17);  // RAW: clen == olen (the walk)
    const uint8_t *src = h + kHeader;
    uint8_t *o = out + desc[2 * f + 1];
    const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u,
                   P5 = 374761393u, seed = 0x9747b28cu;
    const uint32_t ns = olen >> 4;
    uint32_t hs;
    if (ns) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
#pragma unroll 4
        for (uint32_t k = 0; k < ns; ++k) {
            uint4 x;
            __builtin_memcpy(&x, src + 16 * k, 16);
            __builtin_memcpy(o + 16 * k, &x, 16);
            v1 = rotl(v1 + x.x * P2, 13) * P1;
            v2 = rotl(v2 + x.y * P2, 13) * P1;
            v3 = rotl(v3 + x.z * P2, 13) * P1;
            v4 = rotl(v4 + x.w * P2, 13) * P1;
        }
        hs = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    } else {
        hs = seed + P5;
    }
    hs += olen;
    uint32_t i = ns << 4;
    for (; i + 4 <= olen; i += 4) {
        const uint32_t wd = g32(src + i);
        __builtin_memcpy(o + i, &wd, 4);
        hs = rotl(hs + wd * P3, 17) * P4;
    }
    for (; i < olen; ++i) {
        const uint8_t b = src[i];
        o[i] = b;
        hs = rotl(hs + (uint32_t)b * P5, 11) * P1;
    }
    hs ^= hs >> 15; hs *= P2; hs ^= hs >> 13; hs *= P3; hs ^= hs >> 16;
    if ((hs & 0x0FFFFFFFu) != check) atomicOr(err, 2u);
}
}  // namespace

int lz4_lanes_per_workgroup() { return kLanes; }
int lz4_max_block() { return kMaxBlock; }

hipError_t launch_lz4_blocks(const uint8_t *stream, int64_t stream_len, const int64_t *blocks, int64_t nblocks,
                             int level, uint8_t *slots, int64_t slot_bytes, int32_t *sizes, uint32_t *checks,
                             int64_t *err, hipStream_t stream_) {
    if (nblocks <= 0) return hipSuccess;
    (void)level;
    int64_t grid = (nblocks + kLanes - 1) / kLanes;
    hipLaunchKernelGGL(k_lz4_blocks, dim3((unsigned)grid), dim3(64), 0, stream_, stream, stream_len, blocks,
                       nblocks, level, slots, slot_bytes, sizes, err);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_xxh32_blocks, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, stream_, stream, blocks,
                       nblocks, checks);
    return hipGetLastError();
}

hipError_t launch_lz4_gather(const uint8_t *stream, const int64_t *blocks, const uint8_t *slots, int64_t slot_bytes,
                             const int32_t *sizes, const uint32_t *checks, const int64_t *frame_off, int64_t nblocks,
                             const int64_t *end_off, int64_t nends, int level, uint8_t *dst, hipStream_t stream_) {
    const int64_t grid = nblocks + (nends + 255) / 256;
    if (grid <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_lz4_gather, dim3((unsigned)grid), dim3(256), 0, stream_, stream, blocks, slots, slot_bytes,
                       sizes, checks, frame_off, nblocks, end_off, nends, level, dst);
    return hipGetLastError();
}

}  // namespace sgx

namespace sgx {
hipError_t launch_lz4_walk(const uint8_t *in, int64_t nbytes, int64_t *desc, int64_t desc_cap, int64_t *info,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_lz4_walk, dim3(1), dim3(64), 0, s, in, nbytes, desc, desc_cap, info);
    return hipGetLastError();
}

hipError_t launch_lz4_walk_streams(const uint8_t *in, const int64_t *soff, int64_t nstreams, int64_t *cnt,
                                   int64_t *desc, unsigned long long *err, bool write, hipStream_t s) {
    if (nstreams <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nstreams + 255) / 256));
    if (write)
        hipLaunchKernelGGL(k_lz4_walk_streams<true>, grid, dim3(256), 0, s, in, soff, nstreams, cnt, desc, err);
    else
        hipLaunchKernelGGL(k_lz4_walk_streams<false>, grid, dim3(256), 0, s, in, soff, nstreams, cnt, desc, err);
    return hipGetLastError();
}

hipError_t launch_lz4_decode(const uint8_t *in, const int64_t *desc, int64_t nframes, uint8_t *out,
                             uint32_t *err, bool force_lanes, hipStream_t s) {
    if (nframes <= 0) return hipSuccess;
    // lane-per-frame decoding of the compressed frames pays off only with enough frames to
    // fill the chip with lanes: measured (tools/prof_lz4.py, bench.py --compress) 4,056
    // frames 10.2 (waves) vs 11.9 ms (lanes), ~32K frames 4.31 vs 4.32 ms, 127K frames 58.3
    // vs 24.6 ms
    const bool lanes = force_lanes || nframes >= kLaneDecodeMinFrames;
    // RAW frames one per lane from fewer frames on (tools/prof_lz4.py: 1,889 frames 0.44 vs
    // 0.49 ms, 7,651 frames 0.57 vs 1.37 ms; one lane's serial copy costs ~0.4 ms, so not for
    // a handful of frames)
    const bool raw_lanes = force_lanes || nframes >= kRawLaneMinFrames;
    hipError_t e = hipSuccess;
    if (raw_lanes) {
        hipLaunchKernelGGL(k_lz4_raw_lanes, dim3((unsigned)((nframes + 63) / 64)), dim3(64), 0, s, in, desc, nframes,
                           out, err);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (!lanes) {
        hipLaunchKernelGGL(k_lz4_decode, dim3((unsigned)nframes), dim3(64), 0, s, in, desc, nframes, out, err,
                           raw_lanes ? 1 : 0);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_lz4_decode_lanes, dim3((unsigned)((nframes + 63) / 64)), dim3(64), 0, s, in, desc, nframes,
                       out, err);
    return hipGetLastError();
}
}  // namespace sgx
