// Spark shuffle compression on the GPU: every partition stream of a map output framed as
// lz4-java's LZ4BlockOutputStream writes it (spark.shuffle.compress=true, codec lz4, the
// Spark 3.0.1 defaults; SerializerManager.wrapStream per partition in
// ShufflePartitionPairsWriter.open).  Byte-identical to liblz4 1.9.x LZ4_compress_default
// per 32 KiB block + XXH32 (seed 0x9747b28c, masked to 28 bits) + the 21-byte block headers and
// the end mark; see oracle/lz4_oracle.c for the restated algorithm and DESIGN.md §12.
//
// Two kernels:
//   k_lz4_blocks  one LANE per block: the block's input bytes and its 8192-entry u16 hash
//                 table live in LDS (48 KiB per lane), so the greedy match search -- a serial
//                 dependence chain by construction of LZ4_compress_default's skip acceleration
//                 and table updates -- runs at LDS latency.  The frame (header + payload) goes
//                 to a fixed-size slot; its size to sizes[b].
//   k_lz4_gather  one workgroup per block copies the slot to the frame's final offset
//                 (offsets scanned on the host from sizes), and writes the partition end marks.
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
constexpr int kMaxBlock = 32768;                   // LDS staging limit per lane
constexpr int kLanes = 1;                          // one block per workgroup (one wave, one busy lane):
                                                   // 48 KiB LDS -> 3 workgroups per CU on separate
                                                   // SIMDs, so the serial lanes never share a wave
constexpr int kHeader = 21;

// unaligned little-endian 32-bit read from the LDS staging buffer: the two aligned dwords
// around it + one v_alignbyte (instead of four ds_read_u8); the buffer is padded by 8 bytes
__device__ __forceinline__ uint32_t lds32(const uint8_t *p) {
    // pointer arithmetic (no int-to-pointer cast) keeps the LDS address space visible to the
    // compiler: ds_read, not flat loads that would also wait on the pending HBM stores
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *w = (const uint32_t *)(p - sh);
    return __builtin_amdgcn_alignbyte(w[1], w[0], sh);
}
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

// LZ4_compress_default of src[0, n) (n < 65547) into out[0, cap); returns the compressed
// size, or -1 if the output would pass `cap` (LZ4_compressBound(n) <= cap by construction,
// so this is a guard against corrupt input, never a path of correct runs).
// `src` and `table` are this lane's LDS slices; output bytes go straight to HBM.
// `table` must be zeroed (LZ4_initStream).
__device__ int lz4_compress_lane(const uint8_t *src, int n, uint16_t *table, uint8_t *out, int cap) {
    const uint8_t *ip = src, *anchor = src, *iend = src + n;
    const uint8_t *mflimit_plus_one = iend - kMfLimit + 1;
    const uint8_t *matchlimit = iend - kLastLiterals;
    uint8_t *op = out;
    uint8_t *const oend = out + cap;
    if (n >= kMfLimit + 1) {
        table[hash4(lds32(ip))] = 0;
        ip++;
        uint32_t fwd_h = hash4(lds32(ip));
        for (;;) {
            const uint8_t *match;
            uint8_t *token;
            bool found = false;
            {
                const uint8_t *fwd = ip;
                int step = 1, search = 1 << 6;
                for (;;) {
                    uint32_t h = fwd_h;
                    uint32_t cur = (uint32_t)(fwd - src);
                    uint32_t midx = table[h];
                    ip = fwd;
                    fwd += step;
                    step = search++ >> 6;
                    if (fwd > mflimit_plus_one) break;
                    match = src + midx;
                    fwd_h = hash4(lds32(fwd));
                    table[h] = (uint16_t)cur;
                    if (lds32(match) == lds32(ip)) { found = true; break; }
                }
            }
            if (!found) break;
            while (ip > anchor && match > src && ip[-1] == match[-1]) { ip--; match--; }
            {
                unsigned lit = (unsigned)(ip - anchor);
                // token + literal length + literals + offset + 1 match-length byte at most
                if (op + 1 + lit / 255 + 1 + lit + 2 + 1 > oend) return -1;
                token = op++;
                uint8_t tk;
                if (lit >= 15) {
                    int len = (int)lit - 15;
                    tk = 15 << 4;
                    for (; len >= 255; len -= 255) *op++ = 255;
                    *op++ = (uint8_t)len;
                } else {
                    tk = (uint8_t)(lit << 4);
                }
                for (unsigned i = 0; i < lit; ++i) op[i] = anchor[i];
                op += lit;
                for (;;) {  // _next_match
                    uint32_t off = (uint32_t)(ip - match);
                    op[0] = (uint8_t)off;
                    op[1] = (uint8_t)(off >> 8);
                    op += 2;
                    const uint8_t *a = ip + kMinMatch, *b = match + kMinMatch;
                    // LZ4_count: 4 bytes per step (first differing byte = ctz of the xor)
                    for (;;) {
                        if (a + 4 > matchlimit) {
                            while (a < matchlimit && *a == *b) { a++; b++; }
                            break;
                        }
                        const uint32_t d = lds32(a) ^ lds32(b);
                        if (d) { a += __builtin_ctz(d) >> 3; break; }
                        a += 4;
                        b += 4;
                    }
                    unsigned mc = (unsigned)(a - (ip + kMinMatch));
                    if (op + mc / 255 + 1 + 3 > oend) return -1;  // run bytes + the next token, offset
                    ip = a;
                    if (mc >= 15) {
                        tk += 15;
                        mc -= 15;
                        for (; mc >= 255; mc -= 255) *op++ = 255;
                        *op++ = (uint8_t)mc;
                    } else {
                        tk += (uint8_t)mc;
                    }
                    *token = tk;
                    anchor = ip;
                    if (ip >= mflimit_plus_one) goto last_literals;
                    table[hash4(lds32(ip - 2))] = (uint16_t)(ip - 2 - src);
                    uint32_t h = hash4(lds32(ip));
                    uint32_t cur = (uint32_t)(ip - src);
                    match = src + table[h];
                    table[h] = (uint16_t)cur;
                    if (lds32(match) != lds32(ip)) break;
                    token = op++;
                    tk = 0;
                }
            }
            fwd_h = hash4(lds32(++ip));
        }
    }
last_literals:
    {
        int last = (int)(iend - anchor);
        if (op + 1 + last / 255 + 1 + last > oend) return -1;
        if (last >= 15) {
            int acc = last - 15;
            *op++ = 15 << 4;
            for (; acc >= 255; acc -= 255) *op++ = 255;
            *op++ = (uint8_t)acc;
        } else {
            *op++ = (uint8_t)(last << 4);
        }
        for (int i = 0; i < last; ++i) op[i] = anchor[i];
        op += last;
    }
    return (int)(op - out);
}

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

// blocks[b] = {src byte offset, length}; one lane per block, kLanes lanes per workgroup.
// Every global access is checked against stream_len / the slot: a block outside the stream
// or an output past its slot sets err[0] (1 = bad block, 2 = output overflow) and records
// {block, offset, length} in err[1..3] instead of touching memory.
__global__ __launch_bounds__(64) void k_lz4_blocks(const uint8_t *__restrict__ stream, int64_t stream_len,
                                                   const int64_t *__restrict__ blocks, int64_t nblocks,
                                                   int level, uint8_t *__restrict__ slots,
                                                   int64_t slot_bytes, int32_t *__restrict__ sizes,
                                                   int64_t *__restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint8_t s_in[kLanes][kMaxBlock + 16];
    __shared__ uint16_t s_tab[kLanes][kTable];
    const int lane = threadIdx.x;
    const int64_t b = (int64_t)blockIdx.x * kLanes;
    // stage this workgroup's blocks cooperatively (all 64 threads, 4 B per thread-step)
    for (int l = 0; l < kLanes; ++l) {
        int64_t bb = (int64_t)blockIdx.x * kLanes + l;
        if (bb >= nblocks) break;
        // aligned dword copy that keeps the source's misalignment (sh bytes) in LDS; the
        // last dword is read byte-wise so nothing past the stream's end is touched
        const int64_t boff = blocks[2 * bb], blen = blocks[2 * bb + 1];
        if (boff < 0 || blen < 0 || blen > kMaxBlock || boff + blen > stream_len) {
            if (threadIdx.x == 0) {
                err[1] = bb;
                err[2] = boff;
                err[3] = blen;
                atomicOr((unsigned long long *)err, 1ull);
            }
            return;  // uniform: the whole workgroup leaves before any barrier
        }
        const uint8_t *g = stream + boff;
        const int n = (int)blen;
        const int sh = (int)((uintptr_t)g & 3u);
        const uint32_t *gw = (const uint32_t *)(g - sh);
        const int full = (sh + n) >> 2;
        uint32_t *sw = (uint32_t *)s_in[l];
#pragma unroll 8
        for (int i = threadIdx.x; i < full; i += 64) sw[i] = gw[i];
        // signed index: threadIdx.x is unsigned, and full * 4 - sh < 0 for a block of
        // n < 4 - sh bytes (a 1-byte tail block at an odd offset reads g[-1..0])
        const int t = (int)threadIdx.x;
        if (t < ((sh + n) & 3)) s_in[l][full * 4 + t] = g[full * 4 - sh + t];
    }
    for (int i = threadIdx.x; i < kLanes * kTable / 2; i += 64) ((uint32_t *)s_tab)[i] = 0u;
    __syncthreads();
    static_assert(kLanes == 1, "the tail below assumes one block per workgroup");
    __shared__ int s_c;
    if (b >= nblocks) return;  // uniform across the workgroup
    const int n = (int)blocks[2 * b + 1];
    const uint8_t *src = s_in[0] + ((uintptr_t)(stream + blocks[2 * b]) & 3u);
    uint8_t *slot = slots + b * slot_bytes;
    if (lane == 0) s_c = lz4_compress_lane(src, n, s_tab[0], slot + kHeader, (int)(slot_bytes - kHeader));
    __syncthreads();
    if (s_c < 0) {
        if (lane == 0) {
            err[1] = b;
            err[2] = blocks[2 * b];
            err[3] = n;
            atomicOr((unsigned long long *)err, 2ull);
        }
        return;
    }
    const bool raw = s_c >= n;  // the compressed block did not shrink: RAW, copied by the wave
    const int c = raw ? n : s_c;
    if (raw)
        for (int i = lane; i < n; i += 64) slot[kHeader + i] = src[i];
    if (lane != 0) return;
    uint32_t check = xxh32_lds_window(s_in[0], (int)(src - s_in[0]), n, 0x9747b28cu) & 0x0FFFFFFFu;
    put_header(slot, (uint8_t)((raw ? 0x10 : 0x20) | level), (uint32_t)c, (uint32_t)n, check);
    sizes[b] = kHeader + c;
}

// frame b: copy sizes[b] bytes of slot b to dst + frame_off[b]; workgroups past nblocks write
// end marks at end_off[r] (partitions with bytes only).
__global__ __launch_bounds__(256) void k_lz4_gather(const uint8_t *__restrict__ slots, int64_t slot_bytes,
                                                    const int32_t *__restrict__ sizes,
                                                    const int64_t *__restrict__ frame_off, int64_t nblocks,
                                                    const int64_t *__restrict__ end_off, int64_t nends,
                                                    int level, uint8_t *__restrict__ dst) {
    const int64_t b = blockIdx.x;
    if (b < nblocks) {
        const uint8_t *s = slots + b * slot_bytes;
        uint8_t *d = dst + frame_off[b];
        const int n = sizes[b];
        for (int i = threadIdx.x; i < n; i += 256) d[i] = s[i];
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
                                                   uint8_t *__restrict__ out, uint32_t *__restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint8_t s_buf[kInplace + 48];
    __shared__ int s_bad;
    const int64_t f = blockIdx.x;
    if (f >= nframes) return;
    const int lane = (int)threadIdx.x;
    const uint8_t *h = in + desc[2 * f + 0];  // header fields validated by the walk
    const uint32_t tok = h[8], clen = g32le(h + 9), olen = g32le(h + 13), check = g32le(h + 17);
    const bool raw = (tok & 0xF0u) == 0x10u;
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
}  // namespace

int lz4_lanes_per_workgroup() { return kLanes; }
int lz4_max_block() { return kMaxBlock; }

hipError_t launch_lz4_blocks(const uint8_t *stream, int64_t stream_len, const int64_t *blocks, int64_t nblocks,
                             int level, uint8_t *slots, int64_t slot_bytes, int32_t *sizes, int64_t *err,
                             hipStream_t stream_) {
    if (nblocks <= 0) return hipSuccess;
    int64_t grid = (nblocks + kLanes - 1) / kLanes;
    hipLaunchKernelGGL(k_lz4_blocks, dim3((unsigned)grid), dim3(64), 0, stream_, stream, stream_len, blocks,
                       nblocks, level, slots, slot_bytes, sizes, err);
    return hipGetLastError();
}

hipError_t launch_lz4_gather(const uint8_t *slots, int64_t slot_bytes, const int32_t *sizes,
                             const int64_t *frame_off, int64_t nblocks, const int64_t *end_off, int64_t nends,
                             int level, uint8_t *dst, hipStream_t stream_) {
    int64_t grid = nblocks + (nends + 255) / 256;
    if (grid <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_lz4_gather, dim3((unsigned)grid), dim3(256), 0, stream_, slots, slot_bytes, sizes,
                       frame_off, nblocks, end_off, nends, level, dst);
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
                             uint32_t *err, hipStream_t s) {
    if (nframes <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_lz4_decode, dim3((unsigned)nframes), dim3(64), 0, s, in, desc, nframes, out, err);
    return hipGetLastError();
}
}  // namespace sgx
