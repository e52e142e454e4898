// sgx_lz4_host.cpp — host side of the LZ4 codec (spark.shuffle.compress=true with
// spark.io.compression.codec=lz4, Spark 3.0.1's defaults): lz4-java's
// LZ4BlockOutputStream framing of partition streams and LZ4BlockInputStream on fetched
// blocks, both on the GPU (sgx_lz4.hip) with grow-only per-thread scratch.
#include "sgx_engine.h"

#include <algorithm>
#include <cstring>

using namespace sgx;

// alloc_dst: allocate the destination (exact size) instead of dst_dev.  Scratch: the
// context's grow-only lz4_* buffers (one allocation per size class, not per call).
int sgx::lz4_frame_impl(sgx_engine *e, Ctx &c, const void *stream_dev, const int64_t *part_offsets,
                        int32_t num_partitions, int32_t block_size, DevBuf *alloc_dst, void *dst_dev,
                        int64_t dst_cap, int64_t *out_lengths) {
    if (!e || !part_offsets || !out_lengths || num_partitions < 1)
        return fail_msg(SGX_ERR_INVALID, "sgx_lz4_frame_partitions: bad arguments");
    if (block_size < 64 || block_size > sgx::lz4_max_block())
        return fail_msg(SGX_ERR_UNSUPPORTED, "LZ4 block size %d outside [64, %d]", block_size, sgx::lz4_max_block());
    const int R = num_partitions;
    std::vector<int64_t> blocks;  // {src offset, length} per block
    std::vector<int32_t> first(R + 1);
    for (int r = 0; r < R; ++r) {
        first[r] = (int32_t)(blocks.size() / 2);
        int64_t a = part_offsets[r], b = part_offsets[r + 1];
        if (b < a || a < 0) return fail_msg(SGX_ERR_INVALID, "partition offsets decrease at %d", r);
        for (int64_t p = a; p < b; p += block_size) {
            blocks.push_back(p);
            blocks.push_back(std::min<int64_t>(block_size, b - p));
        }
    }
    const int64_t nb = (int64_t)blocks.size() / 2;
    first[R] = (int32_t)nb;
    if (nb > 0 && !stream_dev) return fail_msg(SGX_ERR_INVALID, "stream is NULL");
    // lz4-java: level = max(0, 32 - nlz(blockSize - 1) - COMPRESSION_LEVEL_BASE (10))
    const int level = std::max(0, 32 - __builtin_clz((unsigned)(block_size - 1)) - 10);
    const int64_t slot = ((int64_t)21 + block_size + block_size / 255 + 16 + 15) / 16 * 16;
    HIP_TRY(hipSetDevice(e->device));
    DevBuf &d_blocks = c.lz4_blocks, &d_slots = c.lz4_slots, &d_sizes = c.lz4_sizes, &d_offs = c.lz4_offs;
    hipStream_t st = c.st;
    // pinned staging: [block list nb x 16 | kernel error 32 | frame sizes nb x 4 | frame offsets (nb + R) x 8]
    const size_t h_blocks = 0, h_err = (size_t)nb * 16, h_sizes = h_err + 32, h_offs = (h_sizes + (size_t)nb * 4 + 7) & ~(size_t)7;
    SGX_TRY(c.lz4_host.ensure(h_offs + ((size_t)nb + R) * 8));
    char *hb = (char *)c.lz4_host.p;
    const int32_t *sizes = (const int32_t *)(hb + h_sizes);
    if (nb > 0) {
        SGX_TRY(d_blocks.ensure((size_t)nb * 16));
        SGX_TRY(d_slots.ensure((size_t)(nb * slot)));
        SGX_TRY(d_sizes.ensure((size_t)nb * 8));  // sizes | checks
        SGX_TRY(c.lz4_info.ensure(64));
        std::memcpy(hb + h_blocks, blocks.data(), (size_t)nb * 16);
        HIP_TRY(hipMemsetAsync(c.lz4_info.p, 0, 32, st));
        HIP_TRY(hipMemcpyAsync(d_blocks.p, hb + h_blocks, (size_t)nb * 16, hipMemcpyHostToDevice, st));
        hipEvent_t c0 = e->ev(), c1 = e->ev();
        HIP_TRY(hipEventRecord(c0, st));
        HIP_TRY(sgx::launch_lz4_blocks((const uint8_t *)stream_dev, part_offsets[R], (const int64_t *)d_blocks.p, nb,
                                       level, (uint8_t *)d_slots.p, slot, (int32_t *)d_sizes.p,
                                       (uint32_t *)d_sizes.p + nb, (int64_t *)c.lz4_info.p, st));
        SGX_TRY(debug_sync(e, st, "k_lz4_blocks + k_xxh32_blocks"));
        HIP_TRY(hipEventRecord(c1, st));
        e->record_stage(SGX_STAGE_COMPRESS, c0, c1);
        HIP_TRY(hipMemcpyAsync(hb + h_sizes, d_sizes.p, (size_t)nb * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(hb + h_err, c.lz4_info.p, 32, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        const int64_t *kerr = (const int64_t *)(hb + h_err);
        if (kerr[0])
            return fail_msg(SGX_ERR_HIP, "internal error: LZ4 block %lld (offset %lld, %lld bytes) %s", (long long)kerr[1],
                            (long long)kerr[2], (long long)kerr[3],
                            (kerr[0] & 1) ? "lies outside the stream" : "overflowed its frame slot");
    }
    // frame offsets (blocks of a partition back to back, then its end mark)
    int64_t *offs = (int64_t *)(hb + h_offs);  // nb frame offsets | end-mark offsets
    int64_t total = 0, nends = 0;
    for (int r = 0; r < R; ++r) {
        int64_t start = total;
        for (int32_t b = first[r]; b < first[r + 1]; ++b) {
            if (sizes[b] < 21 || sizes[b] > slot) return fail_msg(SGX_ERR_HIP, "LZ4 block %d: bad frame size %d", b, sizes[b]);
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
        return fail_msg(SGX_ERR_INVALID, "LZ4 frames need %lld bytes, destination holds %lld", (long long)total,
                    (long long)dst_cap);
    if (nb > 0) {
        SGX_TRY(d_offs.ensure((size_t)(nb + nends) * 8));
        HIP_TRY(hipMemcpyAsync(d_offs.p, offs, (size_t)(nb + nends) * 8, hipMemcpyHostToDevice, st));
        HIP_TRY(sgx::launch_lz4_gather((const uint8_t *)stream_dev, (const int64_t *)d_blocks.p,
                                       (const uint8_t *)d_slots.p, slot, (const int32_t *)d_sizes.p,
                                       (const uint32_t *)d_sizes.p + nb, (const int64_t *)d_offs.p, nb,
                                       (const int64_t *)d_offs.p + nb, nends, level, (uint8_t *)dst_dev, st));
        SGX_TRY(debug_sync(e, st, "k_lz4_gather"));
        HIP_TRY(hipStreamSynchronize(st));
    }
    return SGX_OK;
}

extern "C" int sgx_lz4_frame_partitions(sgx_engine *e, const void *stream_dev, const int64_t *part_offsets,
                                        int32_t num_partitions, int32_t block_size, void *dst_dev,
                                        int64_t dst_cap, int64_t *out_lengths) {
    sgx::TraceRange trace_("sgx_lz4_frame_partitions");
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    return lz4_frame_impl(e, *c, stream_dev, part_offsets, num_partitions, block_size, nullptr, dst_dev, dst_cap,
                          out_lengths);
}

// LZ4BlockInputStream on the reduce side: decompress fetched LZ4-framed partition streams
extern "C" int sgx_lz4_unframe(sgx_engine *e, const void *framed_dev, int64_t framed_bytes, void *dst_dev,
                               int64_t dst_cap, int64_t *out_bytes) {
    sgx::TraceRange trace_("sgx_lz4_unframe");
    if (!e) return fail_msg(SGX_ERR_INVALID, "engine is NULL");
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    return lz4_unframe_impl(e, *c, framed_dev, framed_bytes, nullptr, dst_dev, dst_cap, out_bytes);
}

static const char *walk_why(int64_t code) {
    static const char *why[] = {"", "truncated header", "bad magic", "unknown compression method",
                                "malformed end mark", "bad block lengths"};
    return why[code > 0 && code < 6 ? code : 0];
}

// Per-stream walk (stream extents known): counts per stream, host scan, descriptors.
static int walk_streams(sgx_engine *e, Ctx &c, const uint8_t *framed, const int64_t *stream_lens, int64_t ns,
                        int64_t *nframes, int64_t *nout) {
    hipStream_t st = c.st;
    // pinned staging: [soff (ns + 1) | cnt / bases 2 ns | err 1] int64
    SGX_TRY(c.lz4_host.ensure((size_t)(3 * ns + 2) * 8));
    int64_t *hs = (int64_t *)c.lz4_host.p, *hc = hs + ns + 1, *herr = hc + 2 * ns;
    hs[0] = 0;
    for (int64_t i = 0; i < ns; ++i) {
        if (stream_lens[i] < 0) return fail_msg(SGX_ERR_INVALID, "negative stream length");
        hs[i + 1] = hs[i] + stream_lens[i];
    }
    SGX_TRY(c.lz4_blocks.ensure((size_t)(3 * ns + 1) * 8));
    SGX_TRY(c.lz4_info.ensure(64));
    int64_t *ds = (int64_t *)c.lz4_blocks.p, *dc = ds + ns + 1;
    unsigned long long *derr = (unsigned long long *)c.lz4_info.p;
    HIP_TRY(hipMemcpyAsync(ds, hs, (size_t)(ns + 1) * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(derr, 0xFF, 8, st));
    HIP_TRY(launch_lz4_walk_streams(framed, ds, ns, dc, nullptr, derr, false, st));
    SGX_TRY(debug_sync(e, st, "k_lz4_walk_streams (count)"));
    HIP_TRY(hipMemcpyAsync(hc, dc, (size_t)ns * 16, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(herr, derr, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if ((unsigned long long)*herr != ~0ull)
        return fail_msg(SGX_ERR_INVALID, "LZ4 stream: %s at byte %lld", walk_why((int64_t)(*herr & 0xFF)),
                        (long long)((unsigned long long)*herr >> 8));
    int64_t k = 0, o = 0;
    for (int64_t i = 0; i < ns; ++i) {  // exclusive scan -> {first frame, output offset}
        const int64_t fk = hc[2 * i], fo = hc[2 * i + 1];
        hc[2 * i] = k;
        hc[2 * i + 1] = o;
        k += fk;
        o += fo;
    }
    *nframes = k;
    *nout = o;
    if (k == 0) return SGX_OK;
    SGX_TRY(c.lz4_desc.ensure((size_t)k * 16));
    HIP_TRY(hipMemcpyAsync(dc, hc, (size_t)ns * 16, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_lz4_walk_streams(framed, ds, ns, dc, (int64_t *)c.lz4_desc.p, derr, true, st));
    SGX_TRY(debug_sync(e, st, "k_lz4_walk_streams (descriptors)"));
    return SGX_OK;
}

// One walk over a buffer of unknown stream extents (one thread chases the headers).
static int walk_single(sgx_engine *e, Ctx &c, const uint8_t *framed, int64_t framed_bytes, bool want_desc,
                       int64_t *nframes, int64_t *nout) {
    // one walk normally suffices: room for a frame per 512 B of input (frames of full 32 KiB
    // blocks are ~64x sparser); a denser stream (tiny partitions) is walked again with room
    // for every frame
    int64_t cap = framed_bytes / 512 + 4096;
    DevBuf &d_info = c.lz4_info, &d_desc = c.lz4_desc;
    hipStream_t st = c.st;
    SGX_TRY(d_info.ensure(64));
    int64_t info[5];
    for (int pass = 0; pass < 2; ++pass) {
        SGX_TRY(d_desc.ensure((size_t)cap * 16));
        HIP_TRY(hipMemsetAsync(d_info.p, 0, 64, st));
        HIP_TRY(sgx::launch_lz4_walk(framed, framed_bytes, (int64_t *)d_desc.p, cap, (int64_t *)d_info.p, st));
        HIP_TRY(hipMemcpyAsync(info, d_info.p, 40, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (info[2] != 0 || info[0] <= cap || !want_desc) break;
        cap = info[0];
    }
    if (info[2] != 0)
        return fail_msg(SGX_ERR_INVALID, "LZ4 stream: %s at byte %lld", walk_why(info[2]), (long long)info[3]);
    *nframes = info[0];
    *nout = info[1];
    return SGX_OK;
}

extern "C" int sgx_lz4_unframe_streams(sgx_engine *e, const void *framed_dev, const int64_t *stream_lens,
                                       int64_t nstreams, void *dst_dev, int64_t dst_cap, int64_t *out_bytes) {
    sgx::TraceRange trace_("sgx_lz4_unframe_streams");
    if (!e || nstreams < 0 || (nstreams > 0 && !stream_lens)) return fail_msg(SGX_ERR_INVALID, "bad arguments");
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    int64_t total = 0;
    for (int64_t i = 0; i < nstreams; ++i) {
        if (stream_lens[i] < 0) return fail_msg(SGX_ERR_INVALID, "negative stream length");
        total += stream_lens[i];
    }
    return lz4_unframe_impl(e, *c, framed_dev, total, nullptr, dst_dev, dst_cap, out_bytes, stream_lens, nstreams);
}

// alloc_dst: size (decompressed + 64 B of decoder padding) and use it.  stream_lens (ns
// entries, summing to framed_bytes): the extents of the LZ4 streams in the buffer, when the
// caller knows them (the reader does), for the per-stream parallel walk.
int sgx::lz4_unframe_impl(sgx_engine *e, Ctx &c, const void *framed_dev, int64_t framed_bytes, DevBuf *alloc_dst,
                          void *dst_dev, int64_t dst_cap, int64_t *out_bytes, const int64_t *stream_lens,
                          int64_t nstreams) {
    if (!e || !out_bytes || framed_bytes < 0 || (framed_bytes > 0 && !framed_dev) || nstreams < 0 ||
        (nstreams > 0 && !stream_lens))
        return fail_msg(SGX_ERR_INVALID, "sgx_lz4_unframe: bad arguments");
    *out_bytes = 0;
    if (framed_bytes == 0) return SGX_OK;
    HIP_TRY(hipSetDevice(e->device));
    hipStream_t st = c.st;
    const uint8_t *framed = (const uint8_t *)framed_dev;
    const bool want = dst_dev || alloc_dst;
    int64_t nframes = 0, nout = 0;
    if (nstreams > 0) {
        int64_t sum = 0;
        for (int64_t i = 0; i < nstreams; ++i) sum += stream_lens[i];
        if (sum != framed_bytes)
            return fail_msg(SGX_ERR_INVALID, "LZ4 stream lengths sum to %lld, not %lld bytes", (long long)sum,
                            (long long)framed_bytes);
        SGX_TRY(walk_streams(e, c, framed, stream_lens, nstreams, &nframes, &nout));
    } else {
        SGX_TRY(walk_single(e, c, framed, framed_bytes, want, &nframes, &nout));
    }
    *out_bytes = nout;
    if (alloc_dst) {
        SGX_TRY(alloc_dst->ensure((size_t)nout + 64));
        dst_dev = alloc_dst->p;
        dst_cap = nout;
    }
    if (!dst_dev) return SGX_OK;
    if (nout > dst_cap)
        return fail_msg(SGX_ERR_INVALID, "LZ4 stream decodes to %lld bytes, destination holds %lld", (long long)nout,
                        (long long)dst_cap);
    if (nframes == 0) return SGX_OK;
    SGX_TRY(c.lz4_info.ensure(64));
    uint32_t *derr = (uint32_t *)((int64_t *)c.lz4_info.p + 4);
    HIP_TRY(hipMemsetAsync(derr, 0, 4, st));
    hipEvent_t d0 = e->ev(), d1 = e->ev();
    HIP_TRY(hipEventRecord(d0, st));
    HIP_TRY(sgx::launch_lz4_decode(framed, (const int64_t *)c.lz4_desc.p, nframes, (uint8_t *)dst_dev, derr,
                                   (e->flags & SGX_FLAG_LZ4_LANE_DECODE) != 0, st));
    SGX_TRY(debug_sync(e, st, "k_lz4_decode"));
    HIP_TRY(hipEventRecord(d1, st));
    e->record_stage(SGX_STAGE_DECOMPRESS, d0, d1);
    uint32_t herr = 0;
    HIP_TRY(hipMemcpyAsync(&herr, derr, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (herr & 1u) return fail_msg(SGX_ERR_INVALID, "LZ4 stream: corrupt compressed block");
    if (herr & 2u) return fail_msg(SGX_ERR_INVALID, "LZ4 stream: block checksum mismatch");
    return SGX_OK;
}
