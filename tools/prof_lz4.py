#!/usr/bin/env python3
"""LZ4 shuffle compression on one GPU: a Kryo (Long, Long) map output of N records
(R = 1024 reducers) is written, then every partition stream is framed as
LZ4BlockOutputStream (32 KiB blocks) by sgx_lz4_frame_partitions into device memory.
Two key distributions: uniform 64-bit keys (Kryo stream barely compresses -> mostly RAW
blocks) and low-entropy keys (k mod 4096: compresses).  Prints one JSON line per case:
wall time of the synchronous C-ABI call (both kernels + the host-side offset scan), input
GB/s, compression ratio, and the CPU oracle on a bounded sample (1 thread) for scale."""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 24)
    ap.add_argument("--partitions", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--lane-decode", action="store_true", help="force the lane-per-frame decoders")
    a = ap.parse_args()
    import numpy as np

    import oracle
    import sparkucx_amd as sgx
    from sparkucx_amd._lib import check, lib

    e = sgx.ShuffleEngine(0, flags=sgx.FLAG_LZ4_LANE_DECODE if a.lane_decode else 0)
    R, n = a.partitions, a.records
    for case in ("uniform", "lowentropy"):
        recs = oracle.gen_uniform16(n, 0x5EEDC0DE)
        if case == "lowentropy":
            recs[:, :8] = (np.arange(n, dtype=np.int64) % 4096).view(np.uint8).reshape(-1, 8)
        sid = 1 if case == "uniform" else 2
        e.register_shuffle(sid, R)
        e.set_serializer(sid, 1)
        e.write_map(sid, 0, recs, n, 16, num_partitions=R)
        lens = e.map_lengths(sid, 0, R)
        offs = np.zeros(R + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        ptr, nbytes = e.map_data(sid, 0)
        flen = np.empty(R, dtype=np.int64)
        check(lib().sgx_lz4_frame_partitions(e.handle, ptr, offs.ctypes.data, R, 32768, None, 0,
                                             flen.ctypes.data), "measure")
        total = int(flen.sum())
        dst = e.alloc(total)
        ts = []
        for _ in range(a.iters + 1):
            t0 = time.perf_counter()
            check(lib().sgx_lz4_frame_partitions(e.handle, ptr, offs.ctypes.data, R, 32768, dst.ptr, total,
                                                 flen.ctypes.data), "frame")
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts[1:]))
        # reduce side: decompress all frames back (LZ4BlockInputStream on the GPU)
        out = e.alloc(int(nbytes))
        got = ctypes.c_int64()
        ds = []
        for _ in range(a.iters + 1):
            t0 = time.perf_counter()
            check(lib().sgx_lz4_unframe(e.handle, dst.ptr, total, out.ptr, int(nbytes), ctypes.byref(got)), "unframe")
            ds.append(time.perf_counter() - t0)
        assert got.value == nbytes
        td = float(np.median(ds[1:]))
        # the reader's path: every partition stream's extent known -> per-stream walks
        ss = []
        e.stats_reset()
        for _ in range(a.iters + 1):
            t0 = time.perf_counter()
            check(lib().sgx_lz4_unframe_streams(e.handle, dst.ptr, flen.ctypes.data, R, out.ptr, int(nbytes),
                                                ctypes.byref(got)), "unframe streams")
            ss.append(time.perf_counter() - t0)
        assert got.value == nbytes
        tds = float(np.median(ss[1:]))
        st = e.stats()
        dec_ms = st.ms["decompress"] / max(1, st.count["decompress"])
        out.free()
        # CPU oracle on a bounded sample: the first 64 partitions' streams
        stream = np.empty(int(offs[64]), dtype=np.uint8)
        check(lib().sgx_memcpy(e.handle, stream.ctypes.data, ptr, int(offs[64])), "copy")
        c0 = time.perf_counter()
        oracle.lz4_frame_partitions(stream, offs[:65])
        ct = time.perf_counter() - c0
        print(json.dumps({"case": case, "lane_decode": a.lane_decode, "records": n, "partitions": R, "stream_bytes": int(nbytes),
                          "framed_bytes": total, "ratio": round(total / nbytes, 4),
                          "gpu_ms": round(t * 1e3, 3), "gpu_input_GBs": round(nbytes / t / 1e9, 2),
                          "gpu_decode_ms": round(td * 1e3, 3), "gpu_decode_out_GBs": round(nbytes / td / 1e9, 2),
                          "gpu_decode_streams_ms": round(tds * 1e3, 3),
                          "gpu_decode_streams_out_GBs": round(nbytes / tds / 1e9, 2),
                          "decode_kernel_ms": round(dec_ms, 3),
                          "cpu_oracle_1thread_GBs": round(int(offs[64]) / ct / 1e9, 3),
                          "cpu_sample_bytes": int(offs[64])}), flush=True)
        dst.free()
        e.unregister_shuffle(sid)
    e.close()


if __name__ == "__main__":
    main()
