#!/usr/bin/env python3
"""LZ4 framing time vs stream size: a Kryo (Long, Long) map of N uniform records (R = 1024),
framed whole (one sgx_lz4_frame_partitions call) and in slices of `--slice` partitions per
call.  Prints one JSON line per N: ms per call, ns per 32 KiB block."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", default="24,26,28")
    ap.add_argument("--slice", type=int, default=64)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    import numpy as np

    import sparkucx_amd as sgx
    from sparkucx_amd._lib import check, lib

    e = sgx.ShuffleEngine(0, 0)
    R = 1024
    for sid, l2 in enumerate(int(x) for x in a.log2n.split(",")):
        n = 1 << l2
        buf = e.alloc(n * 16)
        e.gen_uniform16(buf, n, 0x5EEDC0DE)
        e.register_shuffle(sid + 1, R)
        e.set_serializer(sid + 1, 1)
        e.write_map(sid + 1, 0, buf, n, 16)
        e.sync()
        buf.free()
        lens = e.map_lengths(sid + 1, 0, R)
        offs = np.zeros(R + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        ptr, nbytes = e.map_data(sid + 1, 0)
        flen = np.empty(R, dtype=np.int64)
        check(lib().sgx_lz4_frame_partitions(e.handle, ptr, offs.ctypes.data, R, 32768, None, 0,
                                             flen.ctypes.data), "measure")
        total = int(flen.sum())
        dst = e.alloc(total)
        nblocks = int(sum((int(l) + 32767) // 32768 for l in lens))

        def whole():
            check(lib().sgx_lz4_frame_partitions(e.handle, ptr, offs.ctypes.data, R, 32768, dst.ptr, total,
                                                 flen.ctypes.data), "frame")

        def sliced():
            s = a.slice
            for p0 in range(0, R, s):
                o = (offs[p0:p0 + s + 1] - offs[p0]).copy()
                fl = np.empty(s, dtype=np.int64)
                check(lib().sgx_lz4_frame_partitions(e.handle, ptr + int(offs[p0]), o.ctypes.data, s, 32768,
                                                     dst.ptr, total, fl.ctypes.data), "frame slice")

        res = {"records": n, "stream_bytes": int(nbytes), "blocks": nblocks}
        for name, fn in (("whole", whole), ("sliced", sliced)):
            ts = []
            for _ in range(a.iters + 1):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            t = float(np.median(ts[1:]))
            res[name + "_ms"] = round(t * 1e3, 3)
            res[name + "_ns_per_block"] = round(t * 1e9 / nblocks, 1)
        print(json.dumps(res), flush=True)
        dst.free()
        e.unregister_shuffle(sid + 1)
    e.close()


if __name__ == "__main__":
    main()
