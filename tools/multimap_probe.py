#!/usr/bin/env python3
"""Probe (measurement tool): the C1 input (2^28 x 16 B) written as M map tasks of N/M records
each, back to back on the engine's stream, vs one map of N records.  A map task of <=128 MB
fits the 256 MiB Infinity Cache, so K4 can re-read what K1+K2 just read from on-die memory
instead of HBM.  Prints per-stage ms per step and the whole-step wall time."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class View:
    """A device sub-buffer in the duck-typed tensor form engine.buffer_arg accepts."""

    is_cuda = True

    def __init__(self, ptr, nbytes):
        self.ptr, self.nbytes = ptr, nbytes

    def data_ptr(self):
        return self.ptr

    def is_contiguous(self):
        return True

    def numel(self):
        return self.nbytes

    def element_size(self):
        return 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 28)
    ap.add_argument("--partitions", type=int, default=1024)
    ap.add_argument("--maps", default="1,8,16,32,64")
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--chunks", default="0", help="comma list of num_chunks (0 = one per CU)")
    a = ap.parse_args()
    import sparkucx_amd as sgx

    for G in [int(x) for x in a.chunks.split(",")]:
        run(sgx, a, G)


def run(sgx, a, G):
    e = sgx.ShuffleEngine(0, num_chunks=G)
    n, R = a.records, a.partitions
    buf = e.alloc(n * 16)
    e.gen_uniform16(buf, n, 0x5EEDC0DE)
    for M in [int(x) for x in a.maps.split(",")]:
        sid = 100 + M
        e.register_shuffle(sid, R)
        per = n // M
        views = [View(buf.ptr + j * per * 16, per * 16) for j in range(M)]
        walls = []
        for it in range(a.iters + 1):
            e.sync()
            e.stats_reset()
            t0 = time.perf_counter()
            for j in range(M):
                e.write_map(sid, j, views[j], per, 16)
            e.sync()
            dt = time.perf_counter() - t0
            if it:
                walls.append(dt)
        st = e.stats()
        row = {"chunks": G, "maps": M, "records_per_map": per, "MB_per_map": per * 16 / 2**20,
               "wall_ms_per_step": round(1e3 * min(walls), 3),
               "shuffled_GBs": round(16 * n / min(walls) / 1e9, 1)}
        for k in ("hist", "scan", "scatter"):
            c = max(1, st.count[k])
            row[k + "_ms_sum_per_step"] = round(st.ms[k] / c * M, 4)
        row["k4_algo_GBs"] = round(32 * n / (row["scatter_ms_sum_per_step"] * 1e-3) / 1e9, 1)
        print(json.dumps(row), flush=True)
        e.unregister_shuffle(sid)
    buf.free()
    e.close()


if __name__ == "__main__":
    main()
