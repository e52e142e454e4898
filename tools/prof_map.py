#!/usr/bin/env python3
"""Profiling driver: run the map-side write (C1 by default) a few times so rocprofv3 can
trace / count the kernels.  Usage under the profiler (program directly after --):
  rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 tools/prof_map.py
  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc1 -o run -- python3 tools/prof_map.py
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 28)
    ap.add_argument("--partitions", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--num-chunks", type=int, default=0)
    ap.add_argument("--dist", default="uniform")
    ap.add_argument("--flags", type=int, default=0, help="sgx_config.flags (FLAG_*)")
    ap.add_argument("--record-bytes", type=int, default=16, choices=[16, 100])
    ap.add_argument("--batches", type=int, default=1, help="> 1: map_begin / append (retained slices) / commit")
    ap.add_argument("--slots", type=int, default=2, help="map ids the writes cycle through (bench.py: 2)")
    ap.add_argument("--per-launch", action="store_true",
                    help="print every write's stage events (PER_LAUNCH json), each write alone on the GPU")
    a = ap.parse_args()
    import numpy as np

    import sparkucx_amd as sgx

    # kernel profiles are of kernels alone: consecutive writes on one stream (overlapping writes
    # make a K4's traced duration include its wait for the previous K4's CUs)
    e = sgx.ShuffleEngine(0, a.num_chunks, flags=a.flags | sgx.FLAG_NO_OVERLAP_WRITES)
    buf = e.alloc(a.records * a.record_bytes)
    if a.record_bytes == 100:
        e.gen_terasort100(buf, a.records, 0x5EEDC0DE)
    elif a.dist == "uniform":
        e.gen_uniform16(buf, a.records, 0x5EEDC0DE)
    else:
        r = np.arange(1, (1 << 24) + 1, dtype=np.float64)
        cdf = np.cumsum(r ** -1.1)
        cdf /= cdf[-1]
        e.gen_zipf16(buf, a.records, 0x5EEDC0DE, cdf)
    if a.record_bytes == 100:
        # evenly spaced 10-byte bounds (the sampled bounds' shape; the kernels do not care)
        hi = (np.arange(1, a.partitions, dtype=np.uint64) * (np.uint64(1 << 63) // np.uint64(a.partitions)) * 2)
        bounds = np.zeros((a.partitions - 1, 10), np.uint8)
        for j in range(8):
            bounds[:, j] = (hi >> np.uint64(56 - 8 * j)) & np.uint64(0xFF)
        e.register_shuffle(1, a.partitions, kind=sgx.PART_RANGE_BYTES10, bounds=bounds, record_bytes=100)
    else:
        e.register_shuffle(1, a.partitions)
    cuts = [a.records * j // a.batches for j in range(a.batches + 1)]
    import json

    per = []  # this launch's stage events (ms), for tools/reconcile_trace.py
    for i in range(a.iters):
        if a.per_launch:
            e.sync()
            e.stats_reset()
        if a.batches <= 1:
            e.write_map(1, i % a.slots, buf, a.records, a.record_bytes)
        else:
            e.map_begin(1, i % a.slots)
        for j in range(a.batches if a.batches > 1 else 0):
            e.map_append(1, i % a.slots, buf, cuts[j + 1] - cuts[j], a.record_bytes, offset=cuts[j] * a.record_bytes,
                         retained=True)
        if a.batches > 1:
            e.map_commit(1, i % a.slots)
        if a.per_launch:
            e.sync()
            st = e.stats()
            per.append({k: round(v, 4) for k, v in st.ms.items() if st.count[k]})
    e.sync()
    if a.per_launch:
        print("PER_LAUNCH " + json.dumps(per))
    st = e.stats()
    print({k: round(v / max(1, st.count[k]), 4) for k, v in st.ms.items() if st.count[k]})
    e.close()


if __name__ == "__main__":
    main()
