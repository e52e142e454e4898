#!/usr/bin/env python3
"""Reduce-side timings on one GPU (UcxShuffleReader.read after the fetch): one map of N
records (uniform or Zipf 16 B, or TeraSort 100 B with sampled RangePartitioner bounds) is
written, then every reducer is read back sorted by key (sortByKey / TeraSort) or grouped
(groupByKey, reduceByKey sum), on device memory.  Prints one JSON line per case with the
engine's per-stage HIP-event times (regroup = fetch gather, sort = LSD digit passes +
partitioner pass, group = grouping kernels)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 26)
    ap.add_argument("--partitions", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--cases", default="sorted:uniform,group:uniform,sum:zipf,sorted:terasort")
    ap.add_argument("--flags", type=int, default=0, help="sgx_config.flags (64 = SGX_FLAG_NO_BUCKET_SORT)")
    a = ap.parse_args()
    import numpy as np

    import sparkucx_amd as sgx

    e = sgx.ShuffleEngine(0, flags=a.flags)
    R = a.partitions
    sid = 0
    for case in a.cases.split(","):
        op, dist = case.split(":")
        sid += 1
        n = a.records if dist != "terasort" else a.records * 16 // 100
        rb = 100 if dist == "terasort" else 16
        buf = e.alloc(n * rb)
        kind, bounds = sgx.PART_HASH, None
        if dist == "uniform":
            e.gen_uniform16(buf, n, 0x5EEDC0DE)
        elif dist == "zipf":
            r = np.arange(1, (1 << 24) + 1, dtype=np.float64)
            cdf = np.cumsum(r ** -1.1)
            cdf /= cdf[-1]
            e.gen_zipf16(buf, n, 0x5EEDC0DE, cdf)
        else:
            e.gen_terasort100(buf, n, 0x5EEDC0DE)
            keys = buf.to_numpy(min(n, 1 << 20) * 100).reshape(-1, 100)[:, :10]
            rng = np.random.default_rng(1)
            sample = keys[rng.choice(len(keys), 20 * R, replace=False)]
            sample = sample[np.lexsort(sample.T[::-1])]
            bounds = np.ascontiguousarray(sample[np.linspace(0, len(sample) - 1, R - 1).astype(int)])
            kind = sgx.PART_RANGE_BYTES10
        e.register_shuffle(sid, R, kind, bounds, True, rb)
        e.write_map(sid, 0, buf, n, rb, R)
        dst = e.alloc(n * rb) if op == "sorted" else None
        if op == "sorted":  # warm-up: first-touch of the sort / gather buffers stays out of the timings
            e.read_sorted(sid, [0], 0, R, dst)
        e.stats_reset()
        walls, walls_host = [], []
        agg = sgx.AGG_SUM if op == "sum" else sgx.AGG_GROUP
        for _ in range(a.iters):
            t0 = time.perf_counter()
            if op == "sorted":
                e.read_sorted(sid, [0], 0, R, dst)
            else:  # results left in HBM (the GPU consumer's case)
                for b in e.read_grouped(sid, [0], 0, R, agg, device=True):
                    b.free()
            walls.append(time.perf_counter() - t0)
        walls_touched = []
        if op != "sorted":  # host arrays: + PCIe copy and first-touch page faults of fresh arrays
            for _ in range(2):
                t0 = time.perf_counter()
                res = e.read_grouped(sid, [0], 0, R, agg)
                walls_host.append(time.perf_counter() - t0)
            # the same into arrays whose pages are already mapped (a JVM direct buffer is zeroed
            # when it is allocated): the copy alone
            out = [np.ones(len(x) + 1, dtype=np.int64) for x in res]
            out = (out[0], out[1], out[2]) if len(out) == 3 else (out[0], None, out[1])
            for _ in range(2):
                t0 = time.perf_counter()
                e.read_grouped(sid, [0], 0, R, agg, out=out)
                walls_touched.append(time.perf_counter() - t0)
        st = e.stats()
        ms = {k: round(v / max(1, st.count[k]), 3) for k, v in st.ms.items() if st.count[k]}
        dev_ms = ms.get("regroup", 0) + ms.get("sort", 0) + ms.get("group", 0)
        print(json.dumps({"case": case, "records": n, "record_bytes": rb, "partitions": R, "stages_ms": ms,
                          "device_ms": round(dev_ms, 3), "device_GBs": round(n * rb / dev_ms / 1e6, 1),
                          "wall_ms_min": round(min(walls) * 1e3, 2),
                          "wall_ms_host_arrays": round(min(walls_host) * 1e3, 2) if walls_host else None,
                          "wall_ms_host_arrays_mapped": round(min(walls_touched) * 1e3, 2) if walls_touched else None}),
              flush=True)
        e.unregister_shuffle(sid)
        if dst is not None:
            dst.free()
        buf.free()
    e.close()


if __name__ == "__main__":
    main()
