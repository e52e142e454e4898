#!/usr/bin/env python3
"""Per-stage timings of the map-side write on the other BASELINE configs (one GPU):
  uniform / Zipf(1.1) 16 B records at R = 200, 1024, 4096, and TeraSort 100 B records with
  sampled RangePartitioner bounds (R = 1024).  Prints one JSON line per config."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def terasort_bounds(host_keys, R, seed):
    import numpy as np

    rng = np.random.default_rng(seed)
    sample = host_keys[rng.choice(len(host_keys), min(len(host_keys), 20 * R), replace=False)]
    sample = sample[np.lexsort(sample.T[::-1])]
    step = len(sample) / R
    return np.ascontiguousarray(sample[[int(step * (i + 1)) for i in range(R - 1)]])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 28)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--configs", default="uniform:200,uniform:1024,uniform:4096,zipf:1024,zipf:4096,terasort:1024")
    a = ap.parse_args()
    import numpy as np

    import sparkucx_amd as sgx

    e = sgx.ShuffleEngine(0)
    sid = 0
    for cfg in a.configs.split(","):
        dist, R = cfg.split(":")
        R = int(R)
        sid += 1
        if dist == "terasort":
            n = a.records * 16 // 100  # same input bytes as the 16 B configs
            rb = 100
            buf = e.alloc(n * rb)
            e.gen_terasort100(buf, n, 0x5EEDC0DE)
            keys = buf.to_numpy(min(n, 1 << 20) * rb).reshape(-1, rb)[:, :10].copy()
            e.register_shuffle(sid, R, sgx.PART_RANGE_BYTES10, terasort_bounds(keys, R, 7), True, rb)
        else:
            n, rb = a.records, 16
            buf = e.alloc(n * rb)
            if dist in ("uniform", "range"):
                e.gen_uniform16(buf, n, 0x5EEDC0DE)
            else:
                r = np.arange(1, (1 << 24) + 1, dtype=np.float64)
                cdf = np.cumsum(r ** -1.1)
                cdf /= cdf[-1]
                e.gen_zipf16(buf, n, 0x5EEDC0DE, cdf)
            if dist == "range":  # RangePartitioner over the Long keys (sortByKey): sampled, distinct bounds
                keys = buf.to_numpy(min(n, 1 << 20) * 16).reshape(-1, 16)[:, :8].copy().view(np.int64).ravel()
                rng = np.random.default_rng(R)
                smp = np.unique(keys[rng.choice(len(keys), 20 * R, replace=False)])
                bounds = smp[np.linspace(0, len(smp) - 1, R + 1).astype(int)[1:-1]]
                e.register_shuffle(sid, R, sgx.PART_RANGE_I64, bounds, True, 16)
            else:
                e.register_shuffle(sid, R)
        e.write_map(sid, 0, buf, n, rb, R)  # warm-up
        e.sync()
        e.stats_reset()
        for _ in range(a.iters):
            e.write_map(sid, 0, buf, n, rb, R)
        e.sync()
        st = e.stats()
        ms = {k: st.ms[k] / max(1, st.count[k]) for k in ("hist", "scan", "scatter")}
        tot = sum(ms.values())
        print(json.dumps({"config": cfg, "records": n, "record_bytes": rb,
                          **{k + "_ms": round(v, 4) for k, v in ms.items()},
                          "map_side_GBs": round(n * rb / (tot * 1e-3) / 1e9, 1),
                          "scatter_algo_GBs": round(2 * n * rb / (ms["scatter"] * 1e-3) / 1e9, 1)}), flush=True)
        e.unregister_shuffle(sid)
        buf.free()
    e.close()


if __name__ == "__main__":
    main()
