#!/usr/bin/env python3
"""A/B sweep of map-side kernel configurations in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24).  Prints median/min per-stage ms per variant and
checks every variant's output against the first one (bit-exact)."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 28)
    ap.add_argument("--partitions", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--variants", default="0:0:0,256:4:16,256:8:16,512:4:16,1024:4:16,256:4:8,256:8:8")
    ap.add_argument("--dist", default="uniform")
    a = ap.parse_args()
    import numpy as np

    import sparkucx_amd as sgx

    # variant = chunks:waves:items[:ENV=VALUE] (the engine reads its A/B switches at creation)
    variants, engines = [], []
    for v in a.variants.split(","):
        f = v.split(":")
        g, w, i = (int(x) for x in f[:3])
        env = dict(kv.split("=") for kv in f[3:])
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        engines.append(sgx.ShuffleEngine(0, g, w, i))
        for k, o in old.items():
            if o is None:
                os.environ.pop(k)
            else:
                os.environ[k] = o
        variants.append(v)
    n, R = a.records, a.partitions
    buf = engines[0].alloc(n * 16)
    if a.dist == "uniform":
        engines[0].gen_uniform16(buf, n, 0x5EEDC0DE)
    else:
        r = np.arange(1, (1 << 24) + 1, dtype=np.float64)
        cdf = np.cumsum(r ** -1.1)
        cdf /= cdf[-1]
        engines[0].gen_zipf16(buf, n, 0x5EEDC0DE, cdf)
    for e in engines:
        e.register_shuffle(1, R)
    res = [{"hist": [], "scan": [], "scatter": []} for _ in variants]
    ref = None
    for rnd in range(a.rounds + 1):
        for vi, (v, e) in enumerate(zip(variants, engines)):
            per = {"hist": [], "scan": [], "scatter": []}
            for it in range(a.iters):
                e.stats_reset()
                e.write_map(1, 0, buf, n, 16)
                e.sync()
                st = e.stats()
                for k in per:
                    per[k].append(st.ms[k] / max(1, st.count[k]))
            if rnd == 0:  # warm-up round: check outputs instead of timing
                out = e.map_output_bytes(1, 0)
                h = hash(out.tobytes()[:: 4097]) ^ int(out[-16:].sum())
                if ref is None:
                    ref = (h, out)
                else:
                    assert np.array_equal(out, ref[1]), f"variant {v} differs"
                del out
                continue
            for k in per:
                res[vi][k].extend(per[k])
    out = []
    for vi, v in enumerate(variants):
        row = {"variant(num_chunks:waves:items[:env])": v}
        for k, xs in res[vi].items():
            row[k + "_med"] = round(statistics.median(xs), 4)
            row[k + "_min"] = round(min(xs), 4)
        row["scatter_algo_GBs"] = round(32 * n / (row["scatter_med"] * 1e-3) / 1e9, 1)
        row["hist_GBs"] = round(16 * n / (row["hist_med"] * 1e-3) / 1e9, 1)
        row["total_ms"] = round(row["hist_med"] + row["scan_med"] + row["scatter_med"], 4)
        out.append(row)
        print(json.dumps(row), flush=True)
    for e in engines:
        e.close()


if __name__ == "__main__":
    main()
