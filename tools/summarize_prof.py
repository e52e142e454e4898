#!/usr/bin/env python3
"""Turn rocprofv3 outputs of tools/gpu_prof.sh (kernel-trace stats + separate FETCH_SIZE /
WRITE_SIZE PMC passes over tools/prof_map.py) into committed summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   copy of rocprofv3's per-kernel stats
  profiles/<tag>_summary.md          per-kernel mean duration and HBM traffic per launch
  profiles/pmc_map.json              per workload: K4 and whole-map-side HBM bytes per step,
                                     read by bench.py (roofline.traffic, roofline_map_side)

HBM traffic per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads exactly half of a wide
coalesced stream on gfx950, so it is doubled; WRITE_SIZE (KiB) is taken as is.  The map side
is every kernel of the write except the input generator, per write (calls / iters).

usage: summarize_prof.py <tag> <out_dir of gpu_prof.sh> <records> <R> <dist> [record_bytes] [layout]
layout: padded (the default map write) or twopass (--flags 256); pmc_map.json keys
a two-pass profile with the suffix "_twopass" (bench.py --no-padded reads that one).
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def pmc(d, counter):
    out = defaultdict(list)
    for fn in ("run_counter_collection.csv",):
        with open(os.path.join(d, fn)) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == counter:
                    out[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return out


def main():
    tag, d, n, R, dist = sys.argv[1:6]
    rb = int(sys.argv[6]) if len(sys.argv) > 6 else 16
    layout = sys.argv[7] if len(sys.argv) > 7 else "padded"
    assert layout in ("padded", "twopass"), layout
    n, R = int(n), int(R)
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(d, "kt", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    stats = {}
    with open(os.path.join(d, "kt", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            stats[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
    fetch, write = pmc(os.path.join(d, "fetch"), "FETCH_SIZE"), pmc(os.path.join(d, "write"), "WRITE_SIZE")
    iters_kt, iters_pmc = 5, 2
    algo = 2 * rb * n
    lines = [f"# rocprofv3 summary `{tag}` — map-side write ({layout}), {n} x {rb} B records ({dist}), R = {R}", "",
             "| kernel | calls/write | mean µs | HBM read GB/launch (FETCH×2) | HBM write GB/launch | traffic GB/s |",
             "|---|---|---|---|---|---|"]
    side = {"read_bytes": 0.0, "write_bytes": 0.0, "us": 0.0}
    k4 = None
    for k, (calls, avg) in sorted(stats.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        if k.replace("sgx::", "").startswith(("k_gen", "k_lds_order_probe")):
            continue  # the input generator; the engine-start LDS ordering check (once per engine)
        per = calls / iters_kt
        rd = statistics.median(fetch[k]) * 2 * 1024 if k in fetch else 0.0
        wr = statistics.median(write[k]) * 1024 if k in write else 0.0
        tr = (rd + wr) / (avg * 1e-9) / 1e9
        lines.append(f"| `{k}` | {per:g} | {avg / 1e3:.1f} | {rd / 1e9:.3f} | {wr / 1e9:.3f} | {tr:.0f} |")
        side["read_bytes"] += rd * per
        side["write_bytes"] += wr * per
        side["us"] += avg / 1e3 * per
        if k.replace("sgx::", "").startswith("k_scatter"):
            # K4: every scatter level of a write (one kernel, or the two levels of the split
            # scatter at R > 1024) against the record's one read and one write
            if k4 is None:
                k4 = {"kernel": k, "hbm_bytes_per_launch": 0, "read_bytes": 0, "write_bytes": 0,
                      "algorithmic_bytes": algo, "mean_ns": 0.0}
            else:
                k4["kernel"] += " + " + k
            k4["hbm_bytes_per_launch"] += int((rd + wr) * per)
            k4["read_bytes"] += int(rd * per)
            k4["write_bytes"] += int(wr * per)
            k4["mean_ns"] += avg * per
    tot = side["read_bytes"] + side["write_bytes"]
    lines += ["", f"Map side per write: {side['us']:.1f} µs of kernels, HBM {tot / 1e9:.3f} GB "
              f"(read {side['read_bytes'] / 1e9:.3f}, write {side['write_bytes'] / 1e9:.3f}); algorithmic "
              f"{algo / 1e9:.3f} GB ({2 * rb} B x records: the record read once and written once) -> "
              f"{tot / algo:.3f}x."]
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    path = os.path.join(prof, "pmc_map.json")
    cur = json.load(open(path)) if os.path.exists(path) else {}
    cur[f"{dist}_n{n}_R{R}_rb{rb}" + ("_twopass" if layout == "twopass" else "")] = {"scatter": k4, "map_side": {
        "hbm_bytes_per_write": int(tot), "read_bytes": int(side["read_bytes"]),
        "write_bytes": int(side["write_bytes"]), "kernel_us": round(side["us"], 1),
        "algorithmic_bytes": algo, "ratio": round(tot / algo, 4)}, "source": tag, "layout": layout}
    json.dump(cur, open(path, "w"), indent=1, sort_keys=True)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
