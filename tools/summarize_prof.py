#!/usr/bin/env python3
"""Turn rocprofv3 outputs (kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE PMC passes)
into committed summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   copy of rocprofv3's per-kernel stats
  profiles/<tag>_summary.md          per-kernel mean duration, HBM traffic per launch
  profiles/pmc_scatter.json          K4 HBM bytes per launch, read by bench.py

HBM traffic per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads exactly half of a wide
coalesced stream on gfx950, so it is doubled; WRITE_SIZE (KiB) is taken as is.

usage: summarize_prof.py <tag> <kernel_trace_dir> <fetch_dir> <write_dir> <records> <R>
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
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                out[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return out


def main():
    tag, kt, fd, wd, n, R = sys.argv[1:7]
    n, R = int(n), int(R)
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(kt, "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    stats = {}
    with open(os.path.join(kt, "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            stats[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
    fetch, write = pmc(fd, "FETCH_SIZE"), pmc(wd, "WRITE_SIZE")
    lines = [f"# rocprofv3 summary `{tag}` — map-side write, {n} x 16 B records, R = {R}", "",
             "| kernel | calls | mean µs | HBM read GB/launch (FETCH×2) | HBM write GB/launch | traffic GB/s |",
             "|---|---|---|---|---|---|"]
    out_json = {}
    for k, (calls, avg) in sorted(stats.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        rd = statistics.median(fetch[k]) * 2 * 1024 if k in fetch else None
        wr = statistics.median(write[k]) * 1024 if k in write else None
        tr = (rd + wr) / (avg * 1e-9) / 1e9 if rd is not None and wr is not None else None
        lines.append(f"| `{k}` | {calls} | {avg / 1e3:.1f} | {rd / 1e9 if rd else 0:.3f} | "
                     f"{wr / 1e9 if wr else 0:.3f} | {tr or 0:.0f} |")
        if "k_scatter16" in k and rd is not None and wr is not None:
            out_json[f"uniform_n{n}_R{R}"] = {"kernel": k, "hbm_bytes_per_launch": int(rd + wr),
                                              "read_bytes": int(rd), "write_bytes": int(wr),
                                              "algorithmic_bytes": 32 * n, "mean_ns": avg, "source": tag}
    lines += ["", f"Algorithmic bytes of K4 per launch: 32 x {n} = {32 * n / 1e9:.3f} GB "
              "(16 B read + 16 B write per record)."]
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    if out_json:
        path = os.path.join(prof, "pmc_scatter.json")
        cur = json.load(open(path)) if os.path.exists(path) else {}
        cur.update(out_json)
        json.dump(cur, open(path, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
