#!/usr/bin/env python3
"""Per-write kernel time of a rocprofv3 kernel trace of bench.py, warm-up writes apart.

rocprofv3's --stats mean covers every launch.  In a short run the first launches run while
the GPU is still leaving its idle clocks: under the tracer, bench.py's 13 C1 writes took K4
1791, 1858, 1858, 1761, then 1629-1711 µs (profiles/r05w3_trace_steady.json).  This tool
splits the trace into writes and reports the map side of the timed steps alone, i.e. the
writes after bench.py's --warmup ones, next to the all-launch mean.
    python tools/trace_steady.py <run_kernel_trace.csv> --warmup 3 [--out file.json]
A write starts at its sample (k_pad_sample, padded) or histogram (k_hist, two-pass) kernel.
The input generator, the engine's start-up probe and runtime copies/fills are left out.
Since round 6 the padded write's tail kernels run beside the next write's K4, so a sum of a
write's kernel durations counts that overlap twice; `interval_us_*` is the time from one
write's first kernel start to the next one's -- the steady-state cost of a write."""
import argparse
import csv
import json
import statistics


def writes_of(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sgx::", "").strip() for r in rows]
    padded = any(n.startswith("k_pad_sample") for n in names)
    out, cur, starts = [], None, []
    for r, name in zip(rows, names):
        if name.startswith(("k_gen", "k_lds_order_probe", "__amd")):
            continue
        first = name.startswith("k_pad_sample") if padded else name.startswith("k_hist")
        if first or cur is None:
            cur = []
            out.append(cur)
            starts.append(int(r["Start_Timestamp"]))
        cur.append((name, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return out, starts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=3, help="bench.py's --warmup: writes left out")
    ap.add_argument("--bytes", type=float, default=8.589934592e9, help="algorithmic bytes per write (C1: 32 B x 2^28)")
    ap.add_argument("--out")
    a = ap.parse_args()
    ws, starts = writes_of(a.trace)
    iv = [(b - x) / 1e3 for x, b in zip(starts, starts[1:])]  # write i -> write i+1, µs
    # a write's own kernels: those of a regular write (the second; the last write's group also
    # holds whatever the run launched after its last step)
    own = {n for n, _ in ws[min(1, len(ws) - 1)]}
    ws = [[(n, d) for n, d in w if n in own] for w in ws]
    side = [sum(d for _, d in w) for w in ws]
    k4 = [max(d for _, d in w) for w in ws]
    steady = side[a.warmup:]
    res = {
        "writes": len(ws),
        "warmup": a.warmup,
        "k4_us_per_write": [round(x, 1) for x in k4],
        "map_side_us_per_write": [round(x, 1) for x in side],
        "map_side_us_all_mean": round(statistics.mean(side), 1),
        "map_side_us_timed_mean": round(statistics.mean(steady), 1) if steady else None,
        "k4_us_timed_mean": round(statistics.mean(k4[a.warmup:]), 1) if steady else None,
        "map_side_frac_timed": round(a.bytes / (statistics.mean(steady) * 1e-6) / 8e12, 4) if steady else None,
        "map_side_frac_all": round(a.bytes / (statistics.mean(side) * 1e-6) / 8e12, 4),
        "interval_us_per_write": [round(x, 1) for x in iv],
        "interval_us_timed_mean": round(statistics.mean(iv[a.warmup:]), 1) if len(iv) > a.warmup else None,
        "interval_frac_timed": (round(a.bytes / (statistics.mean(iv[a.warmup:]) * 1e-6) / 8e12, 4)
                                if len(iv) > a.warmup else None),
    }
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
