#!/usr/bin/env python3
"""Overlap of the map side with the exchange, from a rocprofv3 kernel trace of
`bench.py --self-exchange` (one GPU, one-rank RCCL communicator) or of one rank of an N > 1
run: for every RCCL all-to-all kernel, the time during which a map-side kernel (histogram,
scan, scatter) of the NEXT map ran concurrently, and the step timeline.
    python tools/overlap_from_trace.py <run_kernel_trace.csv>
"""
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = []
    for r in rows:
        name = r["Kernel_Name"]
        kind = ("map" if any(k in name for k in ("k_hist", "k_scan", "k_scatter")) else
                "a2a" if ("ncclDevKernel" in name or "nccl" in name.lower()) else None)
        if kind:
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, name.split("(")[0][:60],
                       int(r["Queue_Id"])))
    ks.sort()
    maps = [k for k in ks if k[2] == "map"]
    comms = [k for k in ks if k[2] == "a2a"]
    out = []
    for s, e, _, name, q in comms:
        ov = sum(max(0, min(e, me) - max(s, ms)) for ms, me, *_ in maps)
        out.append({"kernel": name, "queue": q, "ms": round((e - s) / 1e6, 4),
                    "map_side_overlap_ms": round(ov / 1e6, 4)})
    long = [o for o in out if o["ms"] > 0.1]  # the all-to-all kernels (the all-gather ones are tiny)
    summ = {"rccl_kernels": len(out), "long_rccl_kernels": len(long),
            "long_ms_mean": round(sum(o["ms"] for o in long) / max(1, len(long)), 4),
            "overlap_ms_mean": round(sum(o["map_side_overlap_ms"] for o in long) / max(1, len(long)), 4),
            "map_kernels": len(maps), "map_queues": sorted({m[4] for m in maps}),
            "rccl_queues": sorted({c[4] for c in comms})}
    print(json.dumps(summ))
    for o in long[:12]:
        print(json.dumps(o))
    # each map kernel's duration while an all-to-all runs beside it (HBM shared with the
    # exchange) against its duration alone (the steps before the first / after the last one)
    by = {}
    for ms, me, _, name, _ in maps:
        ov = sum(max(0, min(e, me) - max(s, ms)) for s, e, *_ in comms if e - s > 1e5)
        frac = ov / max(1, me - ms)
        key = "overlapped" if frac > 0.9 else "alone" if frac == 0 else None
        if key:
            by.setdefault(name, {}).setdefault(key, []).append((me - ms) / 1e6)
    for name, d in by.items():
        row = {"map_kernel": name}
        for key in ("alone", "overlapped"):
            v = d.get(key, [])
            row[key + "_ms_mean"] = round(sum(v) / len(v), 4) if v else None
            row[key + "_n"] = len(v)
        if row["alone_ms_mean"] and row["overlapped_ms_mean"]:
            row["stretch"] = round(row["overlapped_ms_mean"] / row["alone_ms_mean"], 3)
        print(json.dumps(row))


if __name__ == "__main__":
    main()
