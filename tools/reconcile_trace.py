#!/usr/bin/env python3
"""The two clocks of one run side by side: the engine's stage events (HIP events on the
compute stream, what bench.py's roofline fields divide by) and rocprofv3's kernel trace of
the SAME launches.  Run tools/prof_map.py --per-launch under the tracer, then:
    python tools/reconcile_trace.py <run_kernel_trace.csv> <prof_map stdout log>
Prints one JSON line per write: K4's event interval vs its traced duration, and the map side
(the events from the first to the last stage boundary) vs the traced span of the write's
kernels (first start to last end) and the sum of their durations."""
import csv
import json
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    per = None
    for line in open(sys.argv[2]):
        if line.startswith("PER_LAUNCH "):
            per = json.loads(line[len("PER_LAUNCH "):])
    if per is None:
        raise SystemExit("no PER_LAUNCH line in the log")
    # the writes: each starts at its sample (padded) or histogram (two-pass) kernel
    writes, cur = [], None
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sgx::", "") for r in rows]
    padded = any(n.startswith("k_pad_sample") for n in names)  # else two-pass writes start at k_hist
    for r, name in zip(rows, names):
        if name.startswith(("k_gen", "k_lds_order_probe", "__amd")):
            continue
        first = name.startswith("k_pad_sample") if padded else name.startswith("k_hist")
        if first or cur is None:
            cur = []
            writes.append(cur)
        cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = []
    for i, (w, ev) in enumerate(zip(writes, per)):
        k4 = [k for k in w if k[0].startswith("k_scatter") and (k[2] - k[1]) > 50_000]
        k4_ms = sum(k[2] - k[1] for k in k4) / 1e6
        span = (max(k[2] for k in w) - min(k[1] for k in w)) / 1e6
        busy = sum(k[2] - k[1] for k in w) / 1e6
        side = ev.get("hist", 0) + ev.get("scan", 0) + ev.get("scatter", 0)
        out.append({"write": i, "k4_kernel": k4[0][0] if k4 else None, "k4_trace_ms": round(k4_ms, 4),
                    "k4_event_ms": ev.get("scatter"), "map_side_event_ms": round(side, 4),
                    "map_side_trace_span_ms": round(span, 4), "map_side_trace_busy_ms": round(busy, 4),
                    "kernels": len(w)})
        print(json.dumps(out[-1]))
    if out:
        n = len(out)
        m = lambda k: round(sum(o[k] or 0 for o in out) / n, 4)
        print(json.dumps({"mean": {k: m(k) for k in ("k4_trace_ms", "k4_event_ms", "map_side_event_ms",
                                                       "map_side_trace_span_ms", "map_side_trace_busy_ms")},
                          "writes": n}))


if __name__ == "__main__":
    main()
