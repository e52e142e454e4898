"""Collect the bench JSON lines of round-6 gpurun runs into one JSONL (profiles/r06/).

usage: python tools/r06/summarize_logs.py gpurun_out/r06a gpurun_out/r06b ... > profiles/r06/r06_runs.jsonl
Each output line: run, log, value, ms_per_step, K4 / map-side fractions, stage ms, exchange.
"""
import json
import os
import sys

for d in sys.argv[1:]:
    for f in sorted(os.listdir(d)):
        if not f.endswith(".log"):
            continue
        line = None
        with open(os.path.join(d, f), errors="replace") as fh:
            for ln in fh:
                if ln.startswith("{") and '"metric"' in ln:
                    line = ln
        if line is None:
            continue
        j = json.loads(line)
        rec = {"run": os.path.basename(d), "log": f, "workload": j["config"].get("workload"),
               "value": j["value"], "ms_per_step": j["ms_per_step"],
               "k4_frac": j["roofline"]["frac"], "map_side_frac": j["roofline_map_side"]["frac"],
               "map_side_ms": j["roofline_map_side"]["ms"], "stages_ms": j.get("stages_ms_per_step"),
               "exchange": j["config"].get("exchange"), "exchange_bytes": j.get("exchange_bytes"),
               "host_ingest": j.get("host_ingest")}
        print(json.dumps(rec))
