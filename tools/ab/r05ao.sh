#!/bin/bash
# Chunks per map (workgroups of K4): 256 (default, one per CU) vs 384 / 512 / 768; C1 and C4.
tag=${1:-r05ao}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
C="--no-cpu-baseline --no-live-pmc"
for i in 1 2; do
  for g in 256 384 512 768; do
    timeout -k 10 180 python -u bench.py $C --num-chunks $g > "$out/c1_g${g}_$i.log" 2>&1 || fail "c1 $g" "$out/c1_g${g}_$i.log"
    timeout -k 10 180 python -u bench.py $C --num-chunks $g --workload c4 > "$out/c4_g${g}_$i.log" 2>&1 || fail "c4 $g" "$out/c4_g${g}_$i.log"
  done
done
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["roofline_map_side"].get("traffic_over_algorithmic"), d["stages_ms_per_step"])
PY
echo done > "$out/DONE"
