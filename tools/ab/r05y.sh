#!/bin/bash
# Nontemporal tile loads: TeraSort K4 (wntl) and the 16 B K4 (cntl) vs the tree.
tag=${1:-r05y}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
C="--no-cpu-baseline --no-live-pmc"
for i in 1 2; do
  timeout -k 10 180 python -u bench.py --workload c4 $C > "$out/c4_tree_$i.log" 2>&1 || fail "c4" "$out/c4_tree_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_wntl.so bench --workload c4 $C > "$out/c4_wntl_$i.log" 2>&1 || fail "c4 wntl" "$out/c4_wntl_$i.log"
  timeout -k 10 180 python -u bench.py $C > "$out/c1_tree_$i.log" 2>&1 || fail "c1" "$out/c1_tree_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_cntl.so bench $C > "$out/c1_cntl_$i.log" 2>&1 || fail "c1 cntl" "$out/c1_cntl_$i.log"
done
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c*_*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
echo done > "$out/DONE"
