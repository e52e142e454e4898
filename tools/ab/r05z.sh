#!/bin/bash
# The 16 B K4 with nontemporal tile loads (cntl) vs the tree: C1, 4 alternations.
tag=${1:-r05z}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
C="--no-cpu-baseline --no-live-pmc"
for i in 1 2 3 4; do
  timeout -k 10 180 python -u bench.py $C > "$out/c1_tree_$i.log" 2>&1 || fail "c1" "$out/c1_tree_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_cntl.so bench $C > "$out/c1_cntl_$i.log" 2>&1 || fail "c1 cntl" "$out/c1_cntl_$i.log"
done
timeout -k 10 180 python -u bench.py --workload c3 $C > "$out/c3_tree.log" 2>&1 || fail "c3" "$out/c3_tree.log"
timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_cntl.so bench --workload c3 $C > "$out/c3_cntl.log" 2>&1 || fail "c3 cntl" "$out/c3_cntl.log"
timeout -k 10 180 python -u bench.py --batches 64 $C > "$out/b64_tree.log" 2>&1 || fail "b64" "$out/b64_tree.log"
timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_cntl.so bench --batches 64 $C > "$out/b64_cntl.log" 2>&1 || fail "b64 cntl" "$out/b64_cntl.log"
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
echo done > "$out/DONE"
