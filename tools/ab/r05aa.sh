#!/bin/bash
# Re-tune after the nontemporal loads: C1 with held-back drain stores (late1), C4 with an
# LDS-only landing barrier (wls0), vs the tree; 3 alternations each.
tag=${1:-r05aa}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
C="--no-cpu-baseline --no-live-pmc"
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py $C > "$out/c1_tree_$i.log" 2>&1 || fail "c1" "$out/c1_tree_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_late1.so bench $C > "$out/c1_late1_$i.log" 2>&1 || fail "c1 late1" "$out/c1_late1_$i.log"
  timeout -k 10 180 python -u bench.py --workload c4 $C > "$out/c4_tree_$i.log" 2>&1 || fail "c4" "$out/c4_tree_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_wls0.so bench --workload c4 $C > "$out/c4_wls0_$i.log" 2>&1 || fail "c4 wls0" "$out/c4_wls0_$i.log"
done
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
echo done > "$out/DONE"
