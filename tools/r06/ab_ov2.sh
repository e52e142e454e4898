#!/bin/bash
# Round 6: same-box alternating A/B of overlapping writes (default) against one stream
# (--no-overlap-writes) on the chunk-major tree, C1 and C4, default steps.
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # run <log> <bench args...>
  local log=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  grep '^{' "$out/$log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$log', j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_map_side']['frac'])"
}
for rep in 1 2 3; do
  run c1_ov_$rep.log --no-cpu-baseline --no-live-pmc 
  run c1_one_$rep.log --no-cpu-baseline --no-live-pmc  --no-overlap-writes
done
for rep in 1 2 3; do
  run c1_one_b$rep.log --no-cpu-baseline --no-live-pmc  --no-overlap-writes
  run c1_ov_b$rep.log --no-cpu-baseline --no-live-pmc 
done
for rep in 1 2; do
  run c4_ov_$rep.log --workload c4 --no-cpu-baseline --no-live-pmc 
  run c4_one_$rep.log --workload c4 --no-cpu-baseline --no-live-pmc  --no-overlap-writes
done
echo done > "$out/DONE"
