#!/bin/bash
# Round 6: chunks per map (K4 workgroups) again, now that sub-bins are chunk-major:
# alternating C1 / C4 / C3 lines at 256 (default), 512 and 768 chunks.
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
line() {  # line <log> <args...>
  local log=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-live-pmc --steps 40 "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  grep '^{' "$out/$log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$log', j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_map_side']['frac'])"
}
for rep in 1 2 3; do
  for ch in 256 512 768; do line c1_${ch}_$rep.log --num-chunks $ch; done
done
for rep in 1 2; do
  for ch in 256 512; do line c4_${ch}_$rep.log --workload c4 --num-chunks $ch; done
done
for rep in 1 2; do
  for ch in 256 512; do line c3_${ch}_$rep.log --workload c3 --num-chunks $ch; done
done
echo done > "$out/DONE"
