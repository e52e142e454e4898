#!/bin/bash
# Round 6: XCD-aware chunk mapping of the 16 B write-combining K4 (xcd1) against the tree (base);
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
line() {  # line <lib> <log> <args...>
  local lib=$1 log=$2; shift 2
  timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_$lib.so bench --no-cpu-baseline --no-live-pmc --steps 40 "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  grep '^{' "$out/$log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$log', j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_map_side']['frac'])"
}
for rep in 1 2 3 4; do
  for lib in base xcd1; do line $lib c1_${lib}_$rep.log; done
done
for rep in 1 2; do
  for lib in base xcd1; do line $lib c3_${lib}_$rep.log --workload c3; done
done
echo done > "$out/DONE"
