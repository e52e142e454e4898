#!/bin/bash
# Round 6: same-box A/B of the C3 front on its own stream (tree vs nopre), of the pinned-staged
# host reads (tree vs nostage: prof_reduce's host-array reads), and the host-batch writer line.
# usage: bash tools/r06/ab_c3.sh <tag>
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # run <lib> <log> <tool> <args...>
  local lib=$1 log=$2 tool=$3; shift 3
  if [ "$lib" = tree ]; then
    timeout -k 10 300 python -u $tool.py "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  else
    timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_$lib.so $(basename $tool) "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  fi
}
for rep in 1 2 3; do
  for lib in tree nopre; do
    run $lib c3_${lib}_$rep.log bench --workload c3 --no-cpu-baseline --no-live-pmc --steps 20
    grep '^{' "$out/c3_${lib}_$rep.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('c3', '$lib', $rep, j['value'], j['ms_per_step'], j['roofline_map_side']['frac'], j['stages_ms_per_step'])"
  done
done
for rep in 1 2; do
  for lib in tree nostage; do
    run $lib red_${lib}_$rep.log tools/prof_reduce --records 67108864 --iters 2 --cases group:uniform,sum:zipf
    grep -h '^{' "$out/red_${lib}_$rep.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('red', '$lib', $rep, d['case'], d['device_ms'], d['wall_ms_host_arrays'], d['wall_ms_host_arrays_mapped'])"
  done
done
run tree b64host.log bench --batches 64 --host-batches --steps 5 --warmup 1 --no-cpu-baseline --no-live-pmc
grep '^{' "$out/b64host.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('b64host', j['value'], j['ms_per_step'], j.get('host_ingest'))"
echo done > "$out/DONE"
