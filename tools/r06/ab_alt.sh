#!/bin/bash
# Round 6: consecutive padded writes on alternating streams -- the GPU suite, then same-box
# alternating A/B against the tree without it (noalt): C1, C4, the self-exchange line.
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1 || { tail -40 "$out/pytest_gpu.log"; exit 1; }
tail -2 "$out/pytest_gpu.log"
run() {  # run <lib> <log> <bench args...>
  local lib=$1 log=$2; shift 2
  if [ "$lib" = tree ]; then
    timeout -k 10 300 python -u bench.py "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  else
    timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_$lib.so bench "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  fi
  grep '^{' "$out/$log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$log', j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_map_side']['frac'], j['stages_ms_per_step'])"
}
for rep in 1 2 3; do
  for lib in tree noalt; do run $lib c1_${lib}_$rep.log --no-cpu-baseline --no-live-pmc --steps 40; done
done
for rep in 1 2; do
  for lib in tree noalt; do run $lib c4_${lib}_$rep.log --workload c4 --no-cpu-baseline --no-live-pmc --steps 40; done
done
for lib in tree noalt; do run $lib selfx_${lib}.log --self-exchange --no-cpu-baseline --no-live-pmc --steps 20; done
echo done > "$out/DONE"
