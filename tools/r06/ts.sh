#!/bin/bash
# Round 6: TeraSort K4 (active-stream compaction) parity, then C4 bench A/B of engine builds.
# usage: bash tools/r06/ts.sh <tag> <lib>...   (lib "tree" = sparkucx_amd/libsgx.so)
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step $log: rc $rc"; tail -30 "$out/$log"; exit $rc; fi
  [ $rc -eq 1 ] && { echo "step $log: rc 1"; tail -40 "$out/$log"; exit 1; }
  return 0
}
line() { grep '^{' "$out/$1" | python3 -c "
import json,sys
j=json.loads(sys.stdin.read())
print('$1', j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_map_side']['frac'], j['stages_ms_per_step'])" || true; }
step 900 pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_padded.py tests/test_streaming_commit.py tests/test_reduce_side.py tests/test_range_sketch.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "terasort or wide or range or c4"
tail -2 "$out/pytest.log"
step 600 pytest_x.log python -u -m pytest tests/test_exchange_multirank.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "terasort"
tail -2 "$out/pytest_x.log"
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = tree ]; then
      step 200 c4_${lib}_$rep.log python -u bench.py --workload c4 --no-cpu-baseline --no-live-pmc --steps 30
    else
      step 200 c4_${lib}_$rep.log python -u tools/ab_run.py tools/ab/libsgx_$lib.so bench --workload c4 --no-cpu-baseline --no-live-pmc --steps 30
    fi
    line c4_${lib}_$rep.log
  done
done
echo done > "$out/DONE"
