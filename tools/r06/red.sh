#!/bin/bash
# Round 6: reduce-side A/B of engine builds (tools/prof_reduce.py), after its parity tests.
# usage: bash tools/r06/red.sh <tag> <lib>...   (lib "tree" = sparkucx_amd/libsgx.so)
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_reduce_side.py tests/test_read_metrics.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = tree ]; then
      timeout -k 10 300 python -u tools/prof_reduce.py --records 67108864 --iters 5 > "$out/red_${lib}_$rep.log" 2>&1 || exit $?
    else
      timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_$lib.so prof_reduce --records 67108864 --iters 5 > "$out/red_${lib}_$rep.log" 2>&1 || exit $?
    fi
    grep -h '^{' "$out/red_${lib}_$rep.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$lib', $rep, d['case'], d['device_ms'], d['stages_ms'])"
  done
done
echo done > "$out/DONE"
