#!/bin/bash
# Reduce-side A/B: test_reduce_side.py on each non-base variant, then alternating
# tools/prof_reduce.py timings.   bash tools/ab/r03_reduce_ab.sh <outtag> "<variants>" [cases]
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
cases=${3:-sorted:uniform,sorted:terasort,group:uniform,sum:zipf}
lib_of() { [ "$1" = tree ] && echo sparkucx_amd/libsgx.so || echo tools/ab/libsgx_$1.so; }
for v in $2; do
  [ "$v" = base ] && continue
  timeout -k 10 400 python -u -m pytest tests/test_reduce_side.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    --sgx-lib $(lib_of $v) > $o/pytest_red_$v.log 2>&1 || { tail -30 $o/pytest_red_$v.log; exit 1; }
  tail -1 $o/pytest_red_$v.log
done
for r in 1 2 3; do
  for v in $2; do
    timeout -k 10 200 python -u tools/ab_run.py $(lib_of $v) prof_reduce --cases $cases | grep '^{' | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> $o/reduce.jsonl
  done
done
python3 - $o/reduce.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j['case'], j['variant'])].append(j['device_ms'])
for k in sorted(d): print(k, 'device_ms', sorted(d[k]))
PY
