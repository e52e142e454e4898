#!/bin/bash
# TeraSort K4 (k_scatter_wide2) A/B: the wide-record GPU tests on the tree's library, then
# alternating map-side timings (terasort:1024) and the reduce side's TeraSort sort.
#   bash tools/ab/r03_wide_ab.sh <outtag> "<variants>"
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
lib_of() { [ "$1" = tree ] && echo sparkucx_amd/libsgx.so || echo tools/ab/libsgx_$1.so; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_reduce_side.py tests/test_exchange_multirank.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest_tree.log 2>&1 || { tail -30 $o/pytest_tree.log; exit 1; }
tail -1 $o/pytest_tree.log
for r in 1 2 3 4; do
  for v in $2; do
    timeout -k 10 200 python -u tools/ab_run.py $(lib_of $v) prof_configs --configs terasort:1024 --iters 5 | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> $o/timings.jsonl
    timeout -k 10 200 python -u tools/ab_run.py $(lib_of $v) prof_reduce --cases sorted:terasort | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> $o/reduce.jsonl
  done
done
python3 - $o <<'PY'
import json, sys, collections
d = collections.defaultdict(list); r = collections.defaultdict(list)
for l in open(sys.argv[1] + '/timings.jsonl'):
    if l.startswith('{'):
        j = json.loads(l); d[j['variant']].append((j['scatter_ms'], j['hist_ms']))
for l in open(sys.argv[1] + '/reduce.jsonl'):
    if l.startswith('{'):
        j = json.loads(l); r[j['variant']].append(j['device_ms'])
for k in d: print(k, 'scatter', sorted(x[0] for x in d[k]), 'hist', sorted(x[1] for x in d[k]), 'reduce sorted:terasort', sorted(r[k]))
PY
