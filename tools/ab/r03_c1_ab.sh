#!/bin/bash
# C1 K4 A/B with more repetitions: prof_configs uniform:1024 and the default bench line,
# alternating the variant libraries.   bash tools/ab/r03_c1_ab.sh <outtag> "<variants>"
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
lib_of() { [ "$1" = tree ] && echo sparkucx_amd/libsgx.so || echo tools/ab/libsgx_$1.so; }
for r in 1 2 3 4 5 6; do
  for v in $2; do
    timeout -k 10 200 python -u tools/ab_run.py $(lib_of $v) prof_configs --configs uniform:1024 --iters 5 | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> $o/timings.jsonl
  done
done
for r in 1 2; do
  for v in $2; do
    timeout -k 10 200 python -u -c "
import sys; sys.argv=['bench.py','--no-cpu-baseline']
import sparkucx_amd._lib as L; L.LIB_PATH='$(lib_of $v)'
import runpy; runpy.run_path('bench.py', run_name='__main__')" 2>/dev/null | grep '^{' | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> $o/bench.jsonl
  done
done
python3 - $o <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1] + '/timings.jsonl'):
    if l.startswith('{'):
        j = json.loads(l); d[j['variant']].append((j['scatter_ms'], j['hist_ms']))
for k in d: print(k, 'scatter', sorted(x[0] for x in d[k]), 'hist', sorted(x[1] for x in d[k]))
for l in open(sys.argv[1] + '/bench.jsonl'):
    j = json.loads(l); print(j['variant'], j['value'], j['stages_ms_per_step'])
PY
