#!/bin/bash
# Round-3 K4 A/B: parity subset on each variant library, then alternating timings.
#   bash tools/ab/r03_ab.sh <outtag> "<variant tags>" [configs]
# variants are tools/ab/libsgx_<tag>.so; "tree" = sparkucx_amd/libsgx.so
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; mkdir -p $o
vars="$2"; cfgs=${3:-uniform:1024,zipf:1024,uniform:200,uniform:4096}
lib_of() { [ "$1" = tree ] && echo sparkucx_amd/libsgx.so || echo tools/ab/libsgx_$1.so; }
for v in $vars; do
  [ "$v" = base ] && continue
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    --sgx-lib $(lib_of $v) -k "golden or hash_random or chunking or carry_pressure or two_level or full_c1 or zipf or kernel_choices or large_r or collisions or one_partition" > $o/pytest_$v.log 2>&1 || { tail -30 $o/pytest_$v.log; exit 1; }
  tail -1 $o/pytest_$v.log
  timeout -k 10 400 python -u -m pytest tests/test_reduce_side.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    --sgx-lib $(lib_of $v) > $o/pytest_red_$v.log 2>&1 || { tail -30 $o/pytest_red_$v.log; exit 1; }
  tail -1 $o/pytest_red_$v.log
done
for r in 1 2 3; do
  for v in $vars; do
    timeout -k 10 200 python -u tools/ab_run.py $(lib_of $v) prof_configs --configs $cfgs --iters 5 | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> $o/timings.jsonl
    [ -n "$REDUCE" ] && timeout -k 10 200 python -u tools/ab_run.py $(lib_of $v) prof_reduce --cases $REDUCE | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> $o/reduce.jsonl
  done
done
python3 - $o/timings.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); d[(j['config'], j['variant'])].append(j)
for k in sorted(d): print(k, 'scatter', [x['scatter_ms'] for x in d[k]], 'hist', [x['hist_ms'] for x in d[k]])
PY
[ -f $o/reduce.jsonl ] && python3 - $o/reduce.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); d[(j['case'], j['variant'])].append(j['device_ms'])
for k in sorted(d): print(k, 'device_ms', d[k])
PY
true
