#!/bin/bash
# 16 B RangePartitioner through the write-combining K4: parity of the range paths, then A/B
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03_range16; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_reduce_side.py tests/test_threads_streaming_combine.py tests/test_exchange_multirank.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "range or directory or golden or kernel_choices or sorted or combine" > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for r in 1 2 3; do
  for v in base tree; do
    lib=sparkucx_amd/libsgx.so; [ $v = base ] && lib=tools/ab/libsgx_base.so
    timeout -k 10 200 python -u tools/ab_run.py $lib prof_configs --configs range:1024,range:200,range:64 --iters 5 | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> $o/timings.jsonl
  done
done
python3 - $o/timings.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j['config'], j['variant'])].append(j)
for k in sorted(d): print(k, 'scatter', [x['scatter_ms'] for x in d[k]], 'hist', [x['hist_ms'] for x in d[k]], [x['map_side_GBs'] for x in d[k]])
PY
