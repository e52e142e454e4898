#!/bin/bash
# C3-shaped A/B: split (device-gated) vs single pass, uniform and Zipf keys, R = 4096; then
# the sorted-read kernel trace
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03c
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "split or 4096 or kernel_choices or 8192 or 2048" > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for d in zipf uniform; do for f in "" "--no-split"; do
  timeout -k 10 200 python bench.py --workload c3 --dist $d --no-cpu-baseline $f > $o/c3_${d}${f}.log 2>&1
  python -c "
import json; d=json.loads([l for l in open('$o/c3_${d}${f}.log') if l.startswith('{')][0]); print('$d$f', d['value'], d['stages_ms_per_step'])"
done; done
bash tools/ab/r03_prof_reduce.sh
echo ALLDONE
