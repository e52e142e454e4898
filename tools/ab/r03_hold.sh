#!/bin/bash
# wide2 held-back drain stores: parity of the range / wide paths per variant, TeraSort A/B, stamps
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03_hold; mkdir -p $o
lib_of() { [ "$1" = tree ] && echo sparkucx_amd/libsgx.so || echo tools/ab/libsgx_$1.so; }
for v in tree hold4; do
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_reduce_side.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    --sgx-lib $(lib_of $v) -k "range or terasort or wide or directory or c4 or sorted" > $o/pytest_$v.log 2>&1 || { tail -30 $o/pytest_$v.log; exit 1; }
  tail -1 $o/pytest_$v.log
done
for r in 1 2 3; do
  for v in hold0 hold4 tree; do
    timeout -k 10 200 python -u tools/ab_run.py $(lib_of $v) prof_configs --configs terasort:1024 --iters 5 | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> $o/timings.jsonl
  done
done
timeout -k 10 200 python -u tools/ab_run.py tools/ab/libsgx_stamps.so wc_stamps --record-bytes 100 --partitions 1024 > $o/stamps.jsonl
cat $o/timings.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print(j['variant'], j['rep'], 'hist', j['hist_ms'], 'scatter', j['scatter_ms'], j['map_side_GBs'])"
cat $o/stamps.jsonl
