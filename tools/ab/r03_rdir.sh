#!/bin/bash
# range-bounds directory: parity of the range paths on the tree, then TeraSort A/B and stamps
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03_rdir; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_reduce_side.py tests/test_range_sketch.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "range or terasort or wide or directory or golden or c4 or sorted or sketch or bounds" > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for r in 1 2 3; do
  for v in base tree; do
    lib=sparkucx_amd/libsgx.so; [ $v = base ] && lib=tools/ab/libsgx_base.so
    timeout -k 10 200 python -u tools/ab_run.py $lib prof_configs --configs terasort:1024 --iters 5 | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> $o/timings.jsonl
  done
done
timeout -k 10 200 python -u tools/ab_run.py tools/ab/libsgx_stamps.so wc_stamps --record-bytes 100 --partitions 1024 > $o/stamps.jsonl
cat $o/timings.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print(j['variant'], j['rep'], 'hist', j['hist_ms'], 'scatter', j['scatter_ms'], j['map_side_GBs'])"
cat $o/stamps.jsonl
