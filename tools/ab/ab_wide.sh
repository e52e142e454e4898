#!/bin/bash
# wide K4 drain A/B: parity tests on the new build, then base/new alternating timings
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/ab_wide
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_reduce_side.py tests/test_range_sketch.py -m gpu -x -q --timeout 120 --timeout-method thread -k "terasort or wide or range or sorted or c4" > "$out/pytest.log" 2>&1
for r in 1 2; do
  for v in base new; do
    lib=sparkucx_amd/libsgx.so; [ $v = base ] && lib=tools/ab/libsgx_base.so
    timeout -k 10 120 python -u tools/ab_run.py $lib prof_configs --configs terasort:1024 --iters 5 > "$out/map_${v}_$r.jsonl" 2>&1
    timeout -k 10 120 python -u tools/ab_run.py $lib prof_reduce --cases sorted:terasort --iters 3 > "$out/red_${v}_$r.jsonl" 2>&1
  done
done
echo done > "$out/DONE"
