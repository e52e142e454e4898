#!/bin/bash
# two-read wide K4 (SGX_FLAG_WIDE_TWO_READ) vs the staged one: parity tests, then map-side timings
# (the in-tree library: DRB 8, one workgroup per CU; tools/ab/libsgx_w3d4.so: DRB 4, two per CU)
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wide or terasort or c4" > "$out/pytest.log" 2>&1
for r in 1 2; do
  for f in 0 32; do
    timeout -k 10 120 python -u tools/prof_map.py --record-bytes 100 --records 33554432 --partitions 1024 --iters 5 --flags $f > "$out/map_f${f}_$r.txt" 2>&1
  done
  timeout -k 10 120 python -u tools/ab_run.py tools/ab/libsgx_w3d4.so prof_map --record-bytes 100 --records 33554432 --partitions 1024 --iters 5 --flags 32 > "$out/map_d4_$r.txt" 2>&1
done
echo done > "$out/DONE"
