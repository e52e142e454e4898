#!/bin/bash
# Pipelined map side (SGX_PIPELINE=1: next map's lean histogram + scan on their own stream,
# overlapping the current map's K4): parity suite in that mode, then bench A/B.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SGX_PIPELINE=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/pytest_pipe.log" 2>&1
for rep in 1 2; do
  for p in 0 1; do
    SGX_PIPELINE=$p timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>&1 \
      | grep -v amdgpu.ids > "$out/bench_p${p}_$rep.log"
  done
done
echo done > "$out/DONE"
