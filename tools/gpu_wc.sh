#!/bin/bash
# Write-combining K4: parity, A/B against the lane-ordered kernel, bench line.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "carry_pressure or random_sizes or golden or variants or geometry" > "$out/pytest_wc.log" 2>&1
timeout -k 10 600 python3 -u tools/sweep_scatter.py --rounds 3 --iters 3 \
  --variants 0:0:0,0:0:0:SGX_SCATTER_WC=0,512:0:0,1024:0:0 > "$out/sweep.log" 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$out/bench.log" 2>&1
echo done > "$out/DONE"
