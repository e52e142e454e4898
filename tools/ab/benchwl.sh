#!/bin/bash
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bench_other" > "$out/pytest.log" 2>&1
echo done > "$out/DONE"
