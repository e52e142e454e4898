#!/bin/bash
# LZ4 framing on the GPU: parity tests first, then the rest of the GPU suite.
#   usage: bash tools/gpu_lz4.sh <tag>
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_lz4.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$out/pytest_lz4.log" 2>&1
if [ -f tools/prof_lz4.py ]; then
  timeout -k 10 300 python -u tools/prof_lz4.py > "$out/lz4_bench.log" 2>&1
fi
echo done > "$out/DONE"
