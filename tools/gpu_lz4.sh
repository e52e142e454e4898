#!/bin/bash
# LZ4 framing on the GPU: parity tests, then timings and a rocprofv3 kernel trace.
#   usage: bash tools/gpu_lz4.sh <tag>
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_lz4.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$out/pytest_lz4.log" 2>&1
timeout -k 10 300 python -u tools/prof_lz4.py > "$out/lz4_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 tools/prof_lz4.py --iters 2 > "$out/kt.log" 2>&1
echo done > "$out/DONE"
