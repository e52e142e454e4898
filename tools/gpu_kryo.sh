#!/bin/bash
# Kryo framing: GPU parity, then the bench with the Kryo serializer and
# a kernel trace of it.   usage: bash tools/gpu_kryo.sh <tag>
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kryo.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$out/pytest_kryo.log" 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u bench.py --serializer kryo --no-cpu-baseline > "$out/bench_kryo.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 bench.py --serializer kryo --steps 5 --warmup 2 --no-cpu-baseline > "$out/kt.log" 2>&1
echo done > "$out/DONE"
