#!/bin/bash
# Round validation on one MI355X: the GPU suite, smoke, the default bench, the Kryo and
# Kryo+LZ4 bench variants, and a rocprofv3 kernel trace of the default bench.
# usage: bash tools/gpu_validate.sh <tag>
set -e
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 240 python -u bench.py > "$out/bench.log" 2>&1
timeout -k 10 240 python -u bench.py --serializer kryo --steps 10 --no-cpu-baseline > "$out/bench_kryo.log" 2>&1
timeout -k 10 300 python -u bench.py --serializer kryo --compress --steps 5 --warmup 2 --no-cpu-baseline > "$out/bench_kryo_lz4.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 bench.py --steps 10 --no-cpu-baseline > "$out/bench_kt.log" 2>&1
echo done > "$out/DONE"
