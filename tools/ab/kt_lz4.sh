#!/bin/bash
# Kernel-trace stats of the C1 Kryo+LZ4 bench (compress + decode kernels)
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 bench.py --serializer kryo --compress --steps 2 --warmup 1 --no-cpu-baseline > "$out/bench.log" 2>&1
echo done > "$out/DONE"
