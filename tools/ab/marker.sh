#!/bin/bash
# roctx ranges of the engine's C-ABI calls beside its kernels (kernel + marker trace, no PMC)
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d "$out/mt" -o run -- \
  python3 bench.py --serializer kryo --compress --records 16777216 --steps 3 --warmup 1 --no-cpu-baseline > "$out/mt.log" 2>&1
echo done > "$out/DONE"
