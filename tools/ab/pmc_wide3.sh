#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the two-read wide K4 (does the second read hit the caches?)
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
  python3 tools/prof_map.py --record-bytes 100 --records 33554432 --partitions 1024 --iters 2 --flags 32 > "$out/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
  python3 tools/prof_map.py --record-bytes 100 --records 33554432 --partitions 1024 --iters 2 --flags 32 > "$out/write.log" 2>&1
echo done > "$out/DONE"
