#!/bin/bash
# Wave- vs lane-per-frame LZ4 decode at a few frame counts (prof_lz4 with and without
# --lane-decode), to place kLaneDecodeMinFrames
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 4194304 16777216; do
  for m in wave lane; do
    extra=""; [ $m = lane ] && extra="--lane-decode"
    timeout -k 10 180 python -u tools/prof_lz4.py --records $n --iters 3 $extra > "$out/${m}_$n.jsonl" 2>&1
  done
done
echo done > "$out/DONE"
