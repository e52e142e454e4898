#!/bin/bash
# Histogram geometry A/B (SGX_HIST_VARIANT, see launch_hist) on C1, correct output checked.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  for v in 0 2 3 4 5 6; do
    echo -n "hist_variant=$v: " >> "$out/ab.log"
    SGX_HIST_VARIANT=$v timeout -k 10 120 python3 tools/prof_map.py --iters 6 2>&1 | grep -v amdgpu.ids | tail -1 >> "$out/ab.log"
  done
done
echo done > "$out/DONE"
