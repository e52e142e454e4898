#!/bin/bash
# Ablations of the write-combining K4 (measurement only): full, no stores, no loads, neither.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for d in 0 1 2 3; do
    echo -n "wc_diag=$d: " >> "$out/diag.log"
    SGX_WC_DIAG=$d timeout -k 10 120 python3 tools/prof_map.py --iters 6 --diag 2>&1 | grep -v amdgpu.ids | tail -1 >> "$out/diag.log"
  done
done
echo done > "$out/DONE"
