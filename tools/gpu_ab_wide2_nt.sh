#!/bin/bash
# TeraSort 100 B K4 (k_scatter_wide2) A/B: plain vs nontemporal drain stores; wide parity first.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SGX_WIDE2_NT=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
  --timeout-method thread -k "wide or terasort or range" > "$out/pytest_nt.log" 2>&1
for rep in 1 2 3; do
  for v in 0 1; do
    echo -n "nt=$v: " >> "$out/ab.log"
    SGX_WIDE2_NT=$v timeout -k 10 200 python3 tools/prof_configs.py --configs terasort:1024 --iters 5 2>&1 \
      | grep -v amdgpu.ids | tail -1 >> "$out/ab.log"
  done
done
echo done > "$out/DONE"
