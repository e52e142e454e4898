#!/bin/bash
# A/B of the write-combining K4's store/wait variants (all produce correct output):
#   SGX_WC_DIAG=4 conditional stores (compiler waits vmcnt(0) per tile), 0 branch-free
#   junk-line stores, 8 branch-free stores + asm loads waited with vmcnt(SI).
# Parity suite first with the variant under test, then timings (C1).
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for d in ${VARIANTS:-0}; do
  SGX_WC_DIAG=$d timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$out/pytest_d$d.log" 2>&1
done
for rep in 1 2 3; do
  for d in ${AB:-16 0}; do
    echo -n "wc_diag=$d: " >> "$out/ab.log"
    SGX_WC_DIAG=$d timeout -k 10 120 python3 tools/prof_map.py --iters 6 2>&1 | grep -v amdgpu.ids | tail -1 >> "$out/ab.log"
  done
done
echo done > "$out/DONE"
