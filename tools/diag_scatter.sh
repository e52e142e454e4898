#!/bin/bash
# Measurement-only ablations of K4 (see sgx_kernels.hip k_scatter16_diag). Output is wrong in modes 1-5.
for m in 0 1 2 3 4 5 0; do
  echo -n "diag=$m "
  SGX_SCATTER_DIAG=$m timeout -k 10 120 python3 tools/prof_map.py --iters 8 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
