#!/bin/bash
# A/B of K4 variants on the same box: default (LDS-DMA), staged 8x16, direct-store geometries.
for rep in 1 2; do
  echo -n "default(dma): "; timeout -k 10 120 python3 tools/prof_map.py --iters 8 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  echo -n "staged 8x16:  "; timeout -k 10 120 python3 tools/sweep_scatter.py --variants 256:8:16 --rounds 2 --iters 3 2>&1 | grep -v amdgpu.ids | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['scatter_med'])" || exit 1
  for d in 816 808 804 416 408; do
    echo -n "direct $d:    "; SGX_SCATTER_DIRECT=$d timeout -k 10 120 python3 tools/prof_map.py --iters 8 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
