#!/bin/bash
# A/B: chunked staged K4 (default) vs chained look-back K4 geometries.
for rep in 1 2; do
  echo -n "chunked 8x16: "; timeout -k 10 120 python3 tools/prof_map.py --iters 8 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  for c in 816 416 808 1607; do
    echo -n "chain $c:    "; SGX_SCATTER_CHAIN=$c timeout -k 10 120 python3 tools/prof_map.py --iters 8 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
