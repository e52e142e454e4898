#!/bin/bash
for rep in 1 2; do for nt in ${NTS:-0 1 2 3}; do
  echo -n "nt=$nt: "; SGX_SCATTER_NT=$nt timeout -k 10 120 python3 tools/sweep_scatter.py --variants 256:8:16 --rounds 2 --iters 3 2>&1 | grep -v amdgpu.ids | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['scatter_med'], d['hist_med'])" || exit 1
done; done
