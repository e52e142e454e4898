#!/bin/bash
# A/B: LDS peer-table ranking vs ballots-only, default (DMA) kernel and forced 8x16 generic.
for rep in 1 2; do
for nt in 0 1; do
  echo -n "no_table=$nt default: "; SGX_NO_PEER_TABLE=$nt timeout -k 10 120 python3 tools/prof_map.py --iters 8 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  echo -n "no_table=$nt 8x16:    "; SGX_NO_PEER_TABLE=$nt SGX_SCATTER_DIAG=0 timeout -k 10 120 python3 tools/sweep_scatter.py --variants 256:8:16 --rounds 2 --iters 3 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
done
