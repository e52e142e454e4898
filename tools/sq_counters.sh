#!/bin/bash
# SQ / LDS counter passes over the C1 map-side write (measurement tool).  Each pass is its
# own rocprofv3 run with --pmc only (no trace domains), program directly after --.
# usage: bash tools/sq_counters.sh <outdir> [prof_map.py args...]
set -e
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES"
P3="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for p in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o run -- python3 tools/prof_map.py "$@" > "$out/p$i.log" 2>&1
done
