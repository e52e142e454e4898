#!/bin/bash
# SQ counter passes over prof_lz4 (base library and the current one)
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES"
P3="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE GRBM_COUNT"
for v in base new; do
  lib=sparkucx_amd/libsgx.so; [ $v = base ] && lib=tools/ab/libsgx_base.so
  i=0; mkdir -p "$out/$v"
  for p in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$out/$v/p$i" -o run -- python3 tools/ab_run.py $lib prof_lz4 --iters 1 > "$out/$v/p$i.log" 2>&1
  done
done
echo done > "$out/DONE"
