#!/bin/bash
# SQ counter passes over the Kryo serializer / decoder (bench --serializer kryo, 2^26 records)
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES"
i=0
for p in "$P1" "$P2"; do
  i=$((i+1))
  mkdir -p "$out/p$i"
  timeout -s KILL 150 rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o run -- python3 bench.py --serializer kryo --records 67108864 --steps 1 --warmup 1 --no-cpu-baseline > "$out/p$i.log" 2>&1
done
echo done > "$out/DONE"
