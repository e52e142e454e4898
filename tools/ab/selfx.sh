#!/bin/bash
# one-GPU rehearsal of the multi-GPU step: bench --self-exchange, plus its kernel trace
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python -u bench.py --self-exchange --steps 10 --warmup 3 --no-cpu-baseline > "$out/bench_selfx.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 bench.py --self-exchange --steps 10 --warmup 3 --no-cpu-baseline > "$out/kt.log" 2>&1
python3 tools/overlap_from_trace.py "$out/kt/run_kernel_trace.csv" > "$out/overlap.jsonl" 2>&1 || true
echo done > "$out/DONE"
