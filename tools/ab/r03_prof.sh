#!/bin/bash
# Round-3 rocprofv3 evidence: the default bench command under --kernel-trace --stats, the
# C1 / C3 map sides (kernel trace + FETCH_SIZE / WRITE_SIZE passes, tools/gpu_prof.sh; C3
# with the two-level split and with the single lane-ordered pass), and the reduce-side
# sorted read with and without the bucket path.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=$GRAFT_REPO_ROOT/gpurun_out/r03p
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/bench_kt -o run -- \
  python3 bench.py --no-cpu-baseline > $o/bench_kt.log 2>&1
bash tools/gpu_prof.sh r03p/c1
bash tools/gpu_prof.sh r03p/u4096 --partitions 4096
bash tools/gpu_prof.sh r03p/z4096 --dist zipf --partitions 4096
bash tools/gpu_prof.sh r03p/u4096_nosplit --partitions 4096 --flags 32
timeout -k 10 300 python3 tools/prof_reduce.py --cases sorted:uniform,group:uniform,sum:zipf,sorted:zipf,sorted:terasort > $o/reduce.jsonl 2>&1
timeout -k 10 300 python3 tools/prof_reduce.py --flags 64 --cases sorted:uniform,sorted:terasort > $o/reduce_nobucket.jsonl 2>&1
echo ALLDONE
