#!/bin/bash
# Round-5 first measurements on the unchanged round-4 tree:
#  - SQ counters of the TeraSort K4 at C4's per-GPU map size
#  - C1 kernel trace with the engine's stage events of the same launches (item 4)
#  - reduce-side kernel trace + FETCH/WRITE passes at 1 GiB (item 8)
#  - --self-exchange kernel trace (item 7)
set -e
tag=${1:-r05a}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/sq_counters.sh "$out/sq_ts" --record-bytes 100 --records 42949672 --iters 2
bash tools/gpu_prof.sh $tag/prof_c1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/red_kt" -o run -- \
  python3 tools/prof_reduce.py --records 67108864 --iters 3 > "$out/red_kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/red_fetch" -o run -- \
  python3 tools/prof_reduce.py --records 67108864 --iters 1 > "$out/red_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/red_write" -o run -- \
  python3 tools/prof_reduce.py --records 67108864 --iters 1 > "$out/red_write.log" 2>&1
bash tools/ab/selfx.sh $tag/selfx
echo done > "$out/DONE"
