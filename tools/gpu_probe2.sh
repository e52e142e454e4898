#!/bin/bash
# Store-pattern floor (aligned vs unaligned runs) + SQ counters of the default K4.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 tools/bin/mb_scatter > "$out/mb_scatter.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 tools/prof_map.py --iters 3 > "$out/kt.log" 2>&1
bash tools/sq_counters.sh "$out/sq" --iters 2
echo done > "$out/DONE"
