#!/bin/bash
# rocprofv3 evidence for one map-side workload (tools/prof_map.py): kernel trace + stats,
# then one FETCH_SIZE pass and one WRITE_SIZE pass (separate runs, --pmc only, program
# directly after --).  Summarise afterwards on the host with tools/summarize_prof.py.
# usage: bash tools/gpu_prof.sh <tag> [prof_map.py args...]
set -e
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 tools/prof_map.py --iters 5 "$@" > "$out/kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
  python3 tools/prof_map.py --iters 2 "$@" > "$out/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
  python3 tools/prof_map.py --iters 2 "$@" > "$out/write.log" 2>&1
echo done > "$out/DONE"
