#!/bin/bash
# Round-6 baseline on one MI355X: default bench line, and a kernel trace of it.
# usage: bash tools/r06/base.sh <tag>
tag=${1:-r06a}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/bench.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-live-pmc > "$out/bench2.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 bench.py --steps 10 --no-cpu-baseline --no-live-pmc > "$out/bench_kt.log" 2>&1 || exit $?
echo done > "$out/DONE"
