#!/bin/bash
# kernel trace of the sorted reads (bucket path and digit passes)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=$GRAFT_REPO_ROOT/gpurun_out/r03r
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt -o run -- \
  python3 tools/prof_reduce.py --cases sorted:uniform,sorted:terasort > $o/kt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt_nb -o run -- \
  python3 tools/prof_reduce.py --flags 64 --cases sorted:uniform,sorted:terasort > $o/kt_nb.log 2>&1
echo ALLDONE
