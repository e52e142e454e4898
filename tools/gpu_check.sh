#!/bin/bash
# One GPU-box session: parity tests, the bench line, a kernel-trace profile of the bench's
# workload and A/B probes.  Every GPU step has its own time limit; steps are chained and the
# first failure ends the script.
#   usage (repo root on the box): bash tools/gpu_check.sh <tag> [skip-tests]
set -e
tag=${1:-run}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread \
    > "$out/pytest_gpu.log" 2>&1
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$out/bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$out/prof.log" 2>&1
timeout -k 10 300 python3 -u tools/multimap_probe.py > "$out/multimap.log" 2>&1
timeout -k 10 600 python3 -u tools/sweep_scatter.py --rounds 3 --iters 3 \
  --variants 0:0:0,256:12:10,256:16:7,256:8:8,256:4:16,512:4:16 > "$out/sweep.log" 2>&1
if [ -x tools/bin/mb_scatter ]; then timeout -k 10 300 tools/bin/mb_scatter > "$out/mb_scatter.log" 2>&1; fi
echo done > "$out/DONE"
