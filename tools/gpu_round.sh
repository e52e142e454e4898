#!/bin/bash
# Round evidence on one GPU: the full GPU parity suite, smoke(), the bench line (C1 with the
# CPU baseline), and rocprofv3 on the SAME bench command: kernel trace + stats, then one
# FETCH_SIZE pass and one WRITE_SIZE pass (--pmc only, separate runs).
#   usage: bash tools/gpu_round.sh <tag> [skip-tests]
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$out/pytest_gpu.log" 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
fi
timeout -k 10 300 python -u bench.py > "$out/bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$out/kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$out/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$out/write.log" 2>&1
echo done > "$out/DONE"
