#!/bin/bash
# Parity subset, A/B sweep, and the rocprofv3 evidence for the bench's workload:
# kernel trace + stats, one FETCH_SIZE pass, one WRITE_SIZE pass (separate runs, --pmc
# only), SQ counter passes.  usage: bash tools/gpu_prof.sh <tag> "<sweep variants>"
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "carry_pressure or random_sizes or golden or variants" > "$out/pytest.log" 2>&1
if [ -n "$2" ]; then
  timeout -k 10 600 python3 -u tools/sweep_scatter.py --rounds 3 --iters 3 --variants "$2" > "$out/sweep.log" 2>&1
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 tools/prof_map.py --iters 5 > "$out/kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
  python3 tools/prof_map.py --iters 2 > "$out/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
  python3 tools/prof_map.py --iters 2 > "$out/write.log" 2>&1
bash tools/sq_counters.sh "$out/sq" --iters 2
echo done > "$out/DONE"
