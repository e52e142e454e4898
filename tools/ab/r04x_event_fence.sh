#!/bin/bash
# Stage events without the system-scope fence (default now) vs with it (libsgx_fence.so):
# C1 bench lines alternated, then a kernel trace of the new default for the inter-kernel gaps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04x
B="--no-cpu-baseline --no-live-pmc"
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py $B > gpurun_out/r04x/nofence_$i.log 2>&1 || exit 1
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_fence.so bench $B > gpurun_out/r04x/fence_$i.log 2>&1 || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04x/kt -o run -- python3 bench.py --steps 10 $B \
    > gpurun_out/r04x/kt.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_padded.py tests/test_gpu_parity.py \
    > gpurun_out/r04x/pytest.log 2>&1 || { tail -20 gpurun_out/r04x/pytest.log; exit 1; }
tail -1 gpurun_out/r04x/pytest.log
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r04x/*fence_*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
