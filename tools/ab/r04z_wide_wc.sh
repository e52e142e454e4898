#!/bin/bash
# Write-combining TeraSort K4 (k_scatter_wide_wc, padded writes): parity tests first, then the
# C4 bench against the previous kernel (libsgx_wwc0.so: -DSGX_WIDE_WC=0), then PMC passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04z
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_padded.py tests/test_gpu_parity.py tests/test_range_sketch.py tests/test_reduce_side.py \
    -k "terasort or range or wide or c4 or padded or bytes10 or TeraSort" > gpurun_out/r04z/pytest.log 2>&1 \
    || { tail -40 gpurun_out/r04z/pytest.log; exit 1; }
tail -1 gpurun_out/r04z/pytest.log
B="--workload c4 --no-cpu-baseline --no-live-pmc"
for i in 1 2; do
  timeout -k 10 180 python -u bench.py $B > gpurun_out/r04z/wc_$i.log 2>&1 || exit 1
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_wwc0.so bench $B > gpurun_out/r04z/w2_$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r04z/w*_*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f, d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
bash tools/gpu_prof.sh r04z/prof_ts2 --record-bytes 100 --records 42949672 || exit 1
