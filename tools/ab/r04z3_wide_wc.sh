#!/bin/bash
# Final TeraSort K4 defaults (write-combining padded + two-pass K4, drain unrolled x2): the
# GPU tests that touch 100 B records, then C4 padded / two-pass against the previous kernel
# (wwc0), then the 4.3 GB PMC passes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04z3
K='terasort or range or wide or c4 or padded or bytes10 or TeraSort or exchange'
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_padded.py \
    tests/test_gpu_parity.py tests/test_range_sketch.py tests/test_reduce_side.py tests/test_exchange_multirank.py -k "$K" \
    > gpurun_out/r04z3/pytest.log 2>&1 || { tail -40 gpurun_out/r04z3/pytest.log; exit 1; }
tail -1 gpurun_out/r04z3/pytest.log
B="--workload c4 --no-cpu-baseline --no-live-pmc"
for i in 1 2; do
  timeout -k 10 180 python -u bench.py $B > gpurun_out/r04z3/c4_wc_$i.log 2>&1 || exit 1
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_wwc0.so bench $B > gpurun_out/r04z3/c4_w2_$i.log 2>&1 || exit 1
  timeout -k 10 180 python -u bench.py $B --no-padded > gpurun_out/r04z3/c4tp_wc_$i.log 2>&1 || exit 1
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_wwc0.so bench $B --no-padded > gpurun_out/r04z3/c4tp_w2_$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r04z3/c4*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f, d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
bash tools/gpu_prof.sh r04z3/prof_ts --record-bytes 100 --records 42949672 || exit 1
bash tools/gpu_prof.sh r04z3/prof_ts_twopass --record-bytes 100 --records 42949672 --flags 256 || exit 1
