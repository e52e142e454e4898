#!/bin/bash
# TeraSort K4 variants at 4.3 GB (42,949,672 records), alternated on one box: the previous
# kernel (wwc0: -DSGX_WIDE_WC=0), the write-combining kernel (default), with an LDS-only
# barrier at the tile landing (wwclb), with its drain unrolled x2 (wwcu2); two-pass legs:
# wwc0 vs wwctp (write-combining two-pass K4 + LDS-only landing barrier).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04z2
K='terasort or range or wide or c4 or padded or bytes10 or TeraSort'
TS="tests/test_padded.py tests/test_gpu_parity.py tests/test_range_sketch.py tests/test_reduce_side.py"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $TS -k "$K" \
    > gpurun_out/r04z2/pytest.log 2>&1 || { tail -40 gpurun_out/r04z2/pytest.log; exit 1; }
tail -1 gpurun_out/r04z2/pytest.log
timeout -k 10 600 python -u -c "
import sys, sparkucx_amd._lib as L, pytest
L.LIB_PATH = 'tools/ab/libsgx_wwctp.so'
sys.exit(pytest.main(['-x', '-q', '--timeout', '200', '--timeout-method', 'thread', '-m', 'gpu', '-k', '$K'] + '$TS'.split()))
" > gpurun_out/r04z2/pytest_wwctp.log 2>&1 || { tail -40 gpurun_out/r04z2/pytest_wwctp.log; exit 1; }
tail -1 gpurun_out/r04z2/pytest_wwctp.log
B="--workload c4 --records 42949672 --steps 10 --no-cpu-baseline --no-live-pmc"
run() {  # run <variant> <log> [extra bench args]
  local v=$1 log=$2; shift 2
  if [ $v = default ]; then cmd="bench.py"; else cmd="tools/ab_run.py tools/ab/libsgx_$v.so bench"; fi
  timeout -k 10 180 python -u $cmd $B "$@" > gpurun_out/r04z2/$log.log 2>&1
}
for i in 1 2; do
  for v in wwc0 default wwclb wwcu2; do run $v ${v}_$i || exit 1; done
  for v in wwc0 wwctp; do run $v twopass_${v}_$i --no-padded || exit 1; done
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r04z2/*_*.log")):
    if "pytest" in f: continue
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f, d["value"], d["ms_per_step"], d["stages_ms_per_step"])
PY
