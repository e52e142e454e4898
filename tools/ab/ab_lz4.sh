#!/bin/bash
# LZ4 decoder A/B: LZ4 GPU tests on the new build, then base/new alternating timings
set -e
tag=${1:-ab_lz4}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_lz4.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
for r in 1 2; do
  for v in base new; do
    lib=sparkucx_amd/libsgx.so; [ $v = base ] && lib=tools/ab/libsgx_base.so
    timeout -k 10 180 python -u tools/ab_run.py $lib prof_lz4 --iters 3 > "$out/lz4_${v}_$r.jsonl" 2>&1
  done
done
echo done > "$out/DONE"
