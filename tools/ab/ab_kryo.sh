#!/bin/bash
# Kryo A/B: Kryo GPU tests on the new build, then the Kryo bench (serialize + decode timings)
# alternating base/new
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kryo.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
for r in 1 2; do
  for v in base new; do
    lib=sparkucx_amd/libsgx.so; [ $v = base ] && lib=tools/ab/libsgx_base.so
    timeout -k 10 240 python -u -c "
import sys; sys.argv=['bench.py','--serializer','kryo','--steps','10','--no-cpu-baseline']
import sparkucx_amd._lib as L; L.LIB_PATH='$lib'
import runpy; runpy.run_path('bench.py', run_name='__main__')" > "$out/bench_${v}_$r.log" 2>&1
  done
done
echo done > "$out/DONE"
