#!/bin/bash
# C1 Kryo+LZ4 bench (compress + reduce-side decode of a 2^28-record map), base vs new library
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base new; do
  lib=sparkucx_amd/libsgx.so; [ $v = base ] && lib=tools/ab/libsgx_base.so
  timeout -k 10 300 python -u -c "
import sys; sys.argv=['bench.py','--serializer','kryo','--compress','--steps','2','--warmup','1','--no-cpu-baseline']
import sparkucx_amd._lib as L; L.LIB_PATH='$lib'
import runpy; runpy.run_path('bench.py', run_name='__main__')" > "$out/bench_$v.log" 2>&1
done
echo done > "$out/DONE"
