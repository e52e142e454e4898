#!/bin/bash
# LZ4 decode variants at three scales: prof_lz4 (2^24 records) and bench --compress at 2^26, 2^28 records
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base global ring0; do
  lib=tools/ab/libsgx_$v.so
  timeout -k 10 180 python -u tools/ab_run.py $lib prof_lz4 --iters 3 > "$out/lz4_$v.jsonl" 2>&1
  for rec in 67108864 268435456; do
    timeout -k 10 300 python -u -c "
import sys; sys.argv=['bench.py','--serializer','kryo','--compress','--steps','2','--warmup','1','--no-cpu-baseline','--records','$rec']
import sparkucx_amd._lib as L; L.LIB_PATH='$lib'
import runpy; runpy.run_path('bench.py', run_name='__main__')" > "$out/bench_${v}_$rec.log" 2>&1
  done
done
echo done > "$out/DONE"
