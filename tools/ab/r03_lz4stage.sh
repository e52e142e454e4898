#!/bin/bash
# LZ4 compressor A/B: HEAD (base), early RAW exit only (raw), whole block staged in LDS (tree).
# LZ4 GPU tests on the tree's library first; then bench.py --serializer kryo --compress at C1
# and tools/prof_lz4.py (2^24 records, uniform / low-entropy keys) per library.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_lz4.py tests/test_kryo.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest_lz4.log" 2>&1
for v in base raw tree; do
  lib=sparkucx_amd/libsgx.so; [ $v != tree ] && lib=tools/ab/libsgx_$v.so
  timeout -k 10 300 python -u -c "
import sys; sys.argv=['bench.py','--serializer','kryo','--compress','--steps','2','--warmup','1','--no-cpu-baseline']
import sparkucx_amd._lib as L; L.LIB_PATH='$lib'
import runpy; runpy.run_path('bench.py', run_name='__main__')" > "$out/bench_$v.log" 2>&1
  timeout -k 10 300 python -u -c "
import sys; sys.argv=['prof_lz4.py','--iters','3']
import sparkucx_amd._lib as L; L.LIB_PATH='$lib'
import runpy; runpy.run_path('tools/prof_lz4.py', run_name='__main__')" > "$out/prof_lz4_$v.log" 2>&1
done
echo done > "$out/DONE"
