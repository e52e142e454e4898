#!/bin/bash
# Three-way LZ4 A/B (tools/ab/libsgx_base.so, tools/ab/libsgx_mid.so, the tree's build):
# LZ4 + Kryo GPU tests on the new build, prof_lz4 alternating, C1 Kryo+LZ4 bench each
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_lz4.py tests/test_exchange_multirank.py tests/test_threads_streaming_combine.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
lib_of() { case $1 in base) echo tools/ab/libsgx_base.so;; mid) echo tools/ab/libsgx_mid.so;; *) echo sparkucx_amd/libsgx.so;; esac; }
for r in 1 2; do
  for v in base mid new; do
    timeout -k 10 180 python -u tools/ab_run.py $(lib_of $v) prof_lz4 --iters 3 > "$out/lz4_${v}_$r.jsonl" 2>&1
  done
done
for v in base mid new; do
  timeout -k 10 300 python -u -c "
import sys; sys.argv=['bench.py','--serializer','kryo','--compress','--steps','2','--warmup','1','--no-cpu-baseline']
import sparkucx_amd._lib as L; L.LIB_PATH='$(lib_of $v)'
import runpy; runpy.run_path('bench.py', run_name='__main__')" > "$out/bench_$v.log" 2>&1
done
echo done > "$out/DONE"
