#!/bin/bash
# LZ4 compressor A/B: the tree's library vs variants (tools/ab/libsgx_<v>.so): LZ4/Kryo GPU
# tests on each variant, then bench.py --serializer kryo --compress (C1) and
# tools/prof_lz4.py, alternating.   bash tools/ab/r03_lz4pf.sh <outtag> "<variants>"
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
lib_of() { [ "$1" = tree ] && echo sparkucx_amd/libsgx.so || echo tools/ab/libsgx_$1.so; }
for v in $2; do
  [ "$v" = base ] && continue
  timeout -k 10 300 python -u -m pytest tests/test_lz4.py tests/test_kryo.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider --sgx-lib $(lib_of $v) > "$out/pytest_$v.log" 2>&1 || { tail -30 "$out/pytest_$v.log"; exit 1; }
  tail -1 "$out/pytest_$v.log"
done
for r in 1 2; do
  for v in $2; do
    timeout -k 10 300 python -u -c "
import sys; sys.argv=['bench.py','--serializer','kryo','--compress','--steps','2','--warmup','1','--no-cpu-baseline']
import sparkucx_amd._lib as L; L.LIB_PATH='$(lib_of $v)'
import runpy; runpy.run_path('bench.py', run_name='__main__')" 2>/dev/null | grep '^{' | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> "$out/bench.jsonl"
    timeout -k 10 300 python -u tools/ab_run.py $(lib_of $v) prof_lz4 --iters 3 | grep '^{' | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> "$out/prof_lz4.jsonl"
  done
done
python3 - "$out" <<'PY'
import json, sys
for l in open(sys.argv[1] + '/bench.jsonl'):
    j = json.loads(l); print(j['variant'], j['rep'], 'value', j['value'], 'compress', j['stages_ms_per_step']['compress'])
for l in open(sys.argv[1] + '/prof_lz4.jsonl'):
    j = json.loads(l); print(j['variant'], j['rep'], j['case'], 'gpu_ms', j['gpu_ms'])
PY
