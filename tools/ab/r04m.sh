#!/bin/bash
# Round 4, run m: LZ4 batch-compressor emission variants: lz4lit (HEAD), tree (one emission block per
# sequence), lz4q (short sequences queued, written once per batch), lz4skip (peer shuffles skipped).
set -e
tag=${1:-r04m}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
lib_of() { [ "$1" = tree ] && echo sparkucx_amd/libsgx.so || echo tools/ab/libsgx_$1.so; }
for v in tree lz4q lz4skip; do
  timeout -k 10 300 python -u -m pytest tests/test_lz4.py tests/test_kryo.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider --sgx-lib $(lib_of $v) > "$out/pytest_$v.log" 2>&1 || { tail -30 "$out/pytest_$v.log"; exit 1; }
  tail -1 "$out/pytest_$v.log"
done
for r in 1 2; do
  for v in lz4lit tree lz4q lz4skip; do
    timeout -k 10 300 python -u -c "
import sys; sys.argv=['bench.py','--serializer','kryo','--compress','--steps','2','--warmup','1','--no-cpu-baseline','--no-live-pmc']
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
echo done > "$out/DONE"
