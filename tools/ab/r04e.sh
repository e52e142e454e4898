#!/bin/bash
# Round 4, run e: LZ4 compressor variants (lz4base: round 3; lz4fp: probe-byte settling;
# lz4shfl: settling + candidate load before the ballots, peer bytes by shuffle; tree: the
# multi-sequence batches of lz4_compress_batch), and TeraSort K4 with nontemporal tile loads
# (widentl) against the tree, two-pass and padded.
set -e
tag=${1:-r04e}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
lib_of() { [ "$1" = tree ] && echo sparkucx_amd/libsgx.so || echo tools/ab/libsgx_$1.so; }
for v in tree lz4fp lz4shfl; do
  timeout -k 10 300 python -u -m pytest tests/test_lz4.py tests/test_kryo.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider --sgx-lib $(lib_of $v) > "$out/pytest_$v.log" 2>&1 || { tail -30 "$out/pytest_$v.log"; exit 1; }
  tail -1 "$out/pytest_$v.log"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_padded.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider --sgx-lib $(lib_of widentl) -k "terasort or wide or c4" > "$out/pytest_widentl.log" 2>&1 || { tail -30 "$out/pytest_widentl.log"; exit 1; }
tail -1 "$out/pytest_widentl.log"
for r in 1 2; do
  for v in lz4base lz4fp lz4shfl tree; do
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
for r in 1 2; do
  for v in tree widentl; do
    for f in 256 0; do
      timeout -k 10 120 python -u tools/ab_run.py $(lib_of $v) prof_map --record-bytes 100 --records 33554432 --partitions 1024 --iters 5 --flags $f > "$out/map_${v}_f${f}_$r.txt" 2>&1
    done
  done
done
tail -n 2 "$out"/map_*.txt
echo done > "$out/DONE"
