#!/bin/bash
# Round 4, run s: padded write with the sample capped at one line in 512 (tools/ab/libsgx_samp512.so)
# against one in 128 (tree): padded-write tests, then C1 / C3 / C4 bench lines alternating.
set -e
tag=${1:-r04s}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
lib_of() { [ "$1" = tree ] && echo sparkucx_amd/libsgx.so || echo tools/ab/libsgx_$1.so; }
timeout -k 10 400 python -u -m pytest tests/test_padded.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider --sgx-lib $(lib_of samp512) > "$out/pytest_samp512.log" 2>&1 || { tail -30 "$out/pytest_samp512.log"; exit 1; }
tail -1 "$out/pytest_samp512.log"
for r in 1 2 3; do
  for v in tree samp512; do
    for w in c1 c3 c4; do
      timeout -k 10 300 python -u -c "
import sys; sys.argv=['bench.py','--workload','$w','--no-cpu-baseline','--no-live-pmc']
import sparkucx_amd._lib as L; L.LIB_PATH='$(lib_of $v)'
import runpy; runpy.run_path('bench.py', run_name='__main__')" 2>/dev/null | grep '^{' | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> "$out/bench.jsonl"
    done
  done
done
python3 - "$out" <<'PY'
import json, sys
for l in open(sys.argv[1] + '/bench.jsonl'):
    j = json.loads(l); print(j['variant'], j['rep'], j['config']['workload'][:3], j['value'], j['roofline_map_side']['ms'], j['stages_ms_per_step'])
PY
echo done > "$out/DONE"
