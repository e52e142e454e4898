#!/bin/bash
# LZ4 GPU tests, then wave/lane decode timings at 2^22 and 2^24 records
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_lz4.py tests/test_threads_streaming_combine.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
for n in 4194304 16777216; do
  timeout -k 10 180 python -u tools/prof_lz4.py --records $n --iters 3 > "$out/default_$n.jsonl" 2>&1
done
echo done > "$out/DONE"
