#!/bin/bash
# Round 4, run k: LZ4 GPU tests (incl. the batch-compressor shapes) and the batch compressor's
# phase stamps (tools/ab/libsgx_lz4st.so, tools/lz4_stamps.py) on three streams.
set -e
tag=${1:-r04k}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_lz4.py tests/test_kryo.py -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
for c in c1 lowentropy uniform; do
  timeout -k 10 200 python -u tools/ab_run.py tools/ab/libsgx_lz4st.so lz4_stamps --case $c >> "$out/stamps.jsonl" 2> "$out/stamps_$c.err"
done
cat "$out/stamps.jsonl"
echo done > "$out/DONE"
