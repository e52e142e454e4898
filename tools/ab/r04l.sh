#!/bin/bash
# Round 4, run l: LZ4 batch-compressor phase stamps on C1's Kryo stream (values ~2^27)
set -e
tag=${1:-r04l}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/ab_run.py tools/ab/libsgx_lz4st.so lz4_stamps --case c1 >> "$out/stamps.jsonl" 2> "$out/stamps_c1.err"
cat "$out/stamps.jsonl"
echo done > "$out/DONE"
