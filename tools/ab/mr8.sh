#!/bin/bash
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_exchange_multirank.py -m gpu -x -v --timeout 400 --timeout-method thread -k eight > "$out/pytest.log" 2>&1
echo done > "$out/DONE"
