#!/bin/bash
# Round 6: the streaming-writer tests on the tree, then the phase stamps of the TeraSort
# write-combining K4 (stamp build, tools/wc_stamps.py) at C4's per-GPU map size.
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_streaming_commit.py tests/test_read_metrics.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_stamps.so wc_stamps --record-bytes 100 --wide-wc --records 33554432 > "$out/stamps_ts.log" 2>&1 || { tail -20 "$out/stamps_ts.log"; exit 1; }
tail -2 "$out/stamps_ts.log"
timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_stamps.so wc_stamps > "$out/stamps_c1.log" 2>&1 || { tail -20 "$out/stamps_c1.log"; exit 1; }
tail -2 "$out/stamps_c1.log"
echo done > "$out/DONE"
