#!/bin/bash
# Round 4, run p: segmented window pass and segmented digit passes (compact piece layout) --
# tools/prof_reduce.py with it (flags 0) and without it (flags 1024), alternating.
set -e
tag=${1:-r04p}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_reduce_side.py -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -40 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
for r in 1 2; do
  for f in 0 1024; do
    timeout -k 10 300 python -u tools/prof_reduce.py --flags $f > "$out/reduce_f${f}_$r.txt" 2>&1
    tail -4 "$out/reduce_f${f}_$r.txt"
  done
done
echo done > "$out/DONE"
