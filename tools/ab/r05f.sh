#!/bin/bash
# Bucket sort with sub-bins: reduce-side parity, then prof_reduce A/B against libsgx_bs0.so.
tag=${1:-r05f}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T -m gpu tests/test_reduce_side.py tests/test_threads_streaming_combine.py tests/test_import_blocks.py \
  > "$out/pytest_reduce.log" 2>&1 || fail "pytest reduce rc $?" "$out/pytest_reduce.log"
tail -1 "$out/pytest_reduce.log"
for i in 1 2; do
  timeout -k 10 300 python -u tools/prof_reduce.py --records 67108864 --iters 3 > "$out/red_new_$i.jsonl" 2>&1 || fail "prof new" "$out/red_new_$i.jsonl"
  timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_${OLD:-bs0}.so prof_reduce --records 67108864 --iters 3 > "$out/red_old_$i.jsonl" 2>&1 || fail "prof old" "$out/red_old_$i.jsonl"
done
grep -h '^{' "$out"/red_*.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['case'], d['device_ms'], d['stages_ms'])" 
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/red_kt" -o run -- \
  python3 tools/prof_reduce.py --records 67108864 --iters 3 > "$out/red_kt.log" 2>&1 || fail "red kt" "$out/red_kt.log"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/red_fetch" -o run -- \
  python3 tools/prof_reduce.py --records 67108864 --iters 1 > "$out/red_fetch.log" 2>&1 || fail "fetch" "$out/red_fetch.log"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/red_write" -o run -- \
  python3 tools/prof_reduce.py --records 67108864 --iters 1 > "$out/red_write.log" 2>&1 || fail "write" "$out/red_write.log"
echo done > "$out/DONE"
