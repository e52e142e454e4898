#!/bin/bash
# Round 5: the one-pass streaming commit (deferred batches, chunk tables) -- its GPU tests,
# the neighbouring suites, and the bench line of the writer sequence Spark drives.
tag=${1:-r05b}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_streaming_commit.py tests/test_threads_streaming_combine.py tests/test_read_metrics.py \
  > "$out/pytest_stream.log" 2>&1 || { echo "pytest rc $?"; tail -40 "$out/pytest_stream.log"; exit 1; }
tail -3 "$out/pytest_stream.log"
timeout -k 10 300 python -u bench.py --batches 64 --no-cpu-baseline > "$out/bench_batches64.log" 2>&1 || { echo "bench rc $?"; tail -20 "$out/bench_batches64.log"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/bench.log" 2>&1 || { echo "bench rc $?"; tail -20 "$out/bench.log"; exit 1; }
for f in bench_batches64 bench; do
  grep '^{' "$out/$f.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$f', j['value'], j['roofline']['frac'], j['roofline_map_side']['frac'], j['roofline_map_side']['ms'], j['roofline_map_side']['traffic_over_algorithmic'], j['config']['map_layout'][:10])"
done
echo done > "$out/DONE"
