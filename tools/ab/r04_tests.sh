#!/bin/bash
# Round 4: the new GPU tests (padded write, import of fetched blocks, coordinator protocol),
# then the default bench line and the two-pass A/B line.
set -e
tag=${1:-r04b}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_padded.py tests/test_import_blocks.py tests/test_coordinator.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$out/pytest_new.log" 2>&1 || { tail -80 "$out/pytest_new.log"; exit 1; }
tail -3 "$out/pytest_new.log"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/bench.log" 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-padded > "$out/bench_twopass.log" 2>&1
for f in bench bench_twopass; do
grep '^{' "$out/$f.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$f', j['value'], j['roofline']['frac'], j['roofline_map_side'], j['stages_ms_per_step'], j.get('fetch_all_blocks'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 bench.py --steps 10 --no-cpu-baseline > "$out/bench_kt.log" 2>&1
echo done > "$out/DONE"
