#!/bin/bash
# Round 4: first GPU run of the single-pass padded map write: its parity
# tests, the map-side parity subset of the suite, then the default bench line and the
# two-pass A/B line, then a kernel trace of the default bench.
set -e
tag=${1:-r04a}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_padded.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest_padded.log" 2>&1 || { tail -60 "$out/pytest_padded.log"; exit 1; }
tail -3 "$out/pytest_padded.log"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/bench.log" 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-padded > "$out/bench_twopass.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 bench.py --steps 10 --no-cpu-baseline > "$out/bench_kt.log" 2>&1
grep '^{' "$out/bench.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['roofline']['frac'], j['roofline_map_side'], j['stages_ms_per_step'], j.get('fetch_all_blocks'))"
grep '^{' "$out/bench_twopass.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['roofline']['frac'], j['roofline_map_side'], j['stages_ms_per_step'], j.get('fetch_all_blocks'))"
echo done > "$out/DONE"
