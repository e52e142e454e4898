#!/bin/bash
# After pruning the superseded TeraSort drain variants: TeraSort / range / padded / exchange GPU
# tests and two C4 bench lines.
tag=${1:-r05aj}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/ \
  -k "terasort or range or wide or c4 or bytes10 or TeraSort" > "$out/pytest_ts.log" 2>&1 || fail "pytest" "$out/pytest_ts.log"
tail -1 "$out/pytest_ts.log"
for i in 1 2; do
  timeout -k 10 180 python -u bench.py --workload c4 --no-cpu-baseline --no-live-pmc > "$out/c4_$i.log" 2>&1 || fail "c4" "$out/c4_$i.log"
  grep '^{' "$out/c4_$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline_map_side']['frac'], d['stages_ms_per_step'])"
done
echo done > "$out/DONE"
