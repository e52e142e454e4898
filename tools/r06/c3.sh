#!/bin/bash
# Round 6: the split's packed level 2 -- split parity (padded + two-pass at R 2048 / 4096 /
# Zipf), the C3 line, and its kernel stats.
# usage: bash tools/r06/c3.sh <tag>
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "step $log: rc $rc"; tail -40 "$out/$log"; exit $rc; fi
  return 0
}
step 600 pytest_split.log python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "4096 or 2048 or zipf or split or 8192 or 6144 or padded"
tail -2 "$out/pytest_split.log"
step 300 bench_c3.log python -u bench.py --workload c3 --no-cpu-baseline --no-live-pmc --steps 20
grep '^{' "$out/bench_c3.log" | python3 -c "
import json,sys
j=json.loads(sys.stdin.read())
print('c3', j['value'], j['ms_per_step'], j['roofline_map_side'], j['stages_ms_per_step'])"
step 300 prof_c3.log rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_c3" -o c3 -- python3 -u bench.py --workload c3 --no-cpu-baseline --no-live-pmc --steps 5 --warmup 2
f=$(find "$out/prof_c3" -name '*kernel_stats.csv' | head -1); cp "$f" "$out/c3_kernel_stats.csv"
python3 -c "
import csv
for r in csv.DictReader(open('$out/c3_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])"
echo done > "$out/DONE"
