#!/bin/bash
# Round-6 validation of the current tree on one MI355X, part A: GPU suite, smoke, the bench
# lines (C1 default with live PMC + CPU baseline, the streaming writer from device and host
# batches, two-pass, C3, C4, C1 / C4 without overlapping writes).  Part B (validate_b.sh): Kryo,
# Kryo + LZ4, self-exchange, the 8-rank rehearsal, the reduce side; part C (validate_prof.sh):
# kernel traces and PMC passes.
# Test failures (pytest rc 1) do not stop the measurements; a crash, abort or timeout does.
tag=${1:-r06v}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # step <timeout> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step $log: rc $rc"; tail -30 "$out/$log"; exit $rc; fi
  [ $rc -eq 1 ] && echo "step $log: rc 1 (test failures)"
  return 0
}
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider
tail -3 "$out/pytest_gpu.log"
step 120 smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 "$out/smoke.log"
step 300 bench.log python -u bench.py
step 300 bench_b64.log python -u bench.py --batches 64 --no-cpu-baseline --no-live-pmc
step 300 bench_b64host.log python -u bench.py --batches 64 --host-batches --steps 5 --warmup 1 --no-cpu-baseline --no-live-pmc
step 300 bench_twopass.log python -u bench.py --no-padded --no-cpu-baseline
step 300 bench_c3.log python -u bench.py --workload c3 --no-cpu-baseline
step 300 bench_c4.log python -u bench.py --workload c4 --no-cpu-baseline
step 300 bench_nooverlap.log python -u bench.py --no-overlap-writes --no-cpu-baseline --no-live-pmc
step 300 bench_c4_nooverlap.log python -u bench.py --workload c4 --no-overlap-writes --no-cpu-baseline --no-live-pmc
for f in bench bench_b64 bench_b64host bench_twopass bench_c3 bench_c4 bench_nooverlap bench_c4_nooverlap; do
  grep '^{' "$out/$f.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$f', j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline'].get('timed_region_k4_interval_ms'), j['roofline_map_side']['frac'], j['roofline_map_side']['traffic_over_algorithmic'], j['stages_ms_per_step'])" || true
done
echo done > "$out/DONE"
