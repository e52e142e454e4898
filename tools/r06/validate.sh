#!/bin/bash
# Round-6 validation of the current tree on one MI355X, part A: GPU suite, smoke, the bench
# lines (C1 default with live PMC + CPU baseline, the streaming writer from device and host
# batches, two-pass, C3, C4, Kryo, Kryo + LZ4, self-exchange, the 8-rank rehearsal) and the
# reduce side.  Part B (tools/r06/validate_prof.sh) collects the kernel traces and PMC passes.
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
step 300 bench_kryo.log python -u bench.py --serializer kryo --no-cpu-baseline --no-live-pmc
step 300 bench_kryo_lz4.log python -u bench.py --serializer kryo --compress --steps 5 --warmup 2 --no-cpu-baseline --no-live-pmc
step 300 bench_selfx.log python -u bench.py --self-exchange --no-cpu-baseline --no-live-pmc
step 600 bench_host8.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --comm host --records 67108864 --steps 6 --warmup 2 --no-cpu-baseline
for f in bench bench_b64 bench_b64host bench_twopass bench_c3 bench_c4 bench_kryo bench_kryo_lz4 bench_selfx bench_host8; do
  grep '^{' "$out/$f.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$f', j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_map_side']['frac'], j['roofline_map_side']['traffic_over_algorithmic'], j['stages_ms_per_step'])" || true
done
step 300 reduce.log python -u tools/prof_reduce.py --records 67108864 --iters 3
grep -h '^{' "$out/reduce.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['case'], d['device_ms'], d['wall_ms_min'], d.get('wall_ms_host_arrays'))"
echo done > "$out/DONE"
