#!/bin/bash
# Round 6: the C3 front on its own stream, pinned-staged host reads, the peer gather's L2
# release / acquire -- the whole GPU suite, then the C3 / self-exchange / 8-rank rehearsal lines
# and the reduce side's host-array reads.
# usage: bash tools/r06/val2.sh <tag>
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
line() { grep '^{' "$out/$1" | python3 -c "
import json,sys
j=json.loads(sys.stdin.read())
print('$1', j['value'], j['ms_per_step'], j['roofline_map_side']['frac'], j['stages_ms_per_step'], j.get('exchange_bytes'), j.get('step_design_hbm'))" || true; }
step 1000 pytest_gpu.log python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
tail -3 "$out/pytest_gpu.log"
step 300 bench_c3.log python -u bench.py --workload c3 --no-cpu-baseline --no-live-pmc --steps 20
line bench_c3.log
step 300 bench_selfx.log python -u bench.py --self-exchange --no-cpu-baseline --steps 20
line bench_selfx.log
step 600 bench_host8.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --comm host --records 67108864 --steps 6 --warmup 2 --no-cpu-baseline
line bench_host8.log
step 300 reduce.log python -u tools/prof_reduce.py --records 67108864 --iters 5
grep '^{' "$out/reduce.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['case'], d['device_ms'], d['wall_ms_min'], d.get('wall_ms_host_arrays'))"
echo done > "$out/DONE"
