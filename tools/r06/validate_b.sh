#!/bin/bash
# Round-6 validation, part B: Kryo, Kryo + LZ4, the self-exchange line, the 8-rank rehearsal
# over host collectives, and the reduce side (tools/prof_reduce.py).
tag=${1:-r06v}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "step $log: rc $rc"; tail -30 "$out/$log"; exit $rc; fi
  return 0
}
step 300 bench_kryo.log python -u bench.py --serializer kryo --no-cpu-baseline --no-live-pmc
step 300 bench_kryo_lz4.log python -u bench.py --serializer kryo --compress --steps 5 --warmup 2 --no-cpu-baseline --no-live-pmc
step 300 bench_selfx.log python -u bench.py --self-exchange --no-cpu-baseline --no-live-pmc
step 600 bench_host8.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --comm host --records 67108864 --steps 6 --warmup 2 --no-cpu-baseline
for f in bench_kryo bench_kryo_lz4 bench_selfx bench_host8; do
  grep '^{' "$out/$f.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$f', j['value'], j['ms_per_step'], j['roofline_map_side']['frac'], j['stages_ms_per_step'], j.get('step_design_hbm', {}).get('frac'))" || true
done
step 300 reduce.log python -u tools/prof_reduce.py --records 67108864 --iters 3
grep -h '^{' "$out/reduce.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['case'], d['device_ms'], d['wall_ms_min'], d.get('wall_ms_host_arrays'), d.get('wall_ms_host_arrays_mapped'))"
echo done > "$out/DONE"
