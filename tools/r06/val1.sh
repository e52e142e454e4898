#!/bin/bash
# Round 6: exchange + streaming-writer validation: multirank parity (peer gather), padded /
# streaming / metrics parity, self-exchange and 8-rank host rehearsal lines, the streaming
# writer from retained device and pageable host batches, and the default line.
# usage: bash tools/r06/val1.sh <tag>
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step $log: rc $rc"; tail -30 "$out/$log"; exit $rc; fi
  [ $rc -eq 1 ] && { echo "step $log: rc 1"; tail -40 "$out/$log"; }
  return 0
}
line() { grep '^{' "$out/$1" | python3 -c "
import json,sys
j=json.loads(sys.stdin.read())
print('$1', j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_map_side']['frac'], j['config'].get('map_layout','')[:8], j['stages_ms_per_step'], j.get('exchange_bytes'), j.get('host_ingest'))" || true; }
step 900 pytest_x.log python -u -m pytest tests/test_exchange_multirank.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
tail -2 "$out/pytest_x.log"
step 600 pytest_p.log python -u -m pytest tests/test_padded.py tests/test_streaming_commit.py tests/test_read_metrics.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
tail -2 "$out/pytest_p.log"
step 300 bench.log python -u bench.py --no-cpu-baseline --no-live-pmc --steps 40
line bench.log
step 300 bench_selfx.log python -u bench.py --self-exchange --no-cpu-baseline --steps 20
line bench_selfx.log
step 600 bench_host8.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --comm host --records 67108864 --steps 6 --warmup 2 --no-cpu-baseline
line bench_host8.log
step 300 bench_b64.log python -u bench.py --batches 64 --no-cpu-baseline --no-live-pmc --steps 20
line bench_b64.log
step 300 bench_b64host.log python -u bench.py --batches 64 --host-batches --no-cpu-baseline --no-live-pmc --steps 5 --warmup 1
line bench_b64host.log
echo done > "$out/DONE"
