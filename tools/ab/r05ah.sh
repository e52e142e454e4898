#!/bin/bash
# The N > 1 bench path on one GPU: 2 ranks over the host-collective backend (rehearsal).
tag=${1:-r05ah}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --comm host --steps 5 --warmup 2 --no-cpu-baseline > "$out/bench_n2_host.log" 2>&1
rc=$?
tail -3 "$out/bench_n2_host.log"
echo "rc $rc"
echo done > "$out/DONE"
exit $rc
