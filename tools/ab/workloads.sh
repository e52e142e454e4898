#!/bin/bash
# bench.py's other workloads: C3 and C4 at N=1, and their exchange legs rehearsed with 4 ranks
# sharing the GPU over the host backend (gloo)
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python -u bench.py --workload c3 --steps 10 --no-cpu-baseline > "$out/c3.log" 2>&1
timeout -k 10 240 python -u bench.py --workload c4 --steps 10 --no-cpu-baseline > "$out/c4.log" 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline > "$out/c1.log" 2>&1
for w in c3 c4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 4 --workload $w --comm host --records 16777216 --steps 3 --warmup 1 > "$out/${w}_p4_host.log" 2>&1
done
echo done > "$out/DONE"
