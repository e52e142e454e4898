#!/bin/bash
# byte-balanced placement: multi-rank GPU tests (host backend, ranks share the GPU) and the C3
# exchange leg with 4 ranks, even vs bytes placement
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_exchange_multirank.py -m gpu -x -v --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
for pl in even bytes; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 \
    bench.py --gpus 4 --workload c3 --comm host --placement $pl --records 16777216 --steps 3 --warmup 1 > "$out/c3_p4_$pl.log" 2>&1
done
echo done > "$out/DONE"
