#!/bin/bash
# Round 4, run d: the GPU tests changed since r04c, the LZ4 / TeraSort A/B
# (tools/ab/r04_lz4_wide.sh), the self-exchange overlap trace on the current exchange path
# (tools/ab/selfx.sh), and PMC passes for the bench's C4 size and uniform R = 4096.
set -e
tag=${1:-r04d}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_coordinator.py tests/test_gpu_parity.py tests/test_padded.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider -k "coordinator or shuffle_client or padded_exchange" \
  > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
bash tools/ab/r04_lz4_wide.sh $tag/ab
bash tools/ab/selfx.sh $tag/selfx
cat "$out/selfx/overlap.jsonl" | tail -3
bash tools/gpu_prof.sh $tag/prof_ts25 --record-bytes 100 --records 33554432
bash tools/gpu_prof.sh $tag/prof_u4096 --partitions 4096
echo done > "$out/DONE"
