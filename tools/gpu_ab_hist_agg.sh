#!/bin/bash
# Histogram A/B: plain LDS atomics (variant 0) vs wave-aggregated ballot/popcount counting
# (variant 7) on uniform and Zipf(1.1) keys at R = 1024 and 4096 (C1 size), output checked.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "variants" > "$out/pytest.log" 2>&1
for rep in 1 2 3; do
  for cfg in uniform:1024 zipf:1024 uniform:4096 zipf:4096; do
    for v in 0 7; do
      echo -n "$cfg hist_variant=$v: " >> "$out/ab.log"
      SGX_HIST_VARIANT=$v timeout -k 10 120 python3 tools/prof_map.py --iters 5 --dist ${cfg%%:*} \
        --partitions ${cfg##*:} 2>&1 | grep -v amdgpu.ids | tail -1 >> "$out/ab.log"
    done
  done
done
echo done > "$out/DONE"
