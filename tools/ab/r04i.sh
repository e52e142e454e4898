#!/bin/bash
# Round 4, run i: the write-combining K4 writing whole 128 B lines (tree) against 64 B
# (tools/ab/libsgx_wc4.so) and 32 B units (wc2): C1 K4 time and HBM bytes (WRITE_SIZE / FETCH_SIZE).
set -e
tag=${1:-r04i}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
lib_of() { [ "$1" = tree ] && echo sparkucx_amd/libsgx.so || echo tools/ab/libsgx_$1.so; }
timeout -k 10 300 python -u -m pytest tests/test_padded.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider --sgx-lib $(lib_of wc4) -k "padded or c1 or uniform" > "$out/pytest_wc4.log" 2>&1 || { tail -30 "$out/pytest_wc4.log"; exit 1; }
tail -1 "$out/pytest_wc4.log"
for r in 1 2; do
  for v in tree wc4 wc2; do
    timeout -k 10 120 python -u tools/ab_run.py $(lib_of $v) prof_map --iters 5 > "$out/map_${v}_$r.txt" 2>&1
  done
done
tail -n 1 "$out"/map_*.txt
for v in tree wc4 wc2; do
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_${v}_$c" -o run -- \
      python3 tools/ab_run.py $(lib_of $v) prof_map --iters 2 > "$out/pmc_${v}_$c.log" 2>&1
  done
done
echo done > "$out/DONE"
