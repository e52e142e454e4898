#!/bin/bash
# Round 6: chunk-major sub-bins for the C3 split (k_pad_caps) -- split / overflow parity, then
# same-box alternating C3 lines against the previous commit (c3pm: partition-major split).
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "4096 or 2048 or 8192 or split or zipf or padded or overflow or fall" > "$out/pytest.log" 2>&1 || { tail -40 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
run() {
  local lib=$1 log=$2; shift 2
  if [ "$lib" = tree ]; then
    timeout -k 10 300 python -u bench.py "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  else
    timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_$lib.so bench "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  fi
  grep '^{' "$out/$log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$log', j['value'], j['ms_per_step'], j['roofline_map_side']['frac'], j['stages_ms_per_step'])"
}
for rep in 1 2 3; do
  for lib in tree c3pm; do run $lib c3_${lib}_$rep.log --workload c3 --no-cpu-baseline --no-live-pmc --steps 20; done
done
echo done > "$out/DONE"
