#!/bin/bash
# Round 6: chunk-major sub-bins (tree) against partition-major (pm) -- padded / streaming /
# exchange / Kryo parity, per-launch K4 times over two map slots (tools/prof_map.py
# --per-launch), then alternating C1 and C4 lines.
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_padded.py tests/test_streaming_commit.py tests/test_kryo.py tests/test_exchange_multirank.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1 || { tail -40 "$out/pytest.log"; exit 1; }
tail -2 "$out/pytest.log"
tool() {  # tool <lib> <log> <tool> <args...>
  local lib=$1 log=$2 t=$3; shift 3
  if [ "$lib" = tree ]; then
    timeout -k 10 300 python -u $t.py "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  else
    timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_$lib.so $(basename $t) "$@" > "$out/$log" 2>&1 || { echo "$log rc $?"; tail -20 "$out/$log"; exit 1; }
  fi
}
for lib in tree pm; do
  tool $lib pl_$lib.log tools/prof_map --iters 12 --per-launch --slots 2
  grep PER_LAUNCH "$out/pl_$lib.log" | sed 's/PER_LAUNCH //' | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$lib per-launch K4 ms', [x.get('scatter') for x in d])"
done
for rep in 1 2; do
  for lib in tree pm; do
    tool $lib c1_${lib}_$rep.log bench --no-cpu-baseline --no-live-pmc --steps 40
    grep '^{' "$out/c1_${lib}_$rep.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('c1', '$lib', $rep, j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_map_side']['frac'])"
  done
done
for rep in 1 2; do
  for lib in tree pm; do
    tool $lib c4_${lib}_$rep.log bench --workload c4 --no-cpu-baseline --no-live-pmc --steps 40
    grep '^{' "$out/c4_${lib}_$rep.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('c4', '$lib', $rep, j['value'], j['ms_per_step'], j['roofline']['frac'], j['roofline_map_side']['frac'])"
  done
done
echo done > "$out/DONE"
