#!/bin/bash
# Reduce side: nontemporal bucket-sort and group outputs (tree) vs plain stores (rnt0); tests first.
tag=${1:-r05ai}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_reduce_side.py > "$out/pytest_reduce.log" 2>&1 || fail "pytest" "$out/pytest_reduce.log"
tail -1 "$out/pytest_reduce.log"
A="--cases sorted:uniform,group:uniform,sum:zipf --iters 3"
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/prof_reduce.py $A > "$out/tree_$i.log" 2>&1 || fail "tree" "$out/tree_$i.log"
  timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_${V:-rnt0}.so prof_reduce $A > "$out/var_$i.log" 2>&1 || fail "var" "$out/var_$i.log"
done
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*_[0-9].log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); print(f.split("/")[-1], d["case"], d["device_ms"], d["stages_ms"])
PY
echo done > "$out/DONE"
