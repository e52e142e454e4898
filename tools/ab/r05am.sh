#!/bin/bash
# Slot asymmetry probe: exact hipMalloc (tree) vs contiguous large buffers (contig), 2 and 3 slots.
# Slot asymmetry probe: exact hipMalloc (tree) vs contiguous large buffers (contig), 2 and 3 slots.
tag=${1:-r05am}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
pr() { python3 - "$1" "$2" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("PER_LAUNCH "):
        per = json.loads(l[len("PER_LAUNCH "):])
        print(sys.argv[2], [p.get("scatter") for p in per])
PY
}
for A in "--iters 12 --per-launch --slots 2" "--iters 12 --per-launch --slots 3"; do
for i in 1; do
  timeout -k 10 240 python -u tools/prof_map.py $A > "$out/tree_s${A##* }_$i.log" 2>&1 || fail "tree" "$out/tree_s${A##* }_$i.log"; pr "$out/tree_s${A##* }_$i.log" tree
  for v in contig; do
    timeout -k 10 240 python -u tools/ab_run.py tools/ab/libsgx_$v.so prof_map $A > "$out/${v}_s${A##* }_$i.log" 2>&1 || fail "$v" "$out/${v}_s${A##* }_$i.log"; pr "$out/${v}_s${A##* }_$i.log" $v
  done
done; done
echo done > "$out/DONE"
