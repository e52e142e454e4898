#!/bin/bash
# Slot asymmetry probe: K4 per launch over 12 writes cycling 2 map ids, exact device buffers
# (tree) vs buffers rounded up to 2 MiB (a2m) / 1 GiB (a1g).
tag=${1:-r05al}
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
A="--iters 12 --per-launch --slots 2"
for i in 1 2; do
  timeout -k 10 240 python -u tools/prof_map.py $A > "$out/tree_$i.log" 2>&1 || fail "tree" "$out/tree_$i.log"; pr "$out/tree_$i.log" tree
  for v in a2m a1g; do
    timeout -k 10 240 python -u tools/ab_run.py tools/ab/libsgx_$v.so prof_map $A > "$out/${v}_$i.log" 2>&1 || fail "$v" "$out/${v}_$i.log"; pr "$out/${v}_$i.log" $v
  done
done
echo done > "$out/DONE"
