#!/bin/bash
# Does one of bench.py's two map slots write slower?  K4 per launch (stage events, each write
# alone) over 12 writes cycling 2 map ids, then 1 map id, then 3.
tag=${1:-r05ak}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
for sl in 2 1 3 2; do
  timeout -k 10 240 python -u tools/prof_map.py --iters 12 --per-launch --slots $sl > "$out/slots${sl}.log" 2>&1 || fail "slots $sl" "$out/slots${sl}.log"
  python3 - "$out/slots${sl}.log" $sl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("PER_LAUNCH "):
        per = json.loads(l[len("PER_LAUNCH "):])
        print("slots", sys.argv[2], [p.get("scatter") for p in per])
PY
done
echo done > "$out/DONE"
