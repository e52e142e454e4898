#!/bin/bash
# C1 Kryo: nontemporal record loads in the serializer (kntl) vs the tree.
tag=${1:-r05an}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
B="--serializer kryo --no-cpu-baseline --no-live-pmc"
for i in 1 2; do
  timeout -k 10 180 python -u bench.py $B > "$out/k_tree_$i.log" 2>&1 || fail "bench" "$out/k_tree_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_kntl.so bench $B > "$out/k_kntl_$i.log" 2>&1 || fail "bench knt" "$out/k_kntl_$i.log"
done
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/k_*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
echo done > "$out/DONE"
