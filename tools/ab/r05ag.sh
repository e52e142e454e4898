#!/bin/bash
# The padded write's sample: 512 (tree) vs 256 / 128 workgroups (fewer closing atomics, more
# loads per lane); C1 and C4 bench alternations.
tag=${1:-r05ag}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
C="--no-cpu-baseline --no-live-pmc"
for i in 1 2; do
  for v in tree g256 g128; do
    if [ $v = tree ]; then R="python -u bench.py"; else R="python -u tools/ab_run.py tools/ab/libsgx_$v.so bench"; fi
    timeout -k 10 180 $R $C > "$out/c1_${v}_$i.log" 2>&1 || fail "c1 $v" "$out/c1_${v}_$i.log"
    timeout -k 10 180 $R $C --workload c4 > "$out/c4_${v}_$i.log" 2>&1 || fail "c4 $v" "$out/c4_${v}_$i.log"
  done
done
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
echo done > "$out/DONE"
