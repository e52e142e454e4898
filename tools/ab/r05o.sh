#!/bin/bash
# TeraSort K4, 1024-record tiles vs HEAD (512): bench C4 at 2^25 and at 42.9 M records, prof_map, same box.
tag=${1:-r05o}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
B="--workload c4 --no-cpu-baseline --no-live-pmc"
A="--record-bytes 100 --records 42949672 --iters 5"
for i in 1 2; do
  for v in tree old; do
    if [ $v = tree ]; then R="python -u"; P="python -u tools/prof_map.py"; else R="python -u tools/ab_run.py tools/ab/libsgx_$v.so bench"; P="python -u tools/ab_run.py tools/ab/libsgx_$v.so prof_map"; fi
    if [ $v = tree ]; then R="$R bench.py"; fi
    timeout -k 10 180 $R $B > "$out/c4_${v}_$i.log" 2>&1 || fail "bench $v" "$out/c4_${v}_$i.log"
    timeout -k 10 180 $R $B --records 42949672 > "$out/c4big_${v}_$i.log" 2>&1 || fail "bench big $v" "$out/c4big_${v}_$i.log"
    timeout -k 10 180 $P $A > "$out/pm_${v}_$i.log" 2>&1 || fail "pm $v" "$out/pm_${v}_$i.log"
    echo "pm $v $(tail -1 $out/pm_${v}_$i.log)"
  done
done
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c4*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
echo done > "$out/DONE"
