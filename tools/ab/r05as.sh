#!/bin/bash
# TeraSort K4: stream starts in the owners registers vs HEAD (3 alternations).
tag=${1:-r05as}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T -m gpu tests/ \
  -k "terasort or range or wide or c4 or bytes10 or TeraSort" > "$out/pytest_ts.log" 2>&1 || fail "pytest ts rc $?" "$out/pytest_ts.log"
tail -1 "$out/pytest_ts.log"
B="--workload c4 --no-cpu-baseline --no-live-pmc"
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py $B > "$out/c4_new_$i.log" 2>&1 || fail "bench rc $?" "$out/c4_new_$i.log"
  for v in ${VARIANTS:-head}; do
    timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_$v.so bench $B > "$out/c4_${v}_$i.log" 2>&1 || fail "bench $v" "$out/c4_${v}_$i.log"
  done
done
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c4_*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
echo done > "$out/DONE"
