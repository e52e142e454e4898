#!/bin/bash
# C1 K4 (k_scatter16_wc) phase stamps on the current tree; C1 bench twice.
tag=${1:-r05u}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_stamps.so wc_stamps > "$out/stamps_c1.log" 2>&1 || fail "stamps" "$out/stamps_c1.log"
tail -1 "$out/stamps_c1.log"
for i in 1 2; do
  timeout -k 10 180 python -u bench.py --no-cpu-baseline --no-live-pmc > "$out/c1_$i.log" 2>&1 || fail "bench" "$out/c1_$i.log"
done
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c1_*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
echo done > "$out/DONE"
