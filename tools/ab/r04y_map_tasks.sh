#!/bin/bash
# Concurrent map tasks in bench.py (--map-tasks T: T threads, one engine stream each) against
# the serial default, C1 and C1 Kryo, alternated; then a kernel trace of T = 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04y
B="--no-cpu-baseline --no-live-pmc"
for i in 1 2; do
  for t in 1 2 3; do
    timeout -k 10 180 python -u bench.py $B --map-tasks $t > gpurun_out/r04y/c1_t${t}_$i.log 2>&1 || exit 1
  done
  for t in 1 2; do
    timeout -k 10 180 python -u bench.py $B --serializer kryo --map-tasks $t > gpurun_out/r04y/kryo_t${t}_$i.log 2>&1 || exit 1
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04y/kt -o run -- python3 bench.py --steps 10 $B --map-tasks 2 \
    > gpurun_out/r04y/kt.log 2>&1 || exit 1
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r04y/*_t*_*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
