#!/bin/bash
# Round 4, run j: bench.py with its live rocprofv3 PMC passes (roofline.traffic from this run)
set -e
tag=${1:-r04j}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in c1 c3 c4; do
  s=$(date +%s)
  timeout -k 10 400 python -u bench.py --workload $w $([ $w = c1 ] || echo --no-cpu-baseline) > "$out/bench_$w.log" 2>&1
  echo "$w: $(( $(date +%s) - s )) s"
  grep '^{' "$out/bench_$w.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['roofline'], j['roofline_map_side'])"
done
echo done > "$out/DONE"
