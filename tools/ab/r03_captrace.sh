#!/bin/bash
# per-kernel times of the hybrid split at three hot-stream caps (rocprofv3 kernel trace),
# one trace per variant and config; then the alternating timing A/B with parity (r03_ab.sh)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03_captrace; mkdir -p $o
for c in zipf:4096 uniform:4096; do
  for v in base cap192 cap448 tree; do
    lib=sparkucx_amd/libsgx.so; [ $v != tree ] && lib=tools/ab/libsgx_$v.so
    d=$o/${v}_${c/:/_}
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 tools/ab_run.py $lib prof_configs --configs $c --iters 5 > $d.log 2>&1
    echo "== $v $c"; python3 - $d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'scatter' in r['Name'] or 'hot' in r['Name'] or 'super' in r['Name'] or 'seg' in r['Name']:
        print(' ', r['Name'].split('(')[0][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
PY
  done
done
bash tools/ab/r03_ab.sh r03_cap_ab "base cap192 cap448 tree" uniform:2048,zipf:4096,uniform:4096,uniform:1024
