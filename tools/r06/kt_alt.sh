#!/bin/bash
# Round 6: kernel traces of the C1 bench with and without alternating write streams, to see
# what rocprofv3 reports for overlapping K4 launches.
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_tree" -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-live-pmc > "$out/kt_tree.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_noalt" -o run -- python3 tools/ab_run.py tools/ab/libsgx_noalt.so bench --steps 10 --no-cpu-baseline --no-live-pmc > "$out/kt_noalt.log" 2>&1 || exit $?
for v in tree noalt; do
  python3 tools/trace_steady.py "$out/kt_$v/run_kernel_trace.csv" --warmup 3 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['k4_us_timed_mean'], d['interval_us_timed_mean'], d['interval_frac_timed'], d['k4_us_per_write'])"
done
echo done > "$out/DONE"
