#!/bin/bash
# Round-6 validation, part C: rocprofv3 kernel traces of the default bench (overlapping writes:
# its timed K4s include their wait for CUs, its roofline phase does not), of the same without
# overlap (and its steady-state map side, tools/trace_steady.py), of the C3 and C4 lines, and
# the PMC passes (tools/gpu_prof.sh over tools/prof_map.py, writes on one stream: FETCH_SIZE and
# WRITE_SIZE in separate runs) for C1, TeraSort and C3.
tag=${1:-r06v}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "step $log: rc $rc"; tail -30 "$out/$log"; exit $rc; fi
  return 0
}
step 300 bench_kt.log rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-live-pmc
step 300 bench_kt_noov.log rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_noov" -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-live-pmc --no-overlap-writes
python3 tools/trace_steady.py "$out/kt_noov/run_kernel_trace.csv" --warmup 3 --out "$out/trace_steady_noov.json"
step 300 bench_kt_c3.log rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_c3" -o run -- python3 bench.py --workload c3 --steps 10 --no-cpu-baseline --no-live-pmc
step 300 bench_kt_c4.log rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_c4" -o run -- python3 bench.py --workload c4 --steps 10 --no-cpu-baseline --no-live-pmc
bash tools/gpu_prof.sh $tag/prof_c1 || exit 1
bash tools/gpu_prof.sh $tag/prof_ts --record-bytes 100 --records 42949672 || exit 1
bash tools/gpu_prof.sh $tag/prof_c3 --partitions 4096 --dist zipf || exit 1
echo done > "$out/DONE"
