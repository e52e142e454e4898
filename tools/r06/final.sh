#!/bin/bash
# Round 6, last validation of the final tree: part A (GPU suite, smoke, bench lines), then the
# PMC / kernel profiles of C1, TeraSort and C3 and a kernel trace of the one-stream bench.
tag=${1:-r06f}
bash tools/r06/validate.sh $tag || exit $?
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_prof.sh $tag/prof_c1 || exit 1
bash tools/gpu_prof.sh $tag/prof_ts --record-bytes 100 --records 42949672 || exit 1
bash tools/gpu_prof.sh $tag/prof_c3 --partitions 4096 --dist zipf || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_noov" -o run -- python3 bench.py --steps 10 --no-cpu-baseline --no-live-pmc --no-overlap-writes > "$out/bench_kt_noov.log" 2>&1 || exit $?
python3 tools/trace_steady.py "$out/kt_noov/run_kernel_trace.csv" --warmup 3 --out "$out/trace_steady_noov.json"
echo done > "$out/DONE2"
