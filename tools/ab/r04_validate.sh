#!/bin/bash
# Round-4 validation of the current tree on one MI355X: GPU suite, smoke, bench lines (C1
# padded and two-pass, C3, C4, Kryo+LZ4), a kernel trace of the default bench, and the PMC
# passes of C1 / TeraSort / C3 (tools/gpu_prof.sh -> tools/summarize_prof.py on the host).
set -e
tag=${1:-r04c}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1 || { tail -60 "$out/pytest_gpu.log"; exit 1; }
tail -2 "$out/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py > "$out/bench.log" 2>&1
timeout -k 10 300 python -u bench.py --no-padded --no-cpu-baseline > "$out/bench_twopass.log" 2>&1
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline > "$out/bench_c3.log" 2>&1
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline > "$out/bench_c4.log" 2>&1
timeout -k 10 300 python -u bench.py --serializer kryo --compress --steps 5 --warmup 2 --no-cpu-baseline > "$out/bench_kryo_lz4.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- \
  python3 bench.py --steps 10 --no-cpu-baseline > "$out/bench_kt.log" 2>&1
bash tools/gpu_prof.sh $tag/prof_c1
bash tools/gpu_prof.sh $tag/prof_c1_twopass --flags 256
bash tools/gpu_prof.sh $tag/prof_ts --record-bytes 100 --records 42949672
bash tools/gpu_prof.sh $tag/prof_c3 --partitions 4096 --dist zipf
echo done > "$out/DONE"
