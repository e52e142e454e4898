#!/bin/bash
# Round 5: streaming commit tests + bench --batches; TeraSort K4 (swizzled carry rows, dword
# drain) parity and A/B against the round-4 kernel (libsgx_wwcold) and swizzle-only (wwcsw).
tag=${1:-r05c}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_streaming_commit.py tests/test_threads_streaming_combine.py tests/test_read_metrics.py \
  > "$out/pytest_stream.log" 2>&1 || fail "pytest stream rc $?" "$out/pytest_stream.log"
tail -1 "$out/pytest_stream.log"
timeout -k 10 600 $T -m gpu tests/test_padded.py tests/test_gpu_parity.py tests/test_reduce_side.py tests/test_exchange_multirank.py \
  -k "terasort or range or wide or c4 or bytes10 or TeraSort" > "$out/pytest_ts.log" 2>&1 || fail "pytest ts rc $?" "$out/pytest_ts.log"
tail -1 "$out/pytest_ts.log"
B="--workload c4 --no-cpu-baseline --no-live-pmc"
for i in 1 2; do
  timeout -k 10 180 python -u bench.py $B > "$out/c4_new_$i.log" 2>&1 || fail "bench rc $?" "$out/c4_new_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_wwcold.so bench $B > "$out/c4_old_$i.log" 2>&1 || fail "bench old" "$out/c4_old_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_wwcsw.so bench $B > "$out/c4_sw_$i.log" 2>&1 || fail "bench sw" "$out/c4_sw_$i.log"
done
timeout -k 10 300 python -u bench.py --batches 64 --no-cpu-baseline > "$out/bench_batches64.log" 2>&1 || fail "bench batches" "$out/bench_batches64.log"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$out/bench.log" 2>&1 || fail "bench" "$out/bench.log"
for g in 512 1024; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-live-pmc --num-chunks $g > "$out/bench_g$g.log" 2>&1 || fail "bench g$g" "$out/bench_g$g.log"
done
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.log")):
    if "pytest" in f: continue
    d = [json.loads(l) for l in open(f) if l.startswith("{")]
    if not d: continue
    d = d[-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline_map_side"]["frac"],
          d["roofline_map_side"]["traffic_over_algorithmic"], d["stages_ms_per_step"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/rec_c1" -o run -- \
  python3 tools/prof_map.py --iters 8 --per-launch > "$out/rec_c1.log" 2>&1 || fail "reconcile c1" "$out/rec_c1.log"
python3 tools/reconcile_trace.py "$out/rec_c1/run_kernel_trace.csv" "$out/rec_c1.log" > "$out/reconcile_c1.jsonl" || true
tail -1 "$out/reconcile_c1.jsonl"
bash tools/gpu_prof.sh $tag/prof_ts --record-bytes 100 --records 42949672 || exit 1
bash tools/sq_counters.sh "$out/sq_ts" --record-bytes 100 --records 42949672 --iters 2 || exit 1
echo done > "$out/DONE"
