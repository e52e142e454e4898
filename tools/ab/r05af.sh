#!/bin/bash
# C3 small kernels: parallel hot-set cut search and one wave per super in the cold estimate,
# vs HEAD; split / padded / parity tests first; C3 bench alternations + a kernel trace.
tag=${1:-r05af}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_padded.py tests/test_gpu_parity.py -k "split or hot or 4096 or 2048 or 8192 or zipf or c3 or padded" > "$out/pytest.log" 2>&1 || fail "pytest" "$out/pytest.log"
tail -1 "$out/pytest.log"
C="--workload c3 --no-cpu-baseline --no-live-pmc"
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py $C > "$out/c3_tree_$i.log" 2>&1 || fail "c3" "$out/c3_tree_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_head.so bench $C > "$out/c3_head_$i.log" 2>&1 || fail "c3 head" "$out/c3_head_$i.log"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o run -- python3 tools/prof_map.py --partitions 4096 --dist zipf --iters 5 > "$out/kt.log" 2>&1 || fail "kt" "$out/kt.log"
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c3_*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
grep -h "hot_select\|cold_super" "$out"/kt/*kernel_stats.csv | cut -c1-120
echo done > "$out/DONE"
