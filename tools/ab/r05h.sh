#!/bin/bash
# Padded write's tail on a second stream: map-side parity, C1 bench A/B against libsgx_tail0
# (HEAD before it), then the reduce-side A/B and PMC (r05f.sh).
tag=${1:-r05h}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T -m gpu tests/test_padded.py tests/test_streaming_commit.py tests/test_threads_streaming_combine.py \
  tests/test_kryo.py tests/test_gpu_parity.py > "$out/pytest_map.log" 2>&1 || fail "pytest map rc $?" "$out/pytest_map.log"
tail -1 "$out/pytest_map.log"
B="--no-cpu-baseline --no-live-pmc"
for i in 1 2; do
  timeout -k 10 180 python -u bench.py $B > "$out/c1_new_$i.log" 2>&1 || fail "bench new" "$out/c1_new_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_tail0.so bench $B > "$out/c1_old_$i.log" 2>&1 || fail "bench old" "$out/c1_old_$i.log"
done
timeout -k 10 180 python -u bench.py $B --serializer kryo > "$out/kryo_new.log" 2>&1 || fail "bench kryo" "$out/kryo_new.log"
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*_*.log")):
    if "pytest" in f: continue
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline_map_side"]["frac"], d["stages_ms_per_step"])
PY
bash tools/ab/r05f.sh $tag/red
echo done > "$out/DONE"
