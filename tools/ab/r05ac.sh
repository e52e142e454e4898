#!/bin/bash
# Single-pass Kryo serializer (look-back) vs the length pass + tile scan (klb0): Kryo / LZ4 /
# streaming / padded GPU tests, then C1 Kryo bench alternations; bucket-sort A/B after.
tag=${1:-r05ac}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/ \
  -k "kryo or Kryo or lz4 or LZ4 or serial or unsafe or streaming or spill or combine" > "$out/pytest_kryo.log" 2>&1 || fail "pytest" "$out/pytest_kryo.log"
tail -1 "$out/pytest_kryo.log"
B="--serializer kryo --no-cpu-baseline --no-live-pmc"
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py $B > "$out/k_tree_$i.log" 2>&1 || fail "bench" "$out/k_tree_$i.log"
  timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_klb0.so bench $B > "$out/k_klb0_$i.log" 2>&1 || fail "bench klb0" "$out/k_klb0_$i.log"
done
timeout -k 10 180 python -u bench.py $B --batches 64 > "$out/kb64_tree.log" 2>&1 || fail "bench b64" "$out/kb64_tree.log"
python3 - "$out" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/k*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["stages_ms_per_step"])
PY
echo done > "$out/DONE"
