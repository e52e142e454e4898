#!/bin/bash
# Kryo decoder with the padded stage: Kryo / LZ4 read tests, then the Kryo bench's decode leg.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kryo.py \
    tests/test_lz4.py tests/test_reduce_side.py > gpurun_out/r04v_pytest.log 2>&1 || { tail -30 gpurun_out/r04v_pytest.log; exit 1; }
tail -1 gpurun_out/r04v_pytest.log
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-live-pmc --serializer kryo"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04v -o run -- python3 $B \
    > gpurun_out/r04v_bench.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, json
f = glob.glob("gpurun_out/r04v/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "kryo" in r["Name"] or "gather_items" in r["Name"]:
        print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:10.1f} us')
d = [json.loads(l) for l in open("gpurun_out/r04v_bench.log") if l.startswith("{")][-1]
print(d["ms_per_step"], d["kryo"])
PY
