#!/bin/bash
# Kryo padded write: kernel-time split of the serializer (padded vs two-pass records).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kryo.py \
    > gpurun_out/r04u_pytest.log 2>&1 || { tail -30 gpurun_out/r04u_pytest.log; exit 1; }
tail -1 gpurun_out/r04u_pytest.log
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-live-pmc --serializer kryo"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04u_pad -o run -- python3 $B \
    > gpurun_out/r04u_pad.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04u_two -o run -- python3 $B --no-padded \
    > gpurun_out/r04u_two.log 2>&1 || exit 1
for d in pad two; do
  f=$(find gpurun_out/r04u_$d -name '*kernel_stats.csv' | head -1)
  echo "== $d"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:10.1f} us')
PY
done
