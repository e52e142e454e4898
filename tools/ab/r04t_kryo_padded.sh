#!/bin/bash
# Kryo padded write: GPU tests of the Kryo / LZ4 / padded paths, then the Kryo bench with the
# padded write (default) and without (--no-padded), interleaved.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_kryo.py tests/test_padded.py tests/test_lz4.py tests/test_import_blocks.py \
    > gpurun_out/r04t_pytest.log 2>&1 || { tail -30 gpurun_out/r04t_pytest.log; exit 1; }
tail -2 gpurun_out/r04t_pytest.log
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-live-pmc --serializer kryo"
for i in 1; do
  timeout -k 10 180 $B > gpurun_out/r04t_kryo_pad_$i.log 2>&1 || exit 1
  timeout -k 10 180 $B --no-padded > gpurun_out/r04t_kryo_twopass_$i.log 2>&1 || exit 1
  timeout -k 10 180 $B --compress > gpurun_out/r04t_kryo_lz4_pad_$i.log 2>&1 || exit 1
  timeout -k 10 180 $B --compress --no-padded > gpurun_out/r04t_kryo_lz4_twopass_$i.log 2>&1 || exit 1
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r04t_kryo_*.log")):
    d = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(f, d["ms_per_step"], d.get("roofline_map_side", {}).get("ms"), d.get("kryo", {}).get("ms"),
          d.get("map_layout", d.get("config", {}).get("map_layout")))
PY
