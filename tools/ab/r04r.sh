#!/bin/bash
# Round 4, run r: Kryo benches after bench.py commits every step's map (LZ4 framing inside the step)
set -e
tag=${1:-r04r}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench.py --serializer kryo --compress --steps 5 --warmup 2 --no-cpu-baseline > "$out/bench_kryo_lz4.log" 2>&1
timeout -k 10 300 python -u bench.py --serializer kryo --no-cpu-baseline > "$out/bench_kryo.log" 2>&1
for f in bench_kryo_lz4 bench_kryo; do
  grep '^{' "$out/$f.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$f', j['value'], j['ms_per_step'], j['stages_ms_per_step'])"
done
echo done > "$out/DONE"
