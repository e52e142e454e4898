#!/bin/bash
# Round-3 validation on one MI355X: GPU suite, default bench line, C3 split vs single pass,
# Kryo+LZ4 bench line, then the Kryo / LZ4 SQ counter passes that round 2's bench bug killed.
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03v
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
timeout -k 10 300 python bench.py > $o/bench.log 2>&1
tail -c 300 $o/bench.log
timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline > $o/bench_c3.log 2>&1
timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline --no-split > $o/bench_c3_nosplit.log 2>&1
timeout -k 10 200 python bench.py --workload c3 --dist uniform --no-cpu-baseline > $o/bench_c3u.log 2>&1
timeout -k 10 200 python bench.py --workload c3 --dist uniform --no-cpu-baseline --no-split > $o/bench_c3u_nosplit.log 2>&1
for f in bench_c3 bench_c3_nosplit bench_c3u bench_c3u_nosplit; do python -c "
import json,sys; d=json.loads([l for l in open('$o/$f.log') if l.startswith('{')][0]); print('$f', d['value'], d['stages_ms_per_step'])"; done
timeout -k 10 300 python bench.py --serializer kryo --compress --no-cpu-baseline --steps 5 --warmup 1 > $o/bench_kryo_lz4.log 2>&1
bash tools/ab/sq_kryo.sh r03v/sq_kryo
bash tools/ab/sq_lz4c.sh r03v/sq_lz4c
echo ALLDONE
