#!/bin/bash
# Round-3 validation on one MI355X: GPU suite, default bench line, Kryo+LZ4 bench line, then
# the Kryo / LZ4 SQ counter passes that round 2's bench bug killed.
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03v
mkdir -p $o
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest.log 2>&1
tail -3 $o/pytest.log
timeout -k 10 300 python bench.py > $o/bench.log 2>&1
tail -c 600 $o/bench.log
timeout -k 10 300 python bench.py --serializer kryo --compress --no-cpu-baseline --steps 5 --warmup 1 > $o/bench_kryo_lz4.log 2>&1
tail -c 400 $o/bench_kryo_lz4.log
bash tools/ab/sq_kryo.sh r03v/sq_kryo
bash tools/ab/sq_lz4c.sh r03v/sq_lz4c
echo ALLDONE
