#!/bin/bash
# TeraSort K4 (512-record tiles, carries in LDS): the tree vs its stores computed but not issued.
tag=${1:-r05r}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
for n in 33554432 42949672; do
  A="--record-bytes 100 --records $n --iters 5"
  for i in 1 2; do
    timeout -k 10 180 python -u tools/prof_map.py $A > "$out/tree_${n}_$i.log" 2>&1 || fail "tree" "$out/tree_${n}_$i.log"
    echo "tree $n $(tail -1 $out/tree_${n}_$i.log)"
    timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_nostore.so prof_map $A > "$out/nostore_${n}_$i.log" 2>&1 || fail "nostore" "$out/nostore_${n}_$i.log"
    echo "nostore $n $(tail -1 $out/nostore_${n}_$i.log)"
  done
done
echo done > "$out/DONE"
