#!/bin/bash
# TeraSort K4 probes: K4 with its stores computed but not issued (nostore) vs the tree vs HEAD~1.
tag=${1:-r05n}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fail() { echo "$1"; tail -40 "$2"; exit 1; }
A="--record-bytes 100 --records 42949672 --iters 5"
for i in 1 2; do
  timeout -k 10 180 python -u tools/prof_map.py $A > "$out/tree_$i.log" 2>&1 || fail "tree" "$out/tree_$i.log"
  echo "tree $(tail -1 $out/tree_$i.log)"
  for v in ${VARIANTS:-nostore old}; do
    timeout -k 10 180 python -u tools/ab_run.py tools/ab/libsgx_$v.so prof_map $A > "$out/${v}_$i.log" 2>&1 || fail "$v" "$out/${v}_$i.log"
    echo "$v $(tail -1 $out/${v}_$i.log)"
  done
done
echo done > "$out/DONE"
