#!/bin/bash
# Where the Zipf reduceByKey's sort stage goes: kernel trace of tools/prof_reduce.py sum:zipf
# next to sorted:uniform.
tag=${1:-r05ap}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in sum:zipf sorted:uniform; do
  n=${c/:/_}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$n" -o run -- python3 tools/prof_reduce.py --cases $c --iters 3 > "$out/$n.log" 2>&1 || { echo "fail $c"; tail -20 "$out/$n.log"; exit 1; }
done
echo done > "$out/DONE"
