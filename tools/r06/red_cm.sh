#!/bin/bash
# Round 6: reduce side and the one-rank peer-gather exchange on the chunk-major layout (tree)
# against the partition-major build (pm)
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
bash tools/r06/red.sh $tag tree pm || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --self-exchange --no-cpu-baseline --no-live-pmc --steps 20 > "$out/selfx_tree_$rep.log" 2>&1 || exit $?
  timeout -k 10 300 python -u tools/ab_run.py tools/ab/libsgx_pm.so bench --self-exchange --no-cpu-baseline --no-live-pmc --steps 20 > "$out/selfx_pm_$rep.log" 2>&1 || exit $?
  for l in tree pm; do grep -h '^{' "$out/selfx_${l}_$rep.log" | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('selfx', '$l', $rep, j['value'], j['ms_per_step'], j.get('step_design_hbm'))"; done
done
