#!/bin/bash
# phase shares of the write-combining K4 (stamp build), C1 and smaller R
set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r03_stamps2; mkdir -p $o
for R in 1024 64; do
  timeout -k 10 120 python -u tools/ab_run.py tools/ab/libsgx_stamps.so wc_stamps --partitions $R >> $o/stamps.jsonl 2>> $o/err.log
done
timeout -k 10 120 python -u tools/ab_run.py tools/ab/libsgx_stamps.so wc_stamps --partitions 1024 --dist zipf >> $o/stamps.jsonl 2>> $o/err.log
cat $o/stamps.jsonl
