#!/bin/bash
# K4 phase stamps (16 B padded write, C1) for the chunk-major tree and a partition-major build
set -e
tag=$1; o=gpurun_out/$tag; mkdir -p $o
for v in stamps stamps_pm stamps stamps_pm; do
  timeout -k 10 150 python3 -u tools/ab_run.py tools/ab/libsgx_$v.so wc_stamps --iters 3 >> $o/$v.jsonl
done
timeout -k 10 150 python3 -u tools/ab_run.py tools/ab/libsgx_stamps.so wc_stamps --iters 3 --partitions 4096 --dist zipf >> $o/stamps_c3.jsonl
echo DONE
