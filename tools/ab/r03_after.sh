#!/bin/bash
# Grouping tests + reduce A/B (base = 445cadb), then the C1 K4 A/B of SGX_WC_LATE=0.
set -e
cd $GRAFT_REPO_ROOT
bash tools/ab/r03_grp.sh
bash tools/ab/r03_c1_ab.sh late "tree late0"
