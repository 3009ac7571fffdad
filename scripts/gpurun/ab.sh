#!/bin/bash
# A/B of library builds / environments on one box (tools/ab_bench.py); ARGS:
# the variants (lib.so[@KEY=VAL...]); CONFIG / REPS / STEPS as ab_bench.py.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-ab}
mkdir -p $O
cd $R
timeout -k 10 ${TT:-900} python -u kube-arbitrator_amd/tools/ab_bench.py "$@" > $O/ab.txt 2>&1 || { tail -30 $O/ab.txt; exit 1; }
cat $O/ab.txt
