#!/bin/bash
# GPU session: allocate-cycle timelines (KBG_TRACE) of C3, production and full-scan mode.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-trace}
mkdir -p $O
cd $R
for full in ${FULL:-0 1}; do
  timeout -k 10 120 python kube-arbitrator_amd/tools/trace_cycle.py ${CONFIG:-3} $full > $O/c${CONFIG:-3}_full$full.txt 2> $O/c${CONFIG:-3}_full$full.trace
  cat $O/c${CONFIG:-3}_full$full.txt
done
