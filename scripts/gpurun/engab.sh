#!/bin/bash
# Host ordering engine alone (tools/engine_bench.py), the tools library against
# variants (tools/variants/libkbg_tools_<name>.so), alternating, on the box's CPU.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in 1 2 3; do
  for L in kube-arbitrator_amd/tools/libkbg_tools.so ${VARIANTS}; do
    for c in ${CFGS:-3 4}; do
      echo -n "$L "; TOOLS_LIB=$L REPS=${REPS:-7} timeout -k 10 300 python kube-arbitrator_amd/tools/engine_bench.py $c 2>&1 | tail -1
    done
  done
done
