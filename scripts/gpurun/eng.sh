#!/bin/bash
# host ordering engine A/B (tools/engine_bench.py) over tool libraries in LIBS, configs in CFGS
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for c in ${CFGS:-3 4}; do
  for k in 1 2; do
    for lib in ${LIBS:-libkbg_tools_old.so libkbg_tools.so}; do
      echo -n "$lib "
      TOOLS_LIB=$R/kube-arbitrator_amd/tools/$lib REPS=${REPS:-5} timeout -k 10 300 python kube-arbitrator_amd/tools/engine_bench.py $c 2>&1 | tail -1
    done
  done
done
