#!/bin/bash
# Kernel experiment builds (kube-arbitrator_amd/tools/build_variants.sh) timed by
# tools/ff_bench.py, one library per run, each under its own time limit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-variants}
mkdir -p $O
cd $R
for lib in kube-arbitrator_amd/tools/variants/libkbg_tools_*.so; do
  n=$(basename $lib .so)
  TOOLS_LIB=$R/$lib timeout -k 10 240 python kube-arbitrator_amd/tools/ff_bench.py ${CONFIG:-3} > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  echo "$n $(cat $O/$n.json)"
done
