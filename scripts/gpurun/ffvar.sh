#!/bin/bash
# Kernel variants (tools/build_variants.sh) timed by tools/ff_bench.py, twice
# each alternating, then the phase stamps of the shipped kernel. Each step
# has its own time limit; stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-ffvar}
mkdir -p $O
cd $R
for i in 1 2; do
for lib in kube-arbitrator_amd/tools/variants/libkbg_tools_*.so; do
  n=$(basename $lib .so)
  TOOLS_LIB=$R/$lib timeout -k 10 240 python kube-arbitrator_amd/tools/ff_bench.py ${CONFIG:-3} > $O/$n.$i.json 2> $O/$n.$i.err || { tail -20 $O/$n.$i.err; exit 1; }
  echo "$n $(cat $O/$n.$i.json)"
done
done
for kv in "" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0"; do
  env $kv timeout -k 10 240 python kube-arbitrator_amd/tools/ff_bench.py ${CONFIG:-3} > $O/kernarg.json 2> $O/kernarg.err || { tail -20 $O/kernarg.err; exit 1; }
  echo "kernarg[$kv] $(cat $O/kernarg.json)"
done
timeout -k 10 240 python kube-arbitrator_amd/tools/ff_stamps.py ${CONFIG:-3} > $O/ff_stamps.json 2> $O/ff_stamps.err || { tail -20 $O/ff_stamps.err; exit 1; }
cat $O/ff_stamps.json
echo FFVAR_DONE
