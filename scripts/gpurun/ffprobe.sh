#!/bin/bash
# Fused first-fit kernel probes: phase stamps (tools/ff_stamps.py over the
# stamp builds in STAMP_LIBS) and launch times (tools/ff_bench.py over LIBS).
# Each step has its own time limit; the script stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ff
mkdir -p $O
cd $R
for lib in ${STAMP_LIBS:-libkbg_tools_stamps.so}; do
  TOOLS_LIB=$R/kube-arbitrator_amd/tools/$lib timeout -k 10 240 python kube-arbitrator_amd/tools/ff_stamps.py ${CFG:-3} > $O/stamps_$lib.json 2> $O/stamps_$lib.err || { tail -20 $O/stamps_$lib.err; exit 1; }
  echo "== stamps $lib"; cat $O/stamps_$lib.json
done
for lib in ${LIBS:-libkbg_tools.so}; do
  TOOLS_LIB=$R/kube-arbitrator_amd/tools/$lib timeout -k 10 240 python kube-arbitrator_amd/tools/ff_bench.py ${CFG:-3} > $O/ff_$lib.json 2> $O/ff_$lib.err || { tail -20 $O/ff_$lib.err; exit 1; }
  echo "== ff_bench $lib $(cat $O/ff_$lib.json)"
done
echo FFPROBE_DONE
