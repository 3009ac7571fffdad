#!/bin/bash
# A/B of the fused first-fit kernel (tools/ff_bench.py) over tool libraries
# named in LIBS, then a parity subset (TESTS). Stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ff
mkdir -p $O
cd $R
for lib in ${LIBS:-libkbg_tools_base.so libkbg_tools.so}; do
  TOOLS_LIB=$R/kube-arbitrator_amd/tools/$lib timeout -k 10 180 python kube-arbitrator_amd/tools/ff_bench.py ${CFG:-3} > $O/ff_$lib.json 2> $O/ff_$lib.err || { tail -20 $O/ff_$lib.err; exit 1; }
  echo "$lib $(cat $O/ff_$lib.json)"
done
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS ${K:+-k "$K"} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
echo FF_DONE
