#!/bin/bash
# Round-4 session D: GPU parity of the current tree (TESTS), then A/B of LIBS
# on C4 and C3. Each step has its own time limit; stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4d
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest ${TESTS:-tests} -m "${MARK:-gpu}" -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
if [ -n "$LIBS" ]; then
  CONFIG=4 REPS=${REPS4:-3} timeout -k 10 700 python kube-arbitrator_amd/tools/ab_bench.py $LIBS > $O/ab_c4.txt 2>&1 || { tail -20 $O/ab_c4.txt; exit 1; }
  tail -3 $O/ab_c4.txt
  CONFIG=3 timeout -k 10 400 python kube-arbitrator_amd/tools/ab_bench.py $LIBS > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
  tail -3 $O/ab_c3.txt
fi
echo R4D_DONE
