#!/bin/bash
# Round-4 session C: launch-cost probe, A/B of the commit-overlap change on C3
# and C4 (LIBS), PMC of C3. Each step has its own time limit; stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4c
mkdir -p $O
cd $R
timeout -k 10 200 python kube-arbitrator_amd/tools/launch_cost.py 3 > $O/launch_cost.json 2> $O/launch_cost.err || { tail -20 $O/launch_cost.err; exit 1; }
cat $O/launch_cost.json
if [ -n "$LIBS" ]; then
  CONFIG=3 timeout -k 10 600 python kube-arbitrator_amd/tools/ab_bench.py $LIBS > $O/ab_c3.txt 2>&1 || { tail -20 $O/ab_c3.txt; exit 1; }
  tail -1 $O/ab_c3.txt
  CONFIG=4 REPS=2 timeout -k 10 700 python kube-arbitrator_amd/tools/ab_bench.py $LIBS > $O/ab_c4.txt 2>&1 || { tail -20 $O/ab_c4.txt; exit 1; }
  tail -1 $O/ab_c4.txt
fi
if [ -z "$NO_PMC" ]; then
  CFGS=3 bash $R/scripts/gpurun/pmc.sh
fi
echo R4C_DONE
