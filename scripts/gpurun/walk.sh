#!/bin/bash
# Resolver walk A/B (tools/ab_bench.py over LIBS) and the walk histogram
# (KBG_PROFILE_RESOLVE). Each step has its own time limit; stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/walk
mkdir -p $O
cd $R
KBG_PROFILE_RESOLVE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-resident > $O/rprof.json 2> $O/rprof.err || { tail -20 $O/rprof.err; exit 1; }
grep "kbg resolve" $O/rprof.err | tail -4
if [ -n "$LIBS" ]; then
  timeout -k 10 900 python kube-arbitrator_amd/tools/ab_bench.py $LIBS > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
  tail -8 $O/ab.txt
fi
echo WALK_DONE
