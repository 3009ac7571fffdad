#!/bin/bash
# Round-4 GPU session B: the PMC passes (scripts/gpurun/pmc.sh, configs
# PMC_CFGS), the C4 bench line, allocate-cycle timelines (KBG_TRACE) and the
# session-open phases. Each step has its own time limit; the script stops at
# the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
if [ -z "$NO_PMC" ]; then
  CFGS=${PMC_CFGS:-"3 5"} bash $R/scripts/gpurun/pmc.sh
fi
if [ -z "$NO_C4" ]; then
  timeout -k 10 420 python bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -30 $O/bench_c4.err; exit 1; }
  cat $O/bench_c4.json
fi
if [ -z "$NO_TRACE" ]; then
  bash $R/scripts/gpurun/trace.sh
  timeout -k 10 180 python tools/open_profile.py 3 > $O/open_c3.txt 2>&1 || { tail -20 $O/open_c3.txt; exit 1; }
  tail -30 $O/open_c3.txt
fi
if [ -z "$NO_RPROF" ]; then  # in-order commit cycle counters (KBG_PROFILE_RESOLVE), C3 production
  KBG_PROFILE_RESOLVE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-resident > $O/rprof_c3.json 2> $O/rprof_c3.err || { tail -20 $O/rprof_c3.err; exit 1; }
  grep -i "resolve" $O/rprof_c3.err | tail -6
fi
echo R4B_DONE
