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
if [ -n "$TESTS" ]; then  # a part of the -m gpu suite first (e.g. a host-engine change)
  timeout -k 10 ${TT:-600} python -u -m pytest $TESTS ${K:+-k "$K"} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_b.log 2>&1 || { tail -40 $O/pytest_b.log; exit 1; }
  tail -2 $O/pytest_b.log
fi
if [ -n "$RPROF_FIRST" ]; then
  KBG_PROFILE_RESOLVE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-resident > $O/rprof_c3.json 2> $O/rprof_c3.err || { tail -20 $O/rprof_c3.err; exit 1; }
  grep -i "resolve" $O/rprof_c3.err | tail -4; python -c "import json;d=json.loads(open('$O/rprof_c3.json').read().strip().splitlines()[-1]);print(d['value'],d['p50_cycle_ms'],d['parity']['ok'],d['production_mode']['breakdown'])"
fi
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
