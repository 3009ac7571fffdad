#!/bin/bash
# Round-3 GPU session: full -m gpu suite, smoke, the driver's default bench
# command, then (PMC=1) the rocprofv3 kernel trace + PMC passes of C3.
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3
mkdir -p $O
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TT:-720} python -u -m pytest ${TESTS:-tests} ${K:+-k "$K"} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
if [ -n "$PMC" ]; then
  CFGS=${CFGS:-3} bash $R/scripts/gpurun/pmc.sh
fi
echo R3_DONE
