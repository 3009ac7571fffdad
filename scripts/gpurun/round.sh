#!/bin/bash
# GPU session of a round: the -m gpu suite (TESTS / K select a part), smoke(),
# the driver's default bench command, optional extra bench configs (CFGS,
# e.g. "5 4") and the PMC passes (PMC=1, configs PMC_CFGS). Every GPU step has
# its own time limit; the script stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-r5}
mkdir -p $O
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TT:-900} python -u -m pytest ${TESTS:-tests} ${K:+-k "$K"} -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
if [ -z "$NO_SMOKE" ]; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; cat $O/bench.json; exit 1; }
  cat $O/bench.json
fi
for cfg in $CFGS; do
  timeout -k 10 600 python bench.py --config $cfg ${CFG_ARGS:---steps 10 --warmup 2 --no-cpu-baseline} > $O/bench_c$cfg.json 2> $O/bench_c$cfg.err || { tail -30 $O/bench_c$cfg.err; cat $O/bench_c$cfg.json; exit 1; }
  cat $O/bench_c$cfg.json
done
if [ -n "$PMC" ]; then
  CFGS=${PMC_CFGS:-3} bash $R/scripts/gpurun/pmc.sh
fi
echo ROUND_DONE
