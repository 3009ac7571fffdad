#!/bin/bash
# GPU session: bench lines only (no CPU baselines); BENCH_ARGS / CONFIGS select the runs.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for c in ${CONFIGS:-3}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench_c$c.json 2> $O/bench_c$c.err
  cat $O/bench_c$c.json
done
