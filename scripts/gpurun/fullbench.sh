#!/bin/bash
# GPU session: full bench lines (CPU baselines included) for the configs in CONFIGS.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/full
mkdir -p $O
cd $R
for c in ${CONFIGS:-1 2 3}; do
  timeout -k 10 ${T:-500} python bench.py --config $c --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > $O/bench_c$c.json 2> $O/bench_c$c.err
  echo "C$c done"
done
