#!/bin/bash
# A/B of an environment switch (AB_ENV, e.g. KBG_NO_REFRESH=1) on the default
# bench, alternating ROUNDS times on one box; prints value and p50 per run.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
for k in $(seq 1 ${ROUNDS:-2}); do
  for v in A B; do
    if [ $v = B ]; then E="$AB_ENV"; else E=""; fi
    env $E timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-resident ${BENCH_ARGS} > $O/b_$v$k.json 2> $O/b_$v$k.err
    python -c "
import json; d=json.load(open('$O/b_$v$k.json')); b=d['production_mode']['breakdown']
print('$v$k', '$E', 'value', round(d['value']/1e6,3), 'p50', round(d['p50_cycle_ms'],3), 'mispred', b['mispredictions'], 'trunc', b['truncations'], 'full p50', round(d['full_scan_mode']['p50_cycle_ms'],3))"
  done
done
