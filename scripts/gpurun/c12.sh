#!/bin/bash
# C1 (100 nodes x 1k tasks) and C2 (1k nodes x 10k tasks) on one GPU: bench
# lines with the CPU baselines (parity-side configs of BASELINE.json).
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for c in 1 2; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err
  cat gpurun_out/bench_c$c.json
done
