#!/bin/bash
# C4 (20k nodes x 500k tasks) on one GPU: bench line without the CPU baseline
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --config 4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
cat gpurun_out/bench_c4.json
