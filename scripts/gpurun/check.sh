#!/bin/bash
# GPU session: parity tests then bench lines. Stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
T=${TESTS:-tests}
timeout -k 10 700 python -u -m pytest $T ${K:+-k "$K"} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
if [ -n "$BENCH_COMM" ]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --comm --no-cpu-baseline > $O/bench_comm.json 2> $O/bench_comm.err
  cat $O/bench_comm.json
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err
  cat $O/bench.json
fi
