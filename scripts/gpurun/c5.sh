#!/bin/bash
# GPU session: victim-action parity (contended / C5 scaled), then the C5 bench line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "victim or contended or config5 or dupkey" > $O/pytest_c5.log 2>&1 || { tail -60 $O/pytest_c5.log; exit 1; }
tail -3 $O/pytest_c5.log
timeout -k 10 400 python bench.py --config 5 --steps 5 --warmup 1 ${C5_ARGS:---no-cpu-baseline} > $O/bench_c5.json 2> $O/bench_c5.err
cat $O/bench_c5.json
