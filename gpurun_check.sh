#!/bin/bash
# GPU session: parity tests then one bench line. Stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err
cat $O/bench.json
