#!/bin/bash
# GPU session: the new round-2 tests first (resident sessions), then the whole GPU suite, then the bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_update_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_update.log 2>&1 || { tail -60 $O/pytest_update.log; exit 1; }
tail -3 $O/pytest_update.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_update_gpu.py > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
cat $O/bench.json
