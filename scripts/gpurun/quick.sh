#!/bin/bash
# GPU session: a subset of the parity tests (TESTS), then the C3 timelines.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_parity_gpu.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_quick.log 2>&1 || { tail -40 $O/pytest_quick.log; exit 1; }
tail -3 $O/pytest_quick.log
bash $R/scripts/gpurun/trace.sh
