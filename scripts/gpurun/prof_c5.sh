#!/bin/bash
# C5 victim-path parity, then a rocprofv3 kernel trace of the C5 bench (summary: profiles/summarize.py).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/prof_c5
cd $R
export TMPDIR=/tmp
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "victim or contended or config5 or dupkey" > $O/pytest_c5.log 2>&1 || { tail -60 $O/pytest_c5.log; exit 1; }
tail -3 $O/pytest_c5.log
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 -- python bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_c5/bench.json 2> $O/prof_c5/bench.err
cat $O/prof_c5/bench.json
