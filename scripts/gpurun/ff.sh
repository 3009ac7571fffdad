#!/bin/bash
# The fused first-fit kernel alone (tools/ff_bench.py: event-timed launches
# by batch size) and its phase stamps (tools/ff_stamps.py, the diagnostic
# build). Each step has its own time limit; stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-ff}
mkdir -p $O
cd $R
timeout -k 10 240 python kube-arbitrator_amd/tools/ff_bench.py ${CONFIG:-3} > $O/ff_bench.json 2> $O/ff_bench.err || { tail -20 $O/ff_bench.err; exit 1; }
cat $O/ff_bench.json
timeout -k 10 240 python kube-arbitrator_amd/tools/ff_stamps.py ${CONFIG:-3} > $O/ff_stamps.json 2> $O/ff_stamps.err || { tail -20 $O/ff_stamps.err; exit 1; }
cat $O/ff_stamps.json
