#!/bin/bash
# In-cycle profiles of the C3 allocate cycle: the ordering engine's cycles per
# step (KBG_PROFILE_ENGINE) and the in-order commit's (KBG_PROFILE_RESOLVE).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-engprof}
mkdir -p $O
cd $R
KBG_PROFILE_ENGINE=1 KBG_PROFILE_RESOLVE=1 timeout -k 10 300 python bench.py --config ${CONFIG:-3} --steps 8 --warmup 2 --no-cpu-baseline --no-resident > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep "kbg engine\|kbg resolve" $O/bench.err | tail -12
