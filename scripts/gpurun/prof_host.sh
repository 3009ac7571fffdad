#!/bin/bash
# Host-side profile lines of the C3 allocate cycle (KBG_PROFILE_RESOLVE,
# KBG_PROFILE_ENGINE) over a short bench run. One GPU step under a time limit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-profhost}
mkdir -p $O
cd $R
KBG_PROFILE_RESOLVE=1 KBG_PROFILE_ENGINE=1 timeout -k 10 300 python bench.py --config ${CFG:-3} --steps 5 --warmup 2 --no-cpu-baseline ${EXTRA} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
grep "kbg resolve\|kbg engine" $O/bench.err | tail -12
python -c "
import json; d=json.load(open('$O/bench.json')); r=d.get('resident_session') or {}; print({k: r[k] for k in r if 'ms' in k})"
