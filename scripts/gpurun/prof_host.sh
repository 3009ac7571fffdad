#!/bin/bash
# GPU session: bench with the host-side cycle counters on (engine and commit), stderr kept.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
lscpu | head -20 > $O/lscpu.txt || true
KBG_PROFILE_RESOLVE=1 KBG_PROFILE_ENGINE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
grep -E "kbg (resolve|engine)" $O/bench_prof.err | tail -12
python -c "import json;d=json.load(open('$O/bench_prof.json'));print(d['p50_cycle_ms'], d['full_scan_mode']['p50_cycle_ms'])"
