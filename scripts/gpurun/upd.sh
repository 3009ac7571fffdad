#!/bin/bash
# A/B of kbg_session_update on the C4 resident-session line: libraries in LIBS
# (KBG_LIB_PATH), alternating ROUNDS times on one box; prints the update phases
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/upd
mkdir -p $O
cd $R
for k in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS:-libkbgpu_old.so libkbgpu.so}; do
    KBG_LIB_PATH=$R/kube-arbitrator_amd/kbgpu/$lib KBG_PROFILE_OPEN=1 timeout -k 10 300 python bench.py --config ${CFG:-4} --steps 3 --warmup 1 --no-cpu-baseline --no-faithful > $O/$lib.$k.json 2> $O/$lib.$k.err
    python - $O/$lib.$k.json $O/$lib.$k.err $lib <<'PY'
import json, re, sys, statistics
d = json.load(open(sys.argv[1])); r = d["resident_session"]
err = open(sys.argv[2]).read()
ev = [float(x) for x in re.findall(r"\[kbg update\] events\s+([\d.]+)", err)][-5:]
dv = [float(x) for x in re.findall(r"\[kbg update\] derive\s+([\d.]+)", err)][-5:]
print(sys.argv[3], "update p50", round(r["churn_update_ms_p50"], 3), r["churn_update_ms"], "events", ev, "derive", dv, "cycle p50", round(d["p50_cycle_ms"], 3))
PY
  done
done
