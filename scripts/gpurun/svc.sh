#!/bin/bash
# The C3 bench on one GPU three ways: single-GPU session, the scan service on a
# one-rank RCCL communicator (KBG_SCAN_SERVICE=1 --comm: rank 0's message,
# broadcast, sum and copy-back costs without peers), owner-resolve on it.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-svc}
mkdir -p $O
cd $R
A="--config ${CONFIG:-3} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-resident"
timeout -k 10 300 python bench.py $A > $O/single.json 2> $O/single.err || { tail -20 $O/single.err; exit 1; }
KBG_SCAN_SERVICE=1 timeout -k 10 300 python bench.py $A --comm > $O/svc.json 2> $O/svc.err || { tail -20 $O/svc.err; exit 1; }
KBG_OWNER_RESOLVE=1 timeout -k 10 300 python bench.py $A --comm > $O/owner.json 2> $O/owner.err || { tail -20 $O/owner.err; exit 1; }
for f in single svc owner; do
  python -c "import json,sys; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); b=d['production_mode']['breakdown']; print('$f', round(d['p50_cycle_ms'],2), {k: (round(b[k],2) if isinstance(b[k], float) else b[k]) for k in ('host_engine_ms','host_resolve_ms','device_roundtrip_ms','exchange_ms','launches','batches','mispredictions')})"
done
