#!/bin/bash
# A/B of a host-side switch (VAR=NAME, values A and B; '-' = unset) on the C3 bench, 3
# alternating runs each, after the parity tests. Each step has its own time
# limit; stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-hostab}
mkdir -p $O
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for i in 1 2 3; do
  for v in ${A:-1} ${B:-0}; do
    if [ "$v" = "-" ]; then SETV="-u $VAR"; else SETV="$VAR=$v"; fi
    env $SETV timeout -k 10 300 python bench.py --config ${CFG:-3} --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${EXTRA} > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail -30 $O/b_${v}_$i.err; exit 1; }
    python -c "
import json,sys; d=json.load(open('$O/b_${v}_$i.json')); b=d['production_mode']['breakdown']; r=d.get('resident_session') or {}
print('$VAR=$v', round(d['value']/1e6,2), 'p50', round(d['p50_cycle_ms'],3), 'eng', round(b['host_engine_ms'],2), 'res', round(b['host_resolve_ms'],2), 'rk', b['resolve_rechecks'], 'ov', b['overlapped_batches'], 'dev', round(b['device_roundtrip_ms'],2), 'churn', r.get('churn_allocate_ms_p50'), 'parity', d['parity']['ok'])"
  done
done
echo HOSTAB_DONE
