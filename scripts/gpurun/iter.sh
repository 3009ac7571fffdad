#!/bin/bash
# Iteration session: a parity subset (TESTS), the C3 cycle timelines, then a
# bench line without CPU baselines. Stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/iter
mkdir -p $O
cd $R
timeout -k 10 ${TT:-600} python -u -m pytest ${TESTS:-tests/test_parity_gpu.py tests/test_scale_gpu.py} ${K:+-k "$K"} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
if [ -z "$NO_TRACE" ]; then bash $R/scripts/gpurun/trace.sh; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json'))
b=d['production_mode']['breakdown']
print('value', round(d['value']/1e6,3), 'M/s p50', round(d['p50_cycle_ms'],3), 'ms; engine', round(b['host_engine_ms'],3), 'resolve', round(b['host_resolve_ms'],3), 'mispred', b['mispredictions'], 'trunc', b['truncations'], 'batches', b['batches'])
r=d['roofline']; print('roofline frac', round(r['frac'],3), 'avg us', round(r['avg_launch_us'],2), 'rows', round(r['rows_per_launch']), 'binding', r.get('binding',{}).get('frac'), 'cycle8d', round(d['cycle_roofline_8d']['frac'],3))
print('resident', d.get('resident_session',{}).get('churn_update_ms_p50'), d.get('resident_session',{}).get('churn_allocate_ms_p50'))
"
echo ITER_DONE
