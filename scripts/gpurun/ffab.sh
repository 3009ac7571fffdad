#!/bin/bash
# A/B of the fused kernel's complete-walk variant against the round-5 staged
# extraction (KBG_FF_STAGED=1): tools/ff_bench.py alternating, then parity
# tests. Each step has its own time limit; stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-ffab}
mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 240 python kube-arbitrator_amd/tools/ff_bench.py ${CONFIG:-3} > $O/ff_new_$i.json 2> $O/ff_new_$i.err || { tail -20 $O/ff_new_$i.err; exit 1; }
  echo "new   $(cat $O/ff_new_$i.json)"
  KBG_FF_STAGED=1 timeout -k 10 240 python kube-arbitrator_amd/tools/ff_bench.py ${CONFIG:-3} > $O/ff_old_$i.json 2> $O/ff_old_$i.err || { tail -20 $O/ff_old_$i.err; exit 1; }
  echo "staged $(cat $O/ff_old_$i.json)"
done
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-resident > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['p50_cycle_ms'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['parity']['ok'])"
fi
echo FFAB_DONE
