#!/bin/bash
# rocprofv3 kernel statistics of the C3 and C4 benches (the
# kernels' average launch durations behind the bench lines' roofline objects).
# Each step has its own time limit; stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-kstats}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-3 4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt$cfg -o kt --output-format csv -- python3 $R/bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-resident > $O/kt_bench_c$cfg.json 2> $O/kt_c$cfg.err || { tail -20 $O/kt_c$cfg.err; exit 1; }
done
echo R4PROF_DONE
