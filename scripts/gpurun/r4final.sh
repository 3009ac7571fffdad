#!/bin/bash
# Round-4 final measurements of the tree: the driver's bench command (C3, with
# the CPU baselines), C4 and C5 lines, the kernel statistics of a C3 bench
# (rocprofv3 --kernel-trace --stats) and a C4 cycle timeline. Each step has its
# own time limit; the script stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final
mkdir -p $O
cd $R
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail -30 $O/bench_c3.err; exit 1; }
tail -c 400 $O/bench_c3.json
for cfg in 4 5; do
  timeout -k 10 600 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c$cfg.json 2> $O/bench_c$cfg.err || { tail -30 $O/bench_c$cfg.err; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-resident > $O/kt_bench.json 2> $O/kt.err || { tail -20 $O/kt.err; exit 1; }
cd $R
timeout -k 10 300 python kube-arbitrator_amd/tools/trace_cycle.py 4 0 > $O/c4_trace.txt 2> $O/c4_trace.log || { tail -20 $O/c4_trace.log; exit 1; }
cat $O/c4_trace.txt
echo FINAL_DONE
