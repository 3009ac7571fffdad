#!/bin/bash
# GPU session for C5 (contended cluster: reclaim, allocate, backfill, preempt):
# bench line, then a rocprofv3 kernel trace of the same command. PMC=1 adds
# the FETCH_SIZE / WRITE_SIZE passes. Each GPU step has its own time limit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --config 5 --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS} > $O/bench_c5.json 2> $O/bench_c5.err
cat $O/bench_c5.json
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5_kt -o kt --output-format csv -- python3 $B > $O/prof_c5_kt_bench.json 2> $O/prof_c5_kt.err
if [ -n "$PMC" ]; then
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_c5_pmc1 -o pmc1 --output-format csv -- python3 $B > $O/prof_c5_pmc1_bench.json 2> $O/prof_c5_pmc1.err
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_c5_pmc2 -o pmc2 --output-format csv -- python3 $B > $O/prof_c5_pmc2_bench.json 2> $O/prof_c5_pmc2.err
fi
echo PROFILES_DONE
