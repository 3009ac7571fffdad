#!/bin/bash
# GPU session: bench (with the CPU baseline), then rocprofv3 kernel trace and
# separate PMC passes of the same bench command. Each GPU step has its own
# time limit; the script stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_kt -o kt --output-format csv -- python3 $B > $O/prof_kt_bench.json 2> $O/prof_kt.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_pmc1 -o pmc1 --output-format csv -- python3 $B > $O/prof_pmc1_bench.json 2> $O/prof_pmc1.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_pmc2 -o pmc2 --output-format csv -- python3 $B > $O/prof_pmc2_bench.json 2> $O/prof_pmc2.err
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/prof_pmc3 -o pmc3 --output-format csv -- python3 $B > $O/prof_pmc3_bench.json 2> $O/prof_pmc3.err
echo PROFILES_DONE
