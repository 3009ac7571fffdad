#!/bin/bash
# rocprofv3 kernel trace + separate PMC passes of the C3 bench (scan kernel)
# and the C5 bench (victim kernel). Each pass is its own run under its own
# time limit; the script stops at the first failure. Outputs: gpurun_out/pmc/
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $O/counters.txt 2>&1 || true
SQ="SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"
SQW="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
for cfg in ${CFGS:-3 5}; do
  B="$R/bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-resident"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c${cfg}_kt -o kt --output-format csv -- python3 $B > $O/c${cfg}_kt_bench.json 2> $O/c${cfg}_kt.err
  echo "c$cfg kernel trace done"
  i=0
  for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "$SQ" "$SQW"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $pass -d $O/c${cfg}_pmc$i -o pmc$i --output-format csv -- python3 $B > $O/c${cfg}_pmc${i}_bench.json 2> $O/c${cfg}_pmc$i.err
    echo "c$cfg pmc pass $i ($pass) done"
  done
done
echo PMC_DONE
