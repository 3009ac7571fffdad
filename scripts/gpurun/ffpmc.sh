#!/bin/bash
# first-fit kernel experiments: ff_bench timing per tool library (LIBS), then
# one PMC pass (VALU, waves, LDS, SALU) of ff_bench per library in PMCLIBS.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ffpmc
mkdir -p $O
cd $R
for lib in ${LIBS:-libkbg_tools.so}; do
  TOOLS_LIB=$R/kube-arbitrator_amd/tools/$lib timeout -k 10 180 python kube-arbitrator_amd/tools/ff_bench.py ${CFG:-3} > $O/ff_$lib.json 2> $O/ff_$lib.err || { tail -20 $O/ff_$lib.err; exit 1; }
  echo "$lib $(cat $O/ff_$lib.json)"
done
cd /tmp && export TMPDIR=/tmp
IFS='|' read -ra SETS <<< "${PMCSETS:-SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES}"
for lib in ${PMCLIBS}; do
  k=0
  for set in "${SETS[@]}"; do
    k=$((k+1))
    TOOLS_LIB=$R/kube-arbitrator_amd/tools/$lib timeout -s KILL 120 rocprofv3 --pmc $set -d $O/pmc_${lib}_$k -o pmc --output-format csv -- python3 $R/kube-arbitrator_amd/tools/ff_bench.py ${CFG:-3} > $O/pmc_${lib}_$k.out 2> $O/pmc_${lib}_$k.err || { tail -20 $O/pmc_${lib}_$k.err; exit 1; }
    echo "pmc $lib set $k done"
  done
done
echo FFPMC_DONE
