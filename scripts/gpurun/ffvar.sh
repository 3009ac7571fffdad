#!/bin/bash
# Kernel variants (tools/build_variants.sh) timed by tools/ff_bench.py, twice
# each alternating, then the phase stamps of the shipped kernel. Each step
# has its own time limit; stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-ffvar}
mkdir -p $O
cd $R
for i in 1 2; do
for lib in kube-arbitrator_amd/tools/variants/libkbg_tools_*.so; do
  n=$(basename $lib .so)
  TOOLS_LIB=$R/$lib timeout -k 10 240 python kube-arbitrator_amd/tools/ff_bench.py ${CONFIG:-3} > $O/$n.$i.json 2> $O/$n.$i.err || { tail -20 $O/$n.$i.err; exit 1; }
  echo "$n $(cat $O/$n.$i.json)"
done
done
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 240 python kube-arbitrator_amd/tools/ff_stamps.py ${CONFIG:-3} > $O/ff_stamps.json 2> $O/ff_stamps.err || { tail -20 $O/ff_stamps.err; exit 1; }
cat $O/ff_stamps.json
echo FFVAR_DONE
