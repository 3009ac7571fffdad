#!/bin/bash
# C4 probes: the predictor's checkpoint copies in one cycle's timeline
# (KBG_TRACE), and an A/B of the early-emit size (KBG_MIN_EMIT) on the C4 bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/c4p
mkdir -p $O
cd $R
timeout -k 10 300 python kube-arbitrator_amd/tools/trace_cycle.py 4 0 > $O/c4_full0.txt 2> $O/c4_full0.trace || { tail -20 $O/c4_full0.trace; exit 1; }
cat $O/c4_full0.txt
L=kube-arbitrator_amd/kbgpu/libkbgpu.so
CONFIG=4 REPS=2 timeout -k 10 900 python kube-arbitrator_amd/tools/ab_bench.py $L $L@KBG_MIN_EMIT=2048 $L@KBG_MIN_EMIT=8192 > $O/ab_emit.txt 2>&1 || { tail -20 $O/ab_emit.txt; exit 1; }
tail -1 $O/ab_emit.txt
echo C4P_DONE
