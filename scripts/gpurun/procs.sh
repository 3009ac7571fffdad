#!/bin/bash
# Multi-process rehearsal of the sharded path on one GPU: the slow C3 proc
# tests, then bench.py --gpus N under torchrun with every rank on device 0
# over the host transport (gloo for the bench's own barriers). Each step has
# its own time limit; the script stops at the first failure.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-r6procs}
mkdir -p $O
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_scan_service_procs.py -m gpu -k "${K:-config3}" -v -rs --timeout 500 --timeout-method thread > $O/pytest_procs.log 2>&1 || { tail -60 $O/pytest_procs.log; exit 1; }
  tail -5 $O/pytest_procs.log
fi
for n in ${NS:-2 4}; do
  KBG_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps ${STEPS:-10} --warmup 2 --dist-backend gloo --transport host > $O/bench_host_n$n.json 2> $O/bench_host_n$n.err || { tail -40 $O/bench_host_n$n.err; exit 1; }
  cat $O/bench_host_n$n.json
done
echo PROCS_DONE
