#!/bin/bash
# scan-kernel variant timing (developer loop)
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=kube-arbitrator_amd/tools/variants
timeout -k 10 300 python kube-arbitrator_amd/tools/scan_bench.py $V/*.so > gpurun_out/scan_bench.jsonl 2> gpurun_out/scan_bench.err
KBG_FORCE_GENERAL_SCAN=1 timeout -k 10 200 python kube-arbitrator_amd/tools/scan_bench.py $V/libkbgpu_B16.so >> gpurun_out/scan_bench.jsonl 2>> gpurun_out/scan_bench.err
cat gpurun_out/scan_bench.jsonl
