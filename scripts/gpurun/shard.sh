#!/bin/bash
# Per-rank critical paths of a sharded allocate (tools/shard_paths.py; PROTOCOL=owner: owner-resolve),
# R device sessions on one GPU; one run per config under its own time limit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${RUN:-shard}
mkdir -p $O
cd $R
for cfg in ${CFGS:-4 3}; do
  timeout -k 10 500 python kube-arbitrator_amd/tools/shard_paths.py $cfg > $O/paths_c$cfg.jsonl 2> $O/paths_c$cfg.err || { tail -20 $O/paths_c$cfg.err; exit 1; }
  cat $O/paths_c$cfg.jsonl | cut -c1-400
done
