#!/bin/bash
# Attention-backward kernel time vs batch (GPU box only): bash tools/din_bwd_batches.sh "ENV=.." B1 B2 ...
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
v=$1; shift
for bt in "$@"; do
  env $v timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/bt_${bt} -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload din --no-cpu-baseline --steps 10 --din-batch $bt > /dev/null 2>&1
done
