#!/bin/bash
# e2e re-rank kernel time under NRK_RR_DBG variants (GPU box only)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2 3; do
  NRK_RR_DBG=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/rr_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload e2e --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2>&1
done
