#!/bin/bash
# Time the DIN train step's attention backward under env variants (GPU box only):
#   bash tools/din_bwd_parts.sh "NRK_DIN_BWD_DBG=0" "NRK_DIN_BWD_DBG=3 NRK_DIN_BWD_SLOTS=3" ...
# NRK_DIN_BWD_DBG bits skip math (timing only): 1 dalpha, 2 z/epilogue/dW, 4 dW MFMAs.
set -eo pipefail
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  env $v timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/parts_$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload din --no-cpu-baseline --steps 10 > /dev/null 2>&1
  echo "$i $v" >> $GRAFT_REPO_ROOT/gpurun_out/parts_index.txt
  i=$((i+1))
done
