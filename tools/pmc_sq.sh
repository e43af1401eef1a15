#!/bin/bash
# SQ counter passes (issue / wait / LDS breakdown) plus FETCH_SIZE and WRITE_SIZE
# (separate passes: MI355X_MICROARCH.md §rocprofv3 PMC slots) and a kernel trace
# of one Python driver script.
# usage (GPU box, repo root): bash tools/pmc_sq.sh TAG SCRIPT [script args...]
set -eo pipefail
TAG=$1; shift
SCRIPT=$GRAFT_REPO_ROOT/$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $SCRIPT "$@" > $OUT/trace.log 2>&1
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
            "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  echo "pass $i: $pass"
  timeout -s KILL 90 rocprofv3 --pmc $pass -f csv -d $OUT/p$i -o run -- python3 $SCRIPT "$@" > $OUT/p$i.log 2>&1
done
echo done
