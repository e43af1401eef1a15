#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate, MI355X_MICROARCH.md HBM section) and a
# kernel trace of the fused DIN step at B = 4096 (tools/din_step.py).
# usage (GPU box, repo root): bash tools/din_pmc.sh TAG [din_step args...]
set -eo pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/din_step.py "$@" > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/din_step.py "$@" > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- python3 $GRAFT_REPO_ROOT/tools/din_step.py "$@" > $OUT/write.log 2>&1
echo done
