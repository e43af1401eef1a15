#!/bin/bash
# Kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE passes of the bench
# (MI355X_MICROARCH.md §HBM: the two TCC counters do not fit one pass).
# usage (on the GPU box, from the repo root): bash tools/profile_round.sh TAG [bench args...]
set -eo pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $OUT/trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $OUT/fetch.json 2> $OUT/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" > $OUT/write.json 2> $OUT/write.err
echo done
