#!/bin/bash
# Run GPU steps in order on the box, each under its own time limit, logging to
# gpurun_out/<tag>_<name>.log.  A step that fails normally (exit 1 / 2: test
# failures, Python errors) does not stop the run; a time limit (124 / 137), an
# abort (134) or a segfault (139) does: nothing more touches the GPU then.
# usage: bash tools/gpu_steps.sh TAG "name|seconds|command" ...
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out
mkdir -p $OUT
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "[$(date +%T)] $name: $cmd" | tee -a $OUT/${TAG}_steps.txt
  timeout -k 10 $secs bash -c "$cmd" > $OUT/${TAG}_${name}.log 2>&1
  rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a $OUT/${TAG}_steps.txt
  if [ $rc -ge 124 ] && [ $rc -ne 255 ]; then
    echo "stopping: $name ended with $rc" | tee -a $OUT/${TAG}_steps.txt
    exit $rc
  fi
done
exit 0
