#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first
# step that faults, aborts or times out (exit status > 1).  A pytest status of
# 1 (test failures) does not stop the chain.
# usage: bash tools/run_checked.sh 'SECONDS|NAME|command' ...
mkdir -p "$GRAFT_REPO_ROOT/gpurun_out"
for spec in "$@"; do
  t=${spec%%|*}; rest=${spec#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "== $name (limit ${t}s)"
  timeout -k 10 "$t" bash -c "$cmd" > "$GRAFT_REPO_ROOT/gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc $rc"
  tail -3 "$GRAFT_REPO_ROOT/gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name"; exit $rc; fi
done
