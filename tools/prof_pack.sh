#!/bin/bash
# Summarise a gpurun_out/prof_TAG directory (tools/profile_round.sh or tools/din_pmc.sh
# output) into gpurun_out/TAG_rocprof_summary.json + TAG_kernel_stats.csv and delete
# the raw per-dispatch CSVs (gpurun copies back at most 64 MiB of gpurun_out/).
# usage (GPU box, repo root): bash tools/prof_pack.sh TAG
set -eo pipefail
TAG=$1
D=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py --stats $D/trace/run_kernel_stats.csv \
  --fetch $D/fetch/run_counter_collection.csv --write $D/write/run_counter_collection.csv \
  --out $GRAFT_REPO_ROOT/gpurun_out/${TAG}_rocprof_summary.json --top 40
cp $D/trace/run_kernel_stats.csv $GRAFT_REPO_ROOT/gpurun_out/${TAG}_kernel_stats.csv
for f in trace.json fetch.json write.json trace.log; do
  if [ -f $D/$f ]; then cp $D/$f $GRAFT_REPO_ROOT/gpurun_out/${TAG}_$f; fi
done
rm -rf $D
echo packed $TAG
