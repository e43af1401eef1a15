#!/bin/bash
# PMC passes for the corpus producer (tools/embed_step.py): MFMA busy + clock,
# issue/wait split, HBM fetch.  usage (GPU box, repo root): bash tools/pmc_embed.sh N
set -eo pipefail
N=${1:-4000000}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_embed
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
S=$GRAFT_REPO_ROOT/tools/embed_step.py
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $S --n $N --reps 2 > $OUT/trace.log 2>&1
i=0
for pass in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  echo "pass $i: $pass"
  timeout -s KILL 90 rocprofv3 --pmc $pass -f csv -d $OUT/p$i -o run -- python3 $S --n $N --reps 2 > $OUT/p$i.log 2>&1
done
echo done
