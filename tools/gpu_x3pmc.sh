#!/bin/bash
# SQ counter passes over the config-4 match shape (2048 x 125k, bf16x3 path): tools/gpu_x3pmc.sh OUTDIR
set -o pipefail
O=$(realpath -m ${1:?outdir}); R=$(pwd); mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM,SQ_LDS_IDX_ACTIVE,SQ_WAVES,SQ_INSTS_MFMA,SQ_ACTIVE_INST_LDS"
i=1
for P in $P1 $P2; do
  timeout -s KILL 120 rocprofv3 --pmc ${P//,/ } --output-format csv -d $O/p$i -o run -- python $R/tools/match_bench.py --only-rows 125000 --iters 3 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  i=$((i+1))
done
cd $R && python tools/pmc_summary.py $O match_x3 > $O/summary.txt && cat $O/summary.txt
