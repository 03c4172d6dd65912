#!/bin/bash
# SQ counter passes over tools/match_bench.py (one rocprofv3 --pmc run per pass, each under its own kill timeout):
#   tools/pmc_match.sh OUTDIR [match_bench args...];  summary: python tools/pmc_summary.py OUTDIR match_x3
set -o pipefail
O=$(realpath -m ${1:?outdir}); shift
R=$(pwd)
ARGS=${*:-"--only-rows 1000000 --iters 5"}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM,SQ_LDS_IDX_ACTIVE,SQ_WAVES,SQ_INSTS_MFMA,SQ_ACTIVE_INST_LDS"
i=1
for P in $P1 $P2; do
  timeout -s KILL 120 rocprofv3 --pmc ${P//,/ } --output-format csv -d $O/p$i -o run -- python $R/tools/match_bench.py $ARGS > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; tail -5 $O/p$i.log; exit $rc; fi
  i=$((i+1))
done
