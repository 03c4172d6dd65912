#!/bin/bash
# SQ/GRBM counter passes over a short bench run (one rocprofv3 --pmc run per pass, each under its own
# kill timeout; never combined with tracing domains):   tools/pmc_run.sh OUTDIR [bench args...]
# Summarise with: python tools/pmc_summary.py OUTDIR [kernel-name filter]
set -o pipefail
O=$(realpath -m ${1:?outdir}); shift
R=$(pwd)
ARGS=${*:-"--steps 3 --warmup 1 --no-cpu-baseline --no-prof"}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_LDS_BANK_CONFLICT,GRBM_GUI_ACTIVE"
P2=${PMC_P2:-"SQ_INSTS_LDS,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM,SQ_LDS_IDX_ACTIVE,SQ_WAVES,SQ_INSTS_MFMA,SQ_ACTIVE_INST_LDS"}
i=1
for P in $P1 $P2; do
  echo "[$(date +%T)] pass $i: $P"
  timeout -s KILL 120 rocprofv3 --pmc ${P//,/ } --output-format csv -d $O/p$i -o run -- python $R/bench.py $ARGS > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; tail -5 $O/p$i.log; exit $rc; fi
  i=$((i+1))
done
echo "[$(date +%T)] done"
