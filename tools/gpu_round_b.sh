#!/bin/bash
# Round-end measurement, part B (repo root): rocprofv3 kernel stats of the bench, PMC traffic passes,
# per-launch layer profile, match bench.  tools/gpu_round_b.sh TAG
set -o pipefail
T=${1:?tag}; R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -20 $O/$name.log; exit $rc; fi; }
BCMD="$R/bench.py --steps 10 --warmup 3 --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $BCMD
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof
cd $R
python tools/pmc_traffic.py --fetch $O/pf --write $O/pw --out $O/pmc_traffic.json
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -r head -8
bash tools/gpu_layer_profile.sh ${T}_iresnet100 > $O/layer_profile.log 2>&1 && cp gpurun_out/lp_${T}_iresnet100/summary.txt $O/layer_profile.txt
bash tools/gpu_layer_profile.sh ${T}_irv1 --arch irv1_facenet > $O/layer_profile_irv1.log 2>&1 && cp gpurun_out/lp_${T}_irv1/summary.txt $O/layer_profile_irv1.txt
step match_bench 300 python tools/match_bench.py
echo "[$(date +%T)] done"
