#!/bin/bash
# Round-end measurement on the GPU box (repo root):  tools/gpu_round.sh TAG [skip-tests]
#   1. pytest -m gpu           -> gpurun_out/TAG/tests.log
#   2. bench.py (default args) -> gpurun_out/TAG/bench.json  (+ --no-prof line for the event overhead)
#   3. rocprofv3 --kernel-trace --stats of the same bench command -> gpurun_out/TAG/prof/
#   (+ host-input, IRV1, ResNet-50, fp8 and 1M-gallery bench lines, tools/match_bench.py)
#   4. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE) -> profiles-ready traffic JSON
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
T=${1:?tag}; SKIP_TESTS=${2:-}
R=$(pwd); O=$R/gpurun_out/$T
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -20 $O/$name.log; exit $rc; fi; }
if [ -z "$SKIP_TESTS" ]; then
  step tests 900 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider -x --timeout 120 --timeout-method thread
  tail -3 $O/tests.log
fi
step bench 400 python bench.py
tail -1 $O/bench.log > $O/bench.json; cat $O/bench.json
step bench_noprof 300 python bench.py --no-prof --no-cpu-baseline
tail -1 $O/bench_noprof.log
step bench_host 300 python bench.py --no-cpu-baseline --host-input
step bench_irv1 300 python bench.py --no-cpu-baseline --arch irv1_facenet
step bench_irv1_f16 300 python bench.py --no-cpu-baseline --arch irv1_facenet --dtype f16
step bench_irv1_graph 300 python bench.py --no-cpu-baseline --no-prof --arch irv1_facenet
step bench_r50_graph 300 python bench.py --no-cpu-baseline --no-prof --arch resnet50_arcface
step bench_bs1 300 python bench.py --no-cpu-baseline --no-prof --batch 1 --steps 200 --warmup 20
step bench_r50_bs1 300 python bench.py --no-cpu-baseline --no-prof --arch resnet50_arcface --batch 1 --steps 200 --warmup 20
step bench_2share 300 python bench.py --no-cpu-baseline --no-prof --gpus 2 --share-device --steps 10 --warmup 3
step bench_r50 300 python bench.py --no-cpu-baseline --arch resnet50_arcface
step bench_fp8 300 python bench.py --no-cpu-baseline --dtype fp8
step bench_1m 300 python bench.py --no-cpu-baseline --gallery-rows 1000000
step match_bench 300 python tools/match_bench.py
for b in bench_noprof bench_host bench_irv1 bench_irv1_f16 bench_irv1_graph bench_r50 bench_r50_graph bench_fp8 bench_1m bench_bs1 bench_r50_bs1 bench_2share; do tail -1 $O/$b.log | cut -c1-400; done
BCMD="$R/bench.py --steps 10 --warmup 3 --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $BCMD
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-prof
cd $R
python tools/pmc_traffic.py --fetch $O/pf --write $O/pw --out $O/pmc_traffic.json
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -r head -12
cd $R && bash tools/gpu_layer_profile.sh ${T}_iresnet100 > $O/layer_profile.log 2>&1 && cp gpurun_out/lp_${T}_iresnet100/summary.txt $O/layer_profile.txt
bash tools/gpu_layer_profile.sh ${T}_irv1 --arch irv1_facenet > $O/layer_profile_irv1.log 2>&1 && cp gpurun_out/lp_${T}_irv1/summary.txt $O/layer_profile_irv1.txt
bash tools/gpu_layer_profile.sh ${T}_bs1 --batch 1 > $O/layer_profile_bs1.log 2>&1 && cp gpurun_out/lp_${T}_bs1/summary.txt $O/layer_profile_bs1.txt
step mtcnn 300 python -u tools/mtcnn_bench.py --out $O/mtcnn.json
echo "[$(date +%T)] done"
