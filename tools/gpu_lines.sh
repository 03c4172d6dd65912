#!/bin/bash
# Quick multi-workload check on the GPU box:  tools/gpu_lines.sh TAG [tests: all | none | -k expr]
#   tests -> gpurun_out/TAG/tests.log; bench lines (no PMC / CPU leg): IResNet100 bs=256 (headline), bs=1,
#   IRV1 bf16, ResNet-50, fp8 -> gpurun_out/TAG/*.json; MTCNN 1080p -> mtcnn.json; one summary line each.
set -o pipefail
T=${1:?tag}; K=${2:-all}
O=gpurun_out/$T; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -30 $O/$name.log; exit $rc; fi; }
if [ "$K" = all ]; then
  step tests 600 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread
  grep -E "passed|failed" $O/tests.log | tail -1
elif [ "$K" != none ]; then
  step tests 600 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K"
  grep -E "passed|failed" $O/tests.log | tail -1
fi
B="python bench.py --no-cpu-baseline --no-pmc --no-n1-1m"
step bench 300 $B
step bench_bs1 300 $B --batch 1 --steps 50 --warmup 10 --no-prof
step bench_irv1 300 $B --arch irv1_facenet
step bench_r50 300 $B --arch resnet50_arcface
step bench_fp8 300 $B --dtype fp8
for b in bench bench_bs1 bench_irv1 bench_r50 bench_fp8; do
  grep '^{' $O/$b.log | tail -1 > $O/$b.json
  python -c "import json,sys; d=json.load(open('$O/$b.json')); print('$b', d['value'], 'faces/s', d['ms_per_step'], 'ms/step', d['dtype'])"
done
python tools/show_bench.py $O/bench.json
step mtcnn 200 python tools/mtcnn_bench.py --out $O/mtcnn.json
cat $O/mtcnn.json | tr -d '\n'; echo
echo "[$(date +%T)] done"
