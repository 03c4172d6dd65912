#!/bin/bash
# Round-end measurement, part A (repo root): GPU tests + bench lines.  tools/gpu_round_a.sh TAG
set -o pipefail
T=${1:?tag}; R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -20 $O/$name.log; exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider -x --timeout 120 --timeout-method thread
tail -3 $O/tests.log
step bench 400 python bench.py
tail -1 $O/bench.log > $O/bench.json; cut -c1-300 $O/bench.json
step bench_noprof 300 python bench.py --no-prof --no-cpu-baseline
step bench_host 300 python bench.py --no-cpu-baseline --host-input
step bench_irv1 300 python bench.py --no-cpu-baseline --arch irv1_facenet
step bench_irv1_f16 300 python bench.py --no-cpu-baseline --arch irv1_facenet --dtype f16
step bench_irv1_graph 300 python bench.py --no-cpu-baseline --no-prof --arch irv1_facenet
step bench_r50 300 python bench.py --no-cpu-baseline --arch resnet50_arcface
step bench_r50_graph 300 python bench.py --no-cpu-baseline --no-prof --arch resnet50_arcface
step bench_fp8 300 python bench.py --no-cpu-baseline --dtype fp8
step bench_1m 300 python bench.py --no-cpu-baseline --gallery-rows 1000000
step bench_bs1 300 python bench.py --no-cpu-baseline --no-prof --batch 1 --steps 200 --warmup 20
step bench_2share 300 python bench.py --no-cpu-baseline --no-prof --gpus 2 --share-device --steps 10 --warmup 3
for b in bench_noprof bench_host bench_irv1 bench_irv1_f16 bench_irv1_graph bench_r50 bench_r50_graph bench_fp8 bench_1m bench_bs1 bench_2share; do tail -1 $O/$b.log | cut -c1-200; done
echo "[$(date +%T)] done"
