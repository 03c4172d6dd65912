set -o pipefail
mkdir -p gpurun_out/r03l
timeout -k 10 300 python -u -m pytest tests/test_gpu_stage.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03l/t.log 2>&1 || { tail -30 gpurun_out/r03l/t.log; exit 1; }
tail -2 gpurun_out/r03l/t.log
bash tools/ab.sh "base prev" 3 --no-cpu-baseline --no-pmc --steps 20 --warmup 5
