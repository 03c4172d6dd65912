set -o pipefail
mkdir -p gpurun_out/r03i
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "large_k or faiss or match" > gpurun_out/r03i/t.log 2>&1 || { tail -40 gpurun_out/r03i/t.log; exit 1; }
tail -3 gpurun_out/r03i/t.log
bash tools/gpu_layer_profile.sh irv1 --arch irv1_facenet > gpurun_out/r03i/lp_irv1.txt 2>&1; cat gpurun_out/lp_irv1/summary.txt | head -60
