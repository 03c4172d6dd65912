set -o pipefail
mkdir -p gpurun_out/r03o
FR_LIBFRHIP=facerecognition_amd/lib/variants/libfrhip_wd8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "wring" > gpurun_out/r03o/t.log 2>&1 || { tail -30 gpurun_out/r03o/t.log; exit 1; }
tail -1 gpurun_out/r03o/t.log
FR_LIBFRHIP=facerecognition_amd/lib/variants/libfrhip_wtrace8.so timeout -k 10 200 python tools/wring_trace.py > gpurun_out/r03o/wtrace8.txt 2>&1 && head -6 gpurun_out/r03o/wtrace8.txt
AB_CLASSES="conv_wring,stage layer3" bash tools/ab.sh "base wd8" 3 --no-cpu-baseline --no-pmc --steps 20 --warmup 5
