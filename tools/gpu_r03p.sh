set -o pipefail
mkdir -p gpurun_out/r03p
FR_LIBFRHIP=facerecognition_amd/lib/variants/libfrhip_wtp2.so timeout -k 10 200 python tools/wring_trace.py > gpurun_out/r03p/wtrace_p2.txt 2>&1 && head -6 gpurun_out/r03p/wtrace_p2.txt
AB_CLASSES="conv_wring" bash tools/ab.sh "base prio1 prio2" 3 --no-cpu-baseline --no-pmc --steps 20 --warmup 5
