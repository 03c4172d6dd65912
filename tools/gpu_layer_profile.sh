#!/bin/bash
# Usage (on the GPU box, repo root): tools/gpu_layer_profile.sh TAG [layer_profile args...]
R=$(pwd); T=$1; shift
mkdir -p gpurun_out/lp_$T
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/lp_$T -o run -- python $R/tools/layer_profile.py --run --plan $R/gpurun_out/lp_$T/plan.txt "$@" > $R/gpurun_out/lp_$T/log 2>&1 ) || { tail -5 gpurun_out/lp_$T/log; exit 1; }
python tools/layer_profile.py --trace gpurun_out/lp_$T/run_kernel_trace.csv --plan gpurun_out/lp_$T/plan.txt > gpurun_out/lp_$T/summary.txt
head -12 gpurun_out/lp_$T/summary.txt; tail -1 gpurun_out/lp_$T/summary.txt
