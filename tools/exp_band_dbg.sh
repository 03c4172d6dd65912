for d in 0 1 2 4 8 7 15; do FR_CONV_DBG=$d tools/gpu_layer_profile.sh x$d > gpurun_out/x$d.txt || exit 1; echo "dbg=$d $(sed -n 3p gpurun_out/x$d.txt)"; done
