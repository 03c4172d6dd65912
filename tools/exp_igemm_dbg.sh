#!/bin/bash
# igemm cost decomposition (timing-only FR_CONV_DBG switches): 16 = no epilogue, 32 = no A DMA, 64 = no B DMA
for d in 0 16 32 64 96 112; do FR_CONV_DBG=$d tools/gpu_layer_profile.sh i$d > gpurun_out/i$d.txt || exit 1; echo "dbg=$d"; sed -n 4,7p gpurun_out/i$d.txt; done
