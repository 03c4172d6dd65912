#!/bin/bash
# conv_direct (tile 14) vs the igemm tiles on IRV1 shapes, bs = 256, f16/bf16 as the IRV1 plan runs them
set -o pipefail
O=gpurun_out/r03s16; mkdir -p $O
run() { timeout -k 10 60 python tools/conv_bench.py "$@" >> $O/sweep.jsonl 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }; }
for t in 14 0 2 3; do
  run --hw 8 --cin 256 --cout 896 --kh 1 --kw 1 --res --act 1 --tile $t    # Block17 up + res
  run --hw 17 --cin 32 --cout 32 --pad 1 --act 1 --tile $t                        # Block35 3x3
  run --hw 17 --cin 256 --cout 96 --kh 1 --kw 1 --act 1 --tile $t                 # Block35 1x1 256 -> 96
  run --hw 17 --cin 96 --cout 256 --kh 1 --kw 1 --tile $t                         # Block35 up (no res here)
  run --hw 8 --cin 256 --cout 896 --kh 1 --kw 1 --tile $t                         # Block17 up (no res here)
  run --hw 38 --cin 64 --cout 96 --kh 1 --kw 1 --dtype f16 --act 1 --tile $t      # conv2d_3b-like (Cout 96)
done
cat $O/sweep.jsonl
