set -o pipefail
mkdir -p gpurun_out/r03k
for shp in "35 32 32" "35 32 48" "35 48 64" "77 32 64" "147 32 32"; do
  set -- $shp
  for t in 2 8 14 15; do
    timeout -k 10 60 python tools/conv_bench.py --hw $1 --cin $2 --cout $3 --tile $t 2>/dev/null | tail -1
  done
  timeout -k 10 60 python tools/conv_bench.py --hw $1 --cin $2 --cout $3 --tile -1 2>/dev/null | tail -1
done > gpurun_out/r03k/tiles.txt
cat gpurun_out/r03k/tiles.txt
