set -o pipefail
O=gpurun_out/x3e; mkdir -p $O
for r in 1 2; do for v in base x3e1 x3e2 x3e3; do
  L=""; [ "$v" != base ] && L=facerecognition_amd/lib/variants/libfrhip_$v.so
  FR_LIBFRHIP=$L timeout -k 10 200 python tools/match_bench.py --iters 50 --only-rows 125000 > $O/b_${v}_$r.log 2>&1 || { echo "$v failed"; tail -5 $O/b_${v}_$r.log; exit 1; }
done; done
