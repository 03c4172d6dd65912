set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "variants_bit or test_embedding_cosine or stage_matches" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
for v in 0 1 2; do
  FR_STAGE_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > $O/bench_v$v.log 2>&1 || { tail -20 $O/bench_v$v.log; exit 1; }
  grep '^{' $O/bench_v$v.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']; print('variant $v value', d['value'], 'fwd', d['forward']['embed_ms'], 'stage3', k['stage layer3']['ms_per_step'])"
done
FR_LIBFRHIP=facerecognition_amd/lib/variants/libfrhip_dbl.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > $O/bench_dbl.log 2>&1 || { tail -20 $O/bench_dbl.log; exit 1; }
grep '^{' $O/bench_dbl.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']; print('double-buffer value', d['value'], 'fwd', d['forward']['embed_ms'], 'stage3', k['stage layer3']['ms_per_step'])"
done
