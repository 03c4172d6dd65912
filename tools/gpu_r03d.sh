set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "wring or variants_bit or test_embedding_cosine or full_batch_properties or split_stage_batches" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 1 0 1; do
  FR_STAGE_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > $O/bench_v$v.log 2>&1 || { tail -20 $O/bench_v$v.log; exit 1; }
  grep '^{' $O/bench_v$v.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); k=d['kernels']; print('variant $v value', d['value'], 'fwd', d['forward']['embed_ms'], 'stage3', k['stage layer3']['ms_per_step'], 'wring', k['conv_wring']['ms_per_step'])"
done
