set -o pipefail
for d in 0 16 0 16; do
  FR_CONV_DBG=$d timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/dbg_$d.log 2>&1 || { tail -5 gpurun_out/dbg_$d.log; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/dbg_$d.log').read().strip().splitlines()[-1])
print('dbg=$d', d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"
done
