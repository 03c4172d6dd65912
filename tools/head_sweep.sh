for hp in "2,28" "2,14" "2,49" "2,56" "1,28" "1,56" "1,98" "0,28" "3,28" "3,56"; do
  FR_AB=head_plan=${hp/,/:} timeout -k 10 100 python bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$hp', d['ms_per_step'], d['kernels']['head']['ms_per_step'])"
done
