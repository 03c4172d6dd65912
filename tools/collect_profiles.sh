#!/bin/bash
# Copy a tools/gpu_round.sh TAG run from gpurun_out/ into the tracked profiles/ (round-named files).
#   tools/collect_profiles.sh TAG ROUND   e.g. tools/collect_profiles.sh r01b r01
T=${1:?tag}; R=${2:?round prefix}; O=gpurun_out/$T
set -e
cp $O/bench.json profiles/${R}_bench.json
: > profiles/${R}_bench_runs.jsonl
for b in bench bench_noprof bench_host bench_irv1 bench_irv1_f16 bench_irv1_graph bench_r50 bench_r50_graph bench_fp8 bench_1m bench_bs1 bench_r50_bs1 bench_2share; do
  [ -f $O/$b.log ] && python3 -c "import json,sys; print(json.dumps({'run': sys.argv[1], 'line': json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])}))" $b $O/$b.log >> profiles/${R}_bench_runs.jsonl
done
cp "$(find $O/prof -name '*kernel_stats.csv' | head -1)" profiles/${R}_bench_kernel_stats.csv
grep '^{' $O/match_bench.log > profiles/${R}_match_bench.jsonl
cp $O/pmc_traffic.json profiles/${R}_pmc_traffic.json
grep -v "^\s*$" $O/tests.log | tail -40 > profiles/${R}_gpu_tests.txt
grep -E "1-cos|agreement|rel err|bs=256" $O/tests.log > profiles/${R}_parity_stats.txt || true
[ -f $O/layer_profile.txt ] && cp $O/layer_profile.txt profiles/${R}_layer_profile.txt
[ -f $O/layer_profile_irv1.txt ] && cp $O/layer_profile_irv1.txt profiles/${R}_irv1_layer_profile.txt
[ -f $O/layer_profile_bs1.txt ] && cp $O/layer_profile_bs1.txt profiles/${R}_bs1_layer_profile.txt
[ -f $O/mtcnn.json ] && cp $O/mtcnn.json profiles/${R}_mtcnn.json
[ -f $O/match_x3_sq_pmc.txt ] && cp $O/match_x3_sq_pmc.txt profiles/${R}_match_x3_sq_pmc.txt
echo "collected $T -> profiles/${R}_*"
