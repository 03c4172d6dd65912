#!/bin/bash
# Small-batch match timing (bs = 1 online path): kernel durations of fr_match_topk at B probes x 10k rows under
# rocprofv3 --kernel-trace --stats, for the split plans given as FR_MATCH_TILES values (0 = the plan's own).
#   tools/match_small.sh TAG B "0 1 2 4" [extra env]
set -o pipefail
T=${1:?tag}; B=${2:-1}; V=${3:-0}; R=$(pwd); O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for t in $V; do
  env FR_AB=match_tiles=$t $4 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$t -o run -- \
    python $R/tools/match_bench.py --only-rows 10000 --probes $B --iters 50 > $O/t$t.log 2>&1 || { tail -5 $O/t$t.log; exit 1; }
  echo "tiles=$t: $(tail -1 $O/t$t.log | cut -c1-120)"
  f=$(find $O/t$t -name "*kernel_stats.csv" | head -1); head -4 $f | cut -d, -f1-4
done
