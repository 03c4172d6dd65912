#!/bin/bash
# Same-box A/B of the match kernels at the config-4 shapes: tools/match_ab.sh "base FR_LIBFRHIP=<variant.so>" [rounds]
set -o pipefail
V=${1:?settings}; N=${2:-2}
for r in $(seq 1 $N); do
  for v in $V; do
    if [ "$v" = base ]; then env_set=""; else env_set="$v"; fi
    echo "== $v round $r"
    env $env_set timeout -k 10 200 python tools/match_bench.py --iters 20 | grep -v "^$" || exit 1
  done
done
