#!/bin/bash
# match_x3 variants on one box: parity tests of each variant library, then same-box timing A/B at the config-4
# shapes.  tools/gpu_x3.sh TAG "name1 name2 ..." ["bench-only names"] (names of
# facerecognition_amd/lib/variants/libfrhip_NAME.so; "base" = the in-tree library; timing-only builds go in the
# third list: they are benched, not tested)
set -o pipefail
T=${1:?tag}; V=${2-}; VB="$V ${3:-}"
O=gpurun_out/$T; mkdir -p $O
lib() { if [ "$1" = base ]; then echo ""; else echo "FR_LIBFRHIP=facerecognition_amd/lib/variants/libfrhip_$1.so"; fi; }
for v in $V; do
  echo "== tests $v"
  env $(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "match" > $O/tests_$v.txt 2>&1 || { tail -30 $O/tests_$v.txt; exit 1; }
  tail -2 $O/tests_$v.txt
done
for r in 1 2; do
  for v in $VB; do
    echo "== bench $v round $r"
    env $(lib $v) timeout -k 10 200 python tools/match_bench.py --iters 20 > $O/bench_${v}_$r.jsonl 2>&1 || { tail -20 $O/bench_${v}_$r.jsonl; exit 1; }
    cat $O/bench_${v}_$r.jsonl
  done
done
