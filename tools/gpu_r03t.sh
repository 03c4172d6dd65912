#!/bin/bash
# graph-slot timing check: ABI + slot test + replay tests, then bench with and without the profiled leg
set -o pipefail
mkdir -p gpurun_out/r03t
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_abi.py \
  tests/test_gpu_models.py -k "abi or prof_slot or replay" > gpurun_out/r03t/tests.txt 2>&1 &&
timeout -k 10 240 python -u bench.py > gpurun_out/r03t/bench_prof.json 2> gpurun_out/r03t/bench_prof.err &&
timeout -k 10 240 python -u bench.py --no-prof > gpurun_out/r03t/bench_noprof.json 2> gpurun_out/r03t/bench_noprof.err &&
timeout -k 10 240 python -u bench.py > gpurun_out/r03t/bench_prof2.json 2>> gpurun_out/r03t/bench_prof.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03t/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/gpurun_out/r03t/bench_rocprof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r03t/rocprof.err
