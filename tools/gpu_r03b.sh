# bench with its live PMC passes + a kernel trace of the steady state (tools/trace_gaps.py)
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
R=$(pwd)
( time timeout -k 10 400 python bench.py ) > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -4 $O/bench.log | cut -c1-1500
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt -o run -- python $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-prof --no-pmc > $R/$O/kt.log 2>&1 || { tail -20 $R/$O/kt.log; exit 1; }
cd $R && python tools/trace_gaps.py $O/kt --steps 3 > $O/gaps.txt && cat $O/gaps.txt
