set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_face_detector.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread > $O/fd.log 2>&1 || { tail -40 $O/fd.log; exit 1; }
grep -E "PASSED|FAILED|detections" $O/fd.log | head -20
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-700
