set -o pipefail
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u bench.py --cpu-sample 0 > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
cat $O/c3.json
