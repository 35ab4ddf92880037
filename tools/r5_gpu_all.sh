#!/bin/bash
# Full GPU test suite, then a short c2 bench line (round-5 check).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/all_test.log 2>&1
rc=$?
tail -3 gpurun_out/all_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_c2.log 2>&1
rc=$?
tail -1 gpurun_out/bench_c2.log | cut -c1-400
exit $rc
