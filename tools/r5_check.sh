#!/bin/bash
# Focused GPU check: the given pytest selection, then a c2 bench line (and,
# with PROF=1, a rocprofv3 kernel summary of the bench).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread "$@" \
  > gpurun_out/check.log 2>&1
rc=$?; tail -2 gpurun_out/check.log; grep "^E " gpurun_out/check.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1
rc=$?; tail -1 gpurun_out/bench_c2.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
if [ "${PROF:-0}" = 1 ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > gpurun_out/prof.log 2>&1
  rc=$?; python tools/prof_summary.py gpurun_out/prof gpurun_out/prof.md 25 > /dev/null
fi
exit $rc
