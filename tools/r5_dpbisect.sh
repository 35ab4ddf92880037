#!/bin/bash
# Run pytest subsets in order; continue past test failures (rc 1) but stop at
# anything else (fault, abort, timeout).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
i=0
for sel in "$@"; do
  i=$((i+1))
  echo "== [$i] $sel" | tee -a gpurun_out/bisect.log
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $sel \
     > gpurun_out/bisect_$i.log 2>&1
  rc=$?
  tail -5 gpurun_out/bisect_$i.log | tee -a gpurun_out/bisect.log
  echo "rc=$rc" | tee -a gpurun_out/bisect.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
