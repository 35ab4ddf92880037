#!/bin/bash
# side-stream head weight gradients: their tests + graph-step/DP tests, then c2 bench A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_graph_step.py tests/test_gpu_dp.py tests/test_gpu_models.py \
  > gpurun_out/side_tests.log 2>&1
rc=$?; tail -2 gpurun_out/side_tests.log; grep "^E " gpurun_out/side_tests.log | head -5
[ $rc -ne 0 ] && exit $rc
for v in 0 1 0 1; do
  MOLCLR_SIDE_WGRAD=$v timeout -k 10 200 python -u bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/side_b$v.log 2>&1 || exit $?
  echo "side=$v $(tail -1 gpurun_out/side_b$v.log | cut -c1-120)"
done
