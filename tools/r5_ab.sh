#!/bin/bash
# c2 and c5 bench lines + rocprof summaries (one box)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c2 c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/ab_$c.log 2>&1 || exit $?
  echo "$c $(tail -1 gpurun_out/ab_$c.log | cut -c1-150)"
  rm -rf gpurun_out/abp_$c
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_$c -o run --output-format csv -- python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > gpurun_out/abp_$c.log 2>&1 || exit $?
  python tools/prof_summary.py gpurun_out/abp_$c gpurun_out/abp_$c.md 40 > /dev/null
done
