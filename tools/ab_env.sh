#!/bin/bash
# A/B of an environment switch on one box: rocprofv3 kernel stats and bench
# lines with $AB_VAR=$AB_A and =$AB_B, config $AB_CFG (c2 default).
#   AB_VAR=MOLCLR_Q6_PP AB_A=0 AB_B=1 bash tools/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cfg=${AB_CFG:-c2}
for v in "$AB_A" "$AB_B"; do
  rm -rf "gpurun_out/ab_$v"
  env "$AB_VAR=$v" timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/ab_$v" -o run --output-format csv -- python bench.py --config "$cfg" --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > "gpurun_out/ab_prof_$v.log" 2>&1 || { echo "prof $v failed"; exit 1; }
done
for r in 1 2; do
  for v in "$AB_A" "$AB_B"; do
    env "$AB_VAR=$v" timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline --no-kernel-timing > "gpurun_out/ab_bench_${v}_$r.log" 2>&1 || { echo "bench $v failed"; exit 1; }
    echo "$AB_VAR=$v run $r: $(grep -o '"value": [0-9.]*' gpurun_out/ab_bench_${v}_$r.log) $(grep -o '"median_value": [0-9.]*' gpurun_out/ab_bench_${v}_$r.log)"
  done
done
for v in "$AB_A" "$AB_B"; do
  python tools/prof_summary.py "gpurun_out/ab_$v" "gpurun_out/ab_$v.md" 25 > /dev/null 2>&1
  echo "== $AB_VAR=$v"; sed -n 3,22p "gpurun_out/ab_$v.md"
done
