#!/bin/bash
# C5 launch-block A/B, shorter blocks and tail ratios (row kernel + serial render)
set -o pipefail
mkdir -p gpurun_out
run() { # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
      > gpurun_out/c5b2_${tag}.json 2>>gpurun_out/c5b2_err.log
}
for r in 1 2; do
  run default_$r ICW_NOP=1 || exit 2
  run b8192_$r ICW_BLOCK=8192 || exit 2
  run b12288_$r ICW_BLOCK=12288 || exit 2
  run t075_$r ICW_TAPER=0.75 || exit 2
  run t092_$r ICW_TAPER=0.92 || exit 2
done
echo ok
