#!/bin/bash
# C5 launch-block length A/B (row kernel + serial render, 0.85 tail): default 16384 vs 32768 / 65536
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for b in default 32768 65536; do
    if [ $b = default ]; then unset ICW_BLOCK; else export ICW_BLOCK=$b; fi
    timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
      > gpurun_out/c5blk_${b}_$r.json 2>>gpurun_out/c5blk_err.log || exit 2
  done
done
unset ICW_BLOCK
echo ok
