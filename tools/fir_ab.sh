#!/bin/bash
# FIR converter forms A/B: every FIR workload with the fused kernel KF2 and with KF + K2 (ICW_FIR_FUSED=0)
mkdir -p gpurun_out
for f in 1 0; do
  for w in ${WLS:-c2fir c3fir c4fir c5fir}; do
    ICW_FIR_FUSED=$f timeout -k 10 200 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --e2e-steps 0 \
      > gpurun_out/bench_${w}_f$f.txt 2>&1 || exit 2
  done
done
