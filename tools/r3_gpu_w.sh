#!/bin/bash
# round 3 pass W: geometric tail for the lane-kernel workloads (VERDICT r02 #2b): C3 / C4 with the
# default uniform blocks against ICW_TAPER 0.5 / 0.7, two runs each, interleaved
mkdir -p gpurun_out
for r in 1 2; do
  for tp in d 0.5 0.7; do
    for w in c3 c4; do
      env=""; [ $tp != d ] && env="ICW_TAPER=$tp"
      env $env timeout -k 10 200 python -u bench.py --workload $w --steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0 \
        > gpurun_out/r3w_${tp}_${w}_$r.json 2>>gpurun_out/r3w_err.log || exit 3
    done
  done
done
echo ok
