#!/bin/bash
# C2 launch-block A/B: default plan vs longer blocks with a geometric tail (bench.py c2, 5 steps each)
mkdir -p gpurun_out
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 > gpurun_out/c2ab_$tag.txt 2>&1 || exit 2; }
run def ICW_X=0
run b64k ICW_BLOCK=65536
run b64k_t25 ICW_BLOCK=65536 ICW_TAPER=0.25
run b32k_t5 ICW_BLOCK=32768 ICW_TAPER=0.5
run def2 ICW_X=0
