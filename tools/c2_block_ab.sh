#!/bin/bash
# C2 launch-block A/B: the default plan (65 536-frame blocks + a 0.25 tail for the row kernel without
# a serial render) against the previous 16 384-frame plan (ICW_BLOCK=16384), bench.py c2, 5 steps each
mkdir -p gpurun_out
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 > gpurun_out/c2ab_$tag.txt 2>&1 || exit 2; }
run def ICW_X=0
run b16k ICW_BLOCK=16384
run def2 ICW_X=0
run b16k2 ICW_BLOCK=16384
