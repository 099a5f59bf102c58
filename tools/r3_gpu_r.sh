#!/bin/bash
# round 3 re-entry pass: the whole -m gpu suite + smoke, then the driver's default bench command
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 2
timeout -k 10 600 python -u bench.py > gpurun_out/r3r_bench_default.json 2> gpurun_out/r3r_bench_err.log || exit 3
cat gpurun_out/r3r_bench_default.json
echo ok
