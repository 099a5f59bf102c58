#!/bin/bash
# round 3 pass S: the driver's default bench command (every stream its own input), then the C2
# kernel stats of the same command under rocprofv3 --kernel-trace --stats
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r3s_bench_default.json 2> gpurun_out/r3s_bench_err.log || exit 3
cat gpurun_out/r3s_bench_default.json
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_c2" -o run \
    -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/r3s_prof_c2.txt 2>&1 || exit 4
echo ok
