#!/bin/bash
# timeline of the single-stream drop-in (C1): kernels and copies of each 576-frame call
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$R/gpurun_out/trace_c1" -o run \
    -- python3 "$R/bench.py" --workload c1 --steps 1 --warmup 1 --no-cpu-baseline ) > gpurun_out/trace_c1.txt 2>&1
rc=$?; echo "[trace_c1] rc=$rc"; exit $rc
