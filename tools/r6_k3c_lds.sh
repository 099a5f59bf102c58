#!/bin/bash
# c5fir: K3c's LDS pad A/B (ICW_K3C_LDS), then FETCH_SIZE / WRITE_SIZE passes (K3a's writes, generator-major)
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd); TAG=${TAG:-r6d}
VAR=ICW_K3C_LDS VALS="- 98304 110592" WLS="c5fir" REPS=2 TAG=${TAG}env bash tools/env_ab.sh || exit 3
for C in FETCH_SIZE WRITE_SIZE; do
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/${TAG}_$C" -o run \
    -- python3 "$R/bench.py" --workload c5fir --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_$C.txt 2>&1 || { echo "pmc $C failed"; exit 3; }
echo "pmc $C ok"
done
