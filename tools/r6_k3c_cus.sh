#!/bin/bash
# K3c on c5fir: the render's own CUs (ICW_RENDER_CUS) A/B, then a kernel-trace and an SQ pass
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd); TAG=${TAG:-r6b}
VAR=ICW_RENDER_CUS VALS="- 64 128" WLS="c5fir" REPS=2 TAG=${TAG}env bash tools/env_ab.sh || exit 3
( cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_trace" -o run \
    -- python3 "$R/bench.py" --workload c5fir --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_trace.txt 2>&1 || { echo "trace failed"; exit 3; }
echo trace ok
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM \
    --output-format csv -d "$R/gpurun_out/${TAG}_sq" -o run \
    -- python3 "$R/bench.py" --workload c5fir --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_sq.txt 2>&1 || { echo "sq failed"; exit 3; }
echo sq ok
