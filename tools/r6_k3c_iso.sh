#!/bin/bash
# c5fir kernel traces with every kernel on one stream (ICW_SERIALIZE=1): the render alone, K3c and K3r
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd); TAG=${TAG:-r6c}
for C in 1 0; do
( cd /tmp && ICW_SERIALIZE=1 ICW_K3R_COMP=$C timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_ser$C" -o run \
    -- python3 "$R/bench.py" --workload c5fir --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_ser$C.txt 2>&1 || { echo "trace $C failed"; exit 3; }
echo "trace comp=$C ok"
done
