#!/bin/bash
# kernel trace (start/end per launch) of one workload's bench: WL=c4 [ENVS="ICW_BLOCK=8192"] bash tools/trace_wl.sh
mkdir -p gpurun_out
R=$(pwd); export TMPDIR=/tmp
tag=${WL}${TAG:+_$TAG}
for e in $ENVS; do export "$e"; done
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace_$tag" -o run \
    -- python3 "$R/bench.py" --workload "$WL" --steps 3 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 ) > "gpurun_out/trace_$tag.txt" 2>&1
rc=$?; echo "[trace_$tag] rc=$rc"; exit $rc
