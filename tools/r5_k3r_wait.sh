#!/bin/bash
# K3r (c5fir): where a wave's cycles go -- waits on counters (SQ_WAIT_ANY), waits to issue
# (SQ_WAIT_INST_ANY), active instruction cycles by kind
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd)
TAG=${TAG:-r5k3rw}
for L in ${LIBS:-libicw.so}; do
( cd /tmp && ICW_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA \
    --output-format csv -d "$R/gpurun_out/${TAG}_${L%.so}" -o run \
    -- python3 "$R/bench.py" --workload c5fir --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_${L%.so}.txt 2>&1 || { echo "pmc $L failed"; exit 3; }
echo "pmc $L ok"
done
