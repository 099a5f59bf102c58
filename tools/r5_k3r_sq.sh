#!/bin/bash
# K3r (c5fir) SQ pass: VALU / SALU / LDS instructions and cycles per wave
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd); TAG=${TAG:-r5k3rsq}
for L in ${LIBS:-libicw.so}; do
( cd /tmp && ICW_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM \
    --output-format csv -d "$R/gpurun_out/${TAG}_${L%.so}" -o run \
    -- python3 "$R/bench.py" --workload c5fir --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_${L%.so}.txt 2>&1 || { echo "sq $L failed"; exit 3; }
echo "sq $L ok"
done
