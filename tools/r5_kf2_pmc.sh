#!/bin/bash
# KF2 (c2fir) by phase: SQ instruction and cycle counters of the full kernel and the diagnostic cuts
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd); TAG=${TAG:-r5kf2p}
for L in ${LIBS:-libicw.so libicw_cut1.so libicw_cut2.so}; do
  for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM" \
           "SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU"; do
    n=$(echo $C | cut -d' ' -f2)
    ( cd /tmp && ICW_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/${TAG}_${L%.so}_$n" -o run \
        -- python3 "$R/bench.py" --workload ${W:-c2fir} --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 --frames 262144 ) \
        > gpurun_out/${TAG}_${L%.so}_$n.txt 2>&1 || { echo "pmc $L $n failed"; exit 3; }
    echo "pmc $L $n ok"
  done
done
echo all-ok
