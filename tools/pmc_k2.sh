#!/bin/bash
# PMC passes over one workload (serialized kernels): WL=c3 bash tools/pmc_k2.sh
# Each pass is its own rocprofv3 run under a hard time limit (counters per pass within the slots).
R=$(pwd); export TMPDIR=/tmp; WL=${WL:-c3}
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  ( cd /tmp && ICW_SERIALIZE=1 timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/pmc_${WL}_$i" -o run \
      -- python3 "$R/bench.py" --workload "$WL" --steps 1 --warmup 1 --no-cpu-baseline ) > gpurun_out/pmc_${WL}_$i.txt 2>&1
  rc=$?; echo "[pmc_${WL}_$i] rc=$rc"; [ $rc -eq 0 ] || exit 2
done
