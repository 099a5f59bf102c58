#!/bin/bash
# PMC passes over one C4 bench step (K2 = icw_output efficiency): one rocprofv3 --pmc run per pass.
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$R/gpurun_out/pmc_k2_$i" -o run \
      -- python3 "$R/bench.py" --workload ${WL:-c4} --steps 1 --warmup 1 --no-cpu-baseline ) > gpurun_out/pmc_k2_$i.txt 2>&1 || exit 2
done
echo ok
