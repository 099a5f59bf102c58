#!/bin/bash
# SQ counters of K3r (c5fir) in two builds, then an instruction-cache pass
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd)
TAG=${TAG:-r5k3rp}
for L in libicw_prev.so libicw.so; do
  ( cd /tmp && ICW_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM \
      --output-format csv -d "$R/gpurun_out/${TAG}_sq_${L%.so}" -o run \
      -- python3 "$R/bench.py" --workload c5fir --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_sq_${L%.so}.txt 2>&1 || { echo "sq $L failed"; exit 3; }
  echo "sq $L ok"
done
for L in libicw_prev.so libicw.so; do
  ( cd /tmp && ICW_LIB=$L timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS \
      --output-format csv -d "$R/gpurun_out/${TAG}_ic_${L%.so}" -o run \
      -- python3 "$R/bench.py" --workload c5fir --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_ic_${L%.so}.txt 2>&1 || { echo "icache $L failed"; exit 4; }
  echo "icache $L ok"
done
echo all-ok
