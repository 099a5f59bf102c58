#!/bin/bash
# K1's clock and cycles per VALU with every kernel on one stream (ICW_SERIALIZE=1) against the
# overlapped pipeline: kernel stats + one SQ pass per mode.  WL=c4 bash tools/sq_serial.sh
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
for M in 1 0; do
  export ICW_SERIALIZE=$M
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ser${M}_prof_$WL" -o run \
      -- python3 "$R/bench.py" --workload $WL --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) \
      > gpurun_out/ser${M}_prof_$WL.txt 2>&1 || { echo "[ser${M}_prof] failed"; exit 2; }
  ( cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d "$R/gpurun_out/ser${M}_sq_$WL" -o run \
      -- python3 "$R/bench.py" --workload $WL --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) \
      > gpurun_out/ser${M}_sq_$WL.txt 2>&1 || { echo "[ser${M}_sq] failed"; exit 3; }
  echo "[ser$M] ok"
done
