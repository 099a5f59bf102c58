#!/bin/bash
# KF2 mono with a rotating node (C3 shape, Shift -> Master): WRITE_SIZE and throughput, working tree vs $PREV
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out; PREV=${PREV:-libicw_met.so}
for L in $PREV libicw.so; do
  ( cd /tmp && ICW_BENCH_GRAPH=shift_master ICW_LIB=$L timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/r5mr_w_${L%.so}" -o run \
      -- python3 "$R/bench.py" --workload c3fir --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/r5mr_w_${L%.so}.txt 2>&1 || { echo "[pmc $L] failed"; exit 3; }
  echo "[pmc $L] ok"
done
ICW_BENCH_GRAPH=shift_master TAG=r5mr LIBS="$PREV libicw.so" WLS="c3fir" REPS=3 bash tools/ab_bench.sh
