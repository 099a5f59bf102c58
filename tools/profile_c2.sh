#!/bin/bash
# One GPU call: the default bench line (with the CPU baseline), the rocprofv3 kernel-trace stats of
# the same command, and the two PMC passes (FETCH_SIZE / WRITE_SIZE) for the HBM traffic.
# Every step has its own time limit; the script stops at the first failure.
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.txt 2>&1 || exit 2
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_c2" -o run \
    -- python3 "$R/bench.py" --no-cpu-baseline ) > gpurun_out/prof_c2.txt 2>&1 || exit 3
for C in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o run \
      -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ) > gpurun_out/pmc_$C.txt 2>&1 || exit 4
done
echo ok
