#!/bin/bash
# Round profile pass on one GPU box: for each workload in $WLS (default "c2 c3 c4 c5"):
#   rocprofv3 --kernel-trace --stats of a bench run, then separate --pmc passes (FETCH_SIZE,
#   WRITE_SIZE, one SQ pass).  Every step has its own time limit; the script stops at the first
#   failure.  Summaries: tools/pmc_summary.py / tools/sq_summary.py -> profiles/.
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
for W in ${WLS:-c2 c3 c4 c5}; do
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$W" -o run \
      -- python3 "$R/bench.py" --workload $W --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) \
      > gpurun_out/prof_$W.txt 2>&1 || { echo "[prof_$W] failed"; exit 2; }
  echo "[prof_$W] ok"
  [ -n "$STATS_ONLY" ] && continue
  for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"; do
    tag=$(echo $C | cut -d' ' -f1)
    ( cd /tmp && timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_${W}_$tag" -o run \
        -- python3 "$R/bench.py" --workload $W --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) \
        > gpurun_out/pmc_${W}_$tag.txt 2>&1 || { echo "[pmc_${W}_$tag] failed"; exit 3; }
    echo "[pmc_${W}_$tag] ok"
  done
done
echo ok
