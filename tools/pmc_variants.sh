#!/bin/bash
# One SQ counter pass per in-tree library build on one workload (VALU accounting of diagnostic
# variants, tools/build_variant.sh):  LIBS="libicw.so libicw_cut1.so" W=c2fir TAG=r4c bash tools/pmc_variants.sh
# Output: gpurun_out/${TAG}_pmc_<lib>/ (rocprofv3 csv); every pass has its own time limit.
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-var}; W=${W:-c2fir}
C=${COUNTERS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM"}
for L in ${LIBS:-libicw.so}; do
  ( cd /tmp && ICW_LIB=$L timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/${TAG}_pmc_${L%.so}" -o run \
      -- python3 "$R/bench.py" --workload $W --steps ${STEPS:-1} --warmup 1 --no-cpu-baseline --e2e-steps 0 \
      --frames ${FRAMES:-262144} ) > gpurun_out/${TAG}_pmc_${L%.so}.txt 2>&1 || { echo "[pmc $L] failed"; exit 3; }
  echo "[pmc $L] ok"
done
echo ok
