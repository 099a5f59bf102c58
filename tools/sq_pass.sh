#!/bin/bash
# SQ counter passes of one workload per in-tree library (A/B builds: tools/build_variant.sh, ab_rev.sh):
#   LIBS="libicw.so libicw_x.so" W=c5fir FRAMES=262144 TAG=x bash tools/sq_pass.sh
# Two counter sets per library (instruction counts; active / wait cycles), each in its own rocprofv3 run
# with its own time limit -> gpurun_out/${TAG}_<lib>_<set>/; summaries: tools/sq_summary.py.
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd); TAG=${TAG:-sq}
for L in ${LIBS:-libicw.so}; do
  for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM" \
           "SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU"; do
    n=$(echo $C | cut -d' ' -f2)
    ( cd /tmp && ICW_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/${TAG}_${L%.so}_$n" -o run \
        -- python3 "$R/bench.py" --workload ${W:-c5fir} --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 \
        ${FRAMES:+--frames $FRAMES} ) > gpurun_out/${TAG}_${L%.so}_$n.txt 2>&1 || { echo "[sq $L $n] failed"; exit 3; }
    echo "[sq $L $n] ok"
  done
done
echo ok
