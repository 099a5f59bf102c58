#!/bin/bash
# round 3 pass T: KF2 stereo I/Q exchange by v_permlane32_swap (A) against HEAD (B, libicw_prev.so):
# FIR parity, the FIR legs twice each, then one SQ pass of c2fir for A
R=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_unaligned.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3t_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/r3t_tests.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for lib in ${LIBS:-libicw.so libicw_prev.so}; do
    for w in ${WLS:-c2fir c3fir c4fir}; do
      ICW_LIB=$lib timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
        > gpurun_out/r3t_${lib%.so}_${w}_$r.json 2>>gpurun_out/r3t_err.log || exit 3
    done
  done
done
echo "[legs] ok"
ICW_LIB=libicw_stp.so timeout -k 10 200 python -u tools/fir_phases.py c2fir c4fir c3fir > gpurun_out/r3t_fir_phases.jsonl 2>>gpurun_out/r3t_err.log || exit 5
cat gpurun_out/r3t_fir_phases.jsonl
( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv -d "$R/gpurun_out/r3t_sq" -o run \
    -- python3 "$R/bench.py" --workload c2fir --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/r3t_sq.txt 2>&1 || exit 4
echo ok
