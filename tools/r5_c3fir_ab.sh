#!/bin/bash
# mono KF2 parity (FIR suites), c3fir WRITE_SIZE of the working tree, then c3fir / c2fir A/B against $PREV
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out; PREV=${PREV:-libicw_met.so}
timeout -k 10 700 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_sig_fast.py tests/test_gpu_full_size.py tests/test_gpu_production_random.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5m_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -2 gpurun_out/r5m_tests.txt; [ $rc -eq 0 ] || exit 2
for L in libicw.so; do
  ( cd /tmp && ICW_LIB=$L timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/r5m_w_${L%.so}" -o run \
      -- python3 "$R/bench.py" --workload c3fir --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/r5m_w_${L%.so}.txt 2>&1 || { echo "[pmc $L] failed"; exit 3; }
  echo "[pmc $L] ok"
done
TAG=r5m LIBS="$PREV libicw.so" WLS="c3fir c2fir" REPS=2 bash tools/ab_bench.sh
