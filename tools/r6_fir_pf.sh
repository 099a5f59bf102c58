#!/bin/bash
# KF2 signature form as persistent workgroups with the DMA look-ahead: the FIR suites, then the A/B
# against the one-tile-per-workgroup form (libicw_sig1.so, 5e6ca1a) and without the look-ahead
# (ICW_FIR_PREFETCH=0) on c2fir / c4fir / c3fir, then an SQ pass of c2fir
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd); TAG=${TAG:-r6k}
timeout -k 10 700 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_fir_sig.py tests/test_gpu_fir.py tests/test_gpu_sig_fast.py \
    tests/test_gpu_production_random.py tests/test_gpu_full_size.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
for r in 1 2; do
  LIBS="libicw.so libicw_sig1.so" WLS="${WLS:-c2fir c4fir c3fir}" REPS=1 STEPS=3 TAG=${TAG}ab$r bash tools/ab_bench.sh || exit 3
  VAR=ICW_FIR_PREFETCH VALS="0" WLS="${WLS:-c2fir c4fir c3fir}" REPS=1 STEPS=3 TAG=${TAG}np$r bash tools/env_ab.sh || exit 3
done
LIBS="libicw.so" W=c2fir TAG=${TAG}sq bash tools/sq_pass.sh || exit 3
echo "profiles ok"
