#!/bin/bash
# KF2's mono signature form with both channels as one computation (IcwFirArgs.lr_same): the FIR
# parity suites, then c3fir against the previous build (libicw_head.so) in alternating runs
mkdir -p gpurun_out; TAG=${TAG:-r6u}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fir_sig.py tests/test_gpu_fir.py tests/test_gpu_sig_fast.py \
    tests/test_gpu_production_random.py tests/test_gpu_full_size.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
LIBS="libicw.so libicw_head.so" WLS="c3fir" REPS=3 STEPS=3 TAG=${TAG}ab bash tools/ab_bench.sh || exit 3
