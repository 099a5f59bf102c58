#!/bin/bash
# KF2's last tile beside the signature form on a side stream (ICW_FIR_SIDE=1, default) against after
# it on the same stream (0): the FIR parity suites, then the A/B on c2fir / c4fir / c3fir
mkdir -p gpurun_out; TAG=${TAG:-r6t}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fir_sig.py tests/test_gpu_fir.py tests/test_gpu_sig_fast.py \
    tests/test_gpu_production_random.py tests/test_gpu_full_size.py tests/test_gpu_dither_flat.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
VAR=ICW_FIR_SIDE VALS="1 0" WLS="c2fir c4fir c3fir" REPS=3 STEPS=3 TAG=${TAG}ab bash tools/env_ab.sh || exit 3
