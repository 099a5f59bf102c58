#!/bin/bash
# Frame-parallel dithered flat renders: their GPU tests, the c2fir / c2 TPDF + flat A/B (ICW_DITH_PAR
# 1 = frame-parallel, 0 = serial render), then the whole -m gpu suite
mkdir -p gpurun_out; TAG=${TAG:-r6e}
timeout -k 10 400 python -u -m pytest tests/test_gpu_dither_flat.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_dith_tests.txt 2>&1
rc=$?; echo "[dither tests] rc=$rc"; tail -3 gpurun_out/${TAG}_dith_tests.txt; [ $rc -eq 0 ] || exit 2
export ICW_BENCH_RENDER=tpdf_flat
VAR=ICW_DITH_PAR VALS="1 0" WLS="c2fir c2" REPS=1 STEPS=2 TAG=${TAG}ab bash tools/env_ab.sh || exit 3
unset ICW_BENCH_RENDER
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_suite.txt 2>&1
rc=$?; echo "[suite] rc=$rc"; tail -3 gpurun_out/${TAG}_suite.txt; exit $rc
