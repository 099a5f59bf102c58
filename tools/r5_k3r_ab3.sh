#!/bin/bash
# K3r: GPU parity (row render, clamp-free blocks) then the c5fir A/B against the committed build
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_render_spec.py tests/test_gpu_parity.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5k3rc_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -2 gpurun_out/r5k3rc_tests.txt; [ $rc -eq 0 ] || exit 2
TAG=r5k3rc bash tools/r5_k3r_ab2.sh
