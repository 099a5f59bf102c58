#!/bin/bash
# The signature form as the default: its own test and the FIR suites, then the round's profile pass
# of the FIR legs (kernel-trace stats, FETCH / WRITE / SQ passes; tools/round_profiles.sh summarises)
mkdir -p gpurun_out; TAG=${TAG:-r6j}
timeout -k 10 700 python -u -m pytest tests/test_gpu_fir_sig.py tests/test_gpu_fir.py tests/test_gpu_sig_fast.py \
    tests/test_gpu_full_size.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
WLS="c2fir c4fir c3fir" bash tools/profile_round.sh || exit 3
