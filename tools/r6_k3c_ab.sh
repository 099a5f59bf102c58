set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_render_spec.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6a_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/r6a_tests.txt; [ $rc -eq 0 ] || exit 2
ICW_K3R_COMP=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_render_spec.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6a_tests_c0.txt 2>&1
rc=$?; echo "[tests comp0] rc=$rc"; tail -3 gpurun_out/r6a_tests_c0.txt; [ $rc -eq 0 ] || exit 2
LIBS="libicw.so libicw_r5.so" WLS="c5fir c5" REPS=2 TAG=r6a bash tools/ab_bench.sh
