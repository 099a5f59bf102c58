#!/bin/bash
# round 3 pass D: K1r in two-wave workgroups -- parity of the row kernel, the round's profiles of
# C2 / C3 / C5 (kernel stats, FETCH / WRITE, SQ), the default bench line
mkdir -p gpurun_out
R=$(pwd); export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream1.py tests/test_gpu_full_size.py tests/test_gpu_graph_random.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3d_pytest.txt 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -2 gpurun_out/r3d_pytest.txt
[ $rc -eq 0 ] || exit 2
WLS="c2 c3 c5" timeout -k 10 900 bash tools/profile_round.sh > gpurun_out/r3d_profile.txt 2>&1 || { echo profile failed; exit 5; }
echo "[profile] ok"
timeout -k 10 900 python bench.py > gpurun_out/r3d_bench_default.json 2> gpurun_out/r3d_bench_default.err || { echo bench failed; exit 4; }
echo "[bench] ok"
