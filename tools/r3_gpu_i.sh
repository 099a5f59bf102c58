#!/bin/bash
# round 3 pass I: the format-specialised unpack (typed loads when aligned) and the stereo FIR
# staging: misaligned-input parity, FIR / stream1 parity, the FIR legs and C1 again
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_unaligned.py tests/test_gpu_fir.py tests/test_gpu_stream1.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3i_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/r3i_tests.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for w in c2fir c3fir c4fir c5fir; do
    timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
      > gpurun_out/r3i_${w}_$r.json 2>>gpurun_out/r3i_err.log || exit 3
  done
done
echo "[fir legs] ok"
timeout -k 10 300 python -u bench.py --workload c1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r3i_c1.json 2>>gpurun_out/r3i_err.log || exit 4
tail -1 gpurun_out/r3i_c1.json
python tools/c1_wav.py /tmp/c1.wav 10 || exit 5
ICW_TIMING=1 ICW_S1_STAMPS=1 timeout -k 10 120 ./examples/icw_transcode /tmp/c1.wav /tmp/c1_out.wav 576 shift 16 \
    > gpurun_out/r3i_c1_576.json 2> gpurun_out/r3i_c1_576.stamps || exit 6
python tools/s1_phases.py gpurun_out/r3i_c1_576.stamps
echo ok
