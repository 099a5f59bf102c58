#!/bin/bash
# round 3 pass G: chain-form DSP programs (no LDS register file) and the K5 rework (batched K0
# loads, rotation table beside the recurrence): parity, the chain A/B, C1 timing and phase stamps
mkdir -p gpurun_out
R=$(pwd); export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3g_pytest_gpu.txt 2>&1
rc=$?; echo "[pytest_gpu] rc=$rc"; tail -2 gpurun_out/r3g_pytest_gpu.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for ch in 0 1; do
    for w in c2 c4 c2fir c4fir; do
      ICW_CHAIN=$ch timeout -k 10 200 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
        > gpurun_out/r3g_ch${ch}_${w}_$r.json 2>>gpurun_out/r3g_err.log || exit 3
    done
  done
done
echo "[chain ab] ok"
timeout -k 10 300 python -u bench.py --workload c1 --steps 3 --warmup 1 > gpurun_out/r3g_c1.json 2>>gpurun_out/r3g_err.log || exit 4
tail -1 gpurun_out/r3g_c1.json
python tools/c1_wav.py /tmp/c1.wav 10 || exit 5
ICW_TIMING=1 ICW_S1_STAMPS=1 timeout -k 10 120 ./examples/icw_transcode /tmp/c1.wav /tmp/c1_out.wav 576 shift 16 \
    > gpurun_out/r3g_c1_576.json 2> gpurun_out/r3g_c1_576.stamps || exit 6
python tools/s1_phases.py gpurun_out/r3g_c1_576.stamps
echo ok
