#!/bin/bash
# round 3 pass C: parity, then the K1 workgroup A/B (1 or 2 waves: the I and Q filters of 32 streams
# on one CU share the channel rows in its L2 / L1), the FIR legs, a c2fir PMC pass, traces
mkdir -p gpurun_out
R=$(pwd); export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3c_pytest_gpu.txt 2>&1
rc=$?; echo "[pytest_gpu] rc=$rc"; tail -2 gpurun_out/r3c_pytest_gpu.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for wg in 1 2; do
    for w in c2 c3 c4 c5; do
      ICW_K1_WG=$wg timeout -k 10 200 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
        > gpurun_out/r3c_wg${wg}_${w}_$r.json 2>>gpurun_out/r3c_err.log || exit 3
    done
  done
done
echo "[k1 wg ab] ok"
for w in c2fir c3fir c4fir c5fir; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
    > gpurun_out/r3c_bench_$w.json 2>>gpurun_out/r3c_err.log || exit 4
done
echo "[fir] ok"
WLS="c2fir" timeout -k 10 600 bash tools/profile_round.sh > gpurun_out/r3c_profile.txt 2>&1 || { echo profile failed; exit 5; }
echo "[profile c2fir] ok"
for W in c3 c4; do WL=$W TAG=r3c timeout -k 10 400 bash tools/trace_wl.sh || exit 6; done
timeout -k 10 400 bash tools/trace_c1.sh || exit 7
echo ok
