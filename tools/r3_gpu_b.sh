#!/bin/bash
# round 3: parity of the one-row hand-off / even-order K1 zero steps / KF2 table variant, then
# the FIR staging A/B, the C3 / C4 benches and a PMC + SQ profile of C4 and C2-FIR
mkdir -p gpurun_out
R=$(pwd); export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3b_pytest_gpu.txt 2>&1
rc=$?; echo "[pytest_gpu] rc=$rc"; tail -3 gpurun_out/r3b_pytest_gpu.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for lib in libicw_nostage.so libicw.so; do
    for w in c2fir c3fir c4fir; do
      ICW_LIB=$lib timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
        > gpurun_out/r3ab_${w}_${lib}_$r.json 2>>gpurun_out/r3ab_err.log || exit 3
    done
  done
done
echo "[fir ab] ok"
for w in c3 c4 c5; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
    > gpurun_out/r3b_bench_$w.json 2>>gpurun_out/r3ab_err.log || exit 4
done
echo "[bench c3 c4 c5] ok"
WLS="c4 c2fir" timeout -k 10 900 bash tools/profile_round.sh > gpurun_out/r3b_profile.txt 2>&1 || { echo profile failed; exit 5; }
echo "[profile] ok"
