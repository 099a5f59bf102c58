#!/bin/bash
# K1r A/B on one GPU box: the row-kernel GPU parity files, then C2 / C5 bench runs alternating an
# older in-tree build (in_cwave_amd/libicw_ab_old.so, built beforehand) with the current one (ICW_LIB).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_live.py tests/test_gpu_fpcheck.py tests/test_c_host.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || exit 1
for r in 1 2; do
  for lib in libicw_ab_old.so libicw.so; do
    ICW_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-other-workloads --steps 5 > gpurun_out/ab_c2_${lib}_$r.json 2>gpurun_out/ab_err.log || exit 2
    ICW_LIB=$lib timeout -k 10 120 python -u bench.py --workload c5 --no-cpu-baseline --no-other-workloads --steps 3 > gpurun_out/ab_c5_${lib}_$r.json 2>>gpurun_out/ab_err.log || exit 3
  done
done
