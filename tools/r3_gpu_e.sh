#!/bin/bash
# round 3 pass E: XCD-aware K1 workgroup order (I and Q waves of a group on one XCD) -- parity of the
# lane kernel, A/B on C3 / C4, a C4 FETCH pass with it
mkdir -p gpurun_out
R=$(pwd); export TMPDIR=/tmp
timeout -k 10 600 env ICW_K1_MODE=plain python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_live.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3e_pytest.txt 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -2 gpurun_out/r3e_pytest.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for lib in libicw_noremap.so libicw.so; do
    for w in c3 c4; do
      ICW_LIB=$lib timeout -k 10 200 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 \
        > gpurun_out/r3e_${w}_${lib}_$r.json 2>>gpurun_out/r3e_err.log || exit 3
    done
  done
done
echo "[ab] ok"
( cd /tmp && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_c4e_FETCH_SIZE" -o run \
    -- python3 "$R/bench.py" --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 ) > gpurun_out/pmc_c4e.txt 2>&1 || exit 4
( cd /tmp && timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_c4e_WRITE_SIZE" -o run \
    -- python3 "$R/bench.py" --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-other-workloads --e2e-steps 0 ) > gpurun_out/pmc_c4e_w.txt 2>&1 || exit 4
echo ok
