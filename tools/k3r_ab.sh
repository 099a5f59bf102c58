#!/bin/bash
mkdir -p gpurun_out
TAG=r5k3r
timeout -k 10 600 python -u -m pytest tests/test_gpu_render_spec.py tests/test_gpu_parity.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt
[ $rc -eq 0 ] || exit 2
for r in 1 2; do
  for S in 1 0; do
    ICW_K3R_SPEC=$S timeout -k 10 200 python -u bench.py --workload c5fir --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > gpurun_out/${TAG}_c5fir_s${S}_$r.json 2>>gpurun_out/${TAG}_err.log || { echo "bench failed"; exit 3; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value'],1), round(d['ms_per_step'],3))" gpurun_out/${TAG}_c5fir_s${S}_$r.json spec=$S
  done
done
