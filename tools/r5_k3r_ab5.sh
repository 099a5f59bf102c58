#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp; R=$(pwd); TAG=${TAG:-r5k3re}
timeout -k 10 600 python -u -m pytest tests/test_gpu_render_spec.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
for L in libicw.so libicw_prev.so; do
  ( cd /tmp && ICW_LIB=$L timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_trace_${L%.so}" -o run \
      -- python3 "$R/bench.py" --workload c5fir --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_trace_${L%.so}.txt 2>&1 || { echo "trace $L failed"; exit 4; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_trace_${L%.so}/run_kernel_stats.csv')):
    if 'render_row' in r['Name']: print('$L', r['Name'][:40], r['AverageNs'])"
done
for r in 1 2; do for W in c5fir; do for L in libicw_prev.so libicw.so; do
  ICW_LIB=$L timeout -k 10 200 python -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > gpurun_out/${TAG}_${W}_${L%.so}_$r.json 2>>gpurun_out/${TAG}_err.log || { echo "bench failed"; exit 6; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value'],1))" gpurun_out/${TAG}_${W}_${L%.so}_$r.json "$W $L"
done; done; done
TAG=r5k3rf_sq bash tools/r5_k3r_sq.sh || exit 7
echo all-ok
