#!/bin/bash
# GPU parity suites touched by the meters / fused-converter changes, then the FIR legs against $PREV on one box
mkdir -p gpurun_out; TAG=${TAG:-r5kf2b}; PREV=${PREV:-libicw_head.so}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_sig_fast.py tests/test_gpu_full_size.py tests/test_gpu_production_random.py tests/test_gpu_unaligned.py tests/test_gpu_amod.py tests/test_gpu_stream1.py tests/test_gpu_graph_random.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit 2
for r in 1 2; do for W in ${WLS:-c2fir c4fir c3fir}; do for L in $PREV libicw.so; do
  ICW_LIB=$L timeout -k 10 200 python -u bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 > gpurun_out/${TAG}_${W}_${L%.so}_$r.json 2>>gpurun_out/${TAG}_err.log || { echo "bench failed"; exit 6; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value'],1), round(d['roofline'].get('achieved',0),2))" gpurun_out/${TAG}_${W}_${L%.so}_$r.json "$W $L"
done; done; done
echo all-ok
