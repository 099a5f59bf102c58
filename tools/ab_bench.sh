#!/bin/bash
# A/B bench on one GPU box, the one parametrised script for builder sessions (replaces the
# round-3 one-off tools/r3_gpu_*.sh):
#   TESTS="tests/test_gpu_parity.py ..."  GPU tests to run first (optional; the A/B runs only if green)
#   LIBS="libicw.so libicw_prev.so"       in-tree libraries to compare (ICW_LIB; tools/ab_rev.sh builds them)
#   WLS="c5 c5fir"  REPS=2  STEPS=3       workloads, alternating repetitions, timed steps
#   TAG=r4x                               output prefix under gpurun_out/
# Every GPU step has its own time limit; the script stops at the first failure.
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread \
      > gpurun_out/${TAG}_tests.txt 2>&1
  rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt
  [ $rc -eq 0 ] || exit 2
fi
for r in $(seq 1 ${REPS:-2}); do
  for W in ${WLS:-c5}; do
    for L in ${LIBS:-libicw.so}; do
      ICW_LIB=$L timeout -k 10 ${BENCH_LIMIT:-200} python -u bench.py --workload $W --steps ${STEPS:-3} --warmup 1 \
          --no-cpu-baseline --e2e-steps 0 > gpurun_out/${TAG}_${W}_${L%.so}_$r.json 2>>gpurun_out/${TAG}_err.log \
          || { echo "[bench $W $L $r] failed"; exit 3; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], sys.argv[4], round(d['value'],1), round(d['ms_per_step'],3))" \
          gpurun_out/${TAG}_${W}_${L%.so}_$r.json $W $L $r
    done
  done
done
echo ok
