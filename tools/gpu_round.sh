#!/bin/bash
# GPU-box driver: each GPU step under its own timeout; stop at the first crash/timeout.
# Test failures (pytest rc 1) do not stop later steps; faults (rc >= 124, 134, 139) do.
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
step() {   # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "[$name] rc=$rc" | tee -a gpurun_out/steps.txt
  return $rc
}
for s in "$@"; do
  case $s in
    probe) step lat_probe 60 ./tools/lat_probe || exit 2 ;;
    k1probe) step k1_probe 120 ./tools/k1_probe 256 8192 || exit 2 ;;
    test)  step pytest_gpu 900 python -m pytest tests -m gpu -q -x; ok $? || exit 2 ;;
    testall) step pytest_gpu 900 python -m pytest tests -m gpu -q; ok $? || exit 2 ;;
    bench) step bench 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 2 ;;
    benchfull) step bench_full 900 python bench.py || exit 2 ;;
    benchall)
      for w in c2 c3 c4 c5; do
        step bench_$w 600 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline || exit 2
      done ;;
    crctest) step pytest_crc 600 python -m pytest tests/test_gpu_crc.py tests/test_gpu_cwave_graph.py -q -x; ok $? || exit 2 ;;
    crcprof)
      R=$(pwd); export TMPDIR=/tmp
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/crcprof" -o run \
          -- python3 "$R/tools/bench_crc.py" --gib 4 --iters 5 ) > gpurun_out/crcprof.txt 2>&1
      rc=$?; echo "[crcprof] rc=$rc" | tee -a gpurun_out/steps.txt; [ $rc -eq 0 ] || exit 2 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 2 ;;
    prof)
      R=$(pwd); export TMPDIR=/tmp
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
          -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ) > gpurun_out/prof.txt 2>&1
      rc=$?; echo "[prof] rc=$rc" | tee -a gpurun_out/steps.txt; [ $rc -eq 0 ] || exit 2 ;;
    profw)   # kernel stats of one workload: WL=c5 bash tools/gpu_round.sh profw
      R=$(pwd); export TMPDIR=/tmp
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$WL" -o run \
          -- python3 "$R/bench.py" --workload "$WL" --steps 2 --warmup 1 --no-cpu-baseline ) > gpurun_out/prof_$WL.txt 2>&1
      rc=$?; echo "[prof_$WL] rc=$rc" | tee -a gpurun_out/steps.txt; [ $rc -eq 0 ] || exit 2 ;;
    profser)   # standalone kernel times: every kernel on one stream
      R=$(pwd); export TMPDIR=/tmp; export ICW_SERIALIZE=1
      ( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/profser_$WL" -o run \
          -- python3 "$R/bench.py" --workload "$WL" --steps 2 --warmup 1 --no-cpu-baseline ) > gpurun_out/profser_$WL.txt 2>&1
      rc=$?; unset ICW_SERIALIZE; echo "[profser_$WL] rc=$rc" | tee -a gpurun_out/steps.txt; [ $rc -eq 0 ] || exit 2 ;;
    pmc)
      R=$(pwd); export TMPDIR=/tmp
      ( cd /tmp && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run \
          -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ) > gpurun_out/pmc_fetch.txt 2>&1
      rc=$?; echo "[pmc_fetch] rc=$rc" | tee -a gpurun_out/steps.txt; [ $rc -eq 0 ] || exit 2
      ( cd /tmp && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o run \
          -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ) > gpurun_out/pmc_write.txt 2>&1
      rc=$?; echo "[pmc_write] rc=$rc" | tee -a gpurun_out/steps.txt; [ $rc -eq 0 ] || exit 2 ;;
  esac
done
