#!/bin/bash
# c5fir A/B on one box: the committed build (libicw_prev.so) against the working tree with K3r's
# clamp-free blocks on and off (ICW_K3R_SPEC), then kernel-trace stats of each.
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r5k3rb}
run() {  # lib spec rep
  ICW_LIB=$1 ICW_K3R_SPEC=$2 timeout -k 10 200 python -u bench.py --workload ${W:-c5fir} --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 \
     > gpurun_out/${TAG}_${1%.so}_s$2_$3.json 2>>gpurun_out/${TAG}_err.log || { echo "bench $1 $2 failed"; exit 3; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline'].get('output_kernel_avg_launch_ms',0),3))" \
     gpurun_out/${TAG}_${1%.so}_s$2_$3.json "$1 spec=$2"
}
for r in 1 2; do
  run libicw_prev.so 1 $r; run libicw.so 1 $r; run libicw.so 0 $r
done
for L in libicw_prev.so libicw.so; do
  ( cd /tmp && ICW_LIB=$L timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/${TAG}_trace_${L%.so}" -o run \
      -- python3 "$OLDPWD/bench.py" --workload ${W:-c5fir} --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/${TAG}_trace_${L%.so}.txt 2>&1 || { echo "trace $L failed"; exit 4; }
  echo "trace $L ok"
done
echo all-ok
