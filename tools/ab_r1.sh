mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
run() { n=$1; shift; w=$1; shift; timeout -k 10 200 env "$@" python bench.py --workload $w --steps 3 --no-cpu-baseline --e2e-steps 0 > gpurun_out/ab_$n.txt 2>&1; }
for w in c2 c3 c4 c5; do
run ${w}_fd $w ICW_FILL_DRAIN=1 || exit 1
run ${w}_nofd $w ICW_FILL_DRAIN=0 || exit 1
done
for f in gpurun_out/ab_*.txt; do python -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')][0]; d=json.loads(l); r=d['roofline']
print('$f', round(d['value'],1), round(d['ms_per_step'],2), round(r['avg_launch_ms'],3), round(r['output_kernel_avg_launch_ms'],3))"; done
