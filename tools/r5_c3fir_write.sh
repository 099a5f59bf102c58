#!/bin/bash
# c3fir WRITE_SIZE per library (which revision added the extra writes), then the NTAP A/B
R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
for L in libicw_r4.so libicw_pad.so libicw_met.so libicw.so; do
  ( cd /tmp && ICW_LIB=$L timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/r5w_${L%.so}" -o run \
      -- python3 "$R/bench.py" --workload c3fir --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0 ) > gpurun_out/r5w_${L%.so}.txt 2>&1 || { echo "[pmc $L] failed"; exit 3; }
  python3 - "$R/gpurun_out/r5w_${L%.so}" $L <<'PY'
import csv,glob,sys,collections
t=collections.defaultdict(float); n=collections.defaultdict(set)
for f in glob.glob(sys.argv[1]+'/**/*counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        t[r['Kernel_Name'][:40]]+=float(r['Counter_Value']); n[r['Kernel_Name'][:40]].add(r['Dispatch_Id'])
for k in t: print(sys.argv[2], k, round(t[k]/len(n[k])/1e6,3), 'GB per dispatch' if False else 'GB(KB/1e6) per dispatch')
PY
done
TAG=r5nt LIBS="libicw.so libicw_nt4o4.so libicw_nt4o5.so" WLS="c2fir c4fir c3fir" REPS=2 bash tools/ab_bench.sh
