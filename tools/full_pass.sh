#!/bin/bash
# The round-end pass on this tree: the full -m gpu suite, smoke, and the driver's default bench command
# (TAG names the outputs under gpurun_out/).  Every step has its own time limit.
mkdir -p gpurun_out; TAG=${TAG:-full}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?; echo "[pytest] rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.txt
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1; echo "[smoke] rc=$?"; tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; echo "[bench] rc=$?"
python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json'))
print('C2', round(d['value'],1), d['roofline']['frac'], 'cpu', round(d['cpu_baseline']['value'],1))
for k,v in d.get('other_workloads',{}).items(): print(k, round(v.get('value',0),1), v.get('fir_tflops'))
"
