#!/bin/bash
# round 5: the whole GPU suite, smoke(), the default bench line (all variants, CPU baseline, drop-in)
# and a kernel trace of the default bench; outputs under gpurun_out/full/.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/full/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/full/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.txt 2>&1 || { tail -20 gpurun_out/full/smoke.txt; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err || { tail -20 gpurun_out/full/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/full/bench.json')); print(d['value'], d['roofline']['kernel_ms_avg']); v=d.get('variants',{}); [print(k, x.get('value'), (x.get('roofline') or {}).get('frac_of_binding')) for k,x in v.items() if isinstance(x, dict)]; print('dropin', json.dumps(d.get('dropin'))[:600])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/full/kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-sample 0 --no-variants --dropin-frames 0 > gpurun_out/full/kt.json 2> gpurun_out/full/kt.err || { tail -20 gpurun_out/full/kt.err; exit 1; }
echo done
