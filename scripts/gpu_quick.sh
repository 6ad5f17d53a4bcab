#!/bin/bash
# GPU box job for a kernel change: the GPU parity suite, one short bench line (no variants, no
# CPU baseline) and, with DIAG=1, the per-wave cycle split of the stamps build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
NOVAR=--no-variants; [ -n "$VARIANTS" ] && NOVAR=
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-sample 0 $NOVAR ${BENCH_ARGS} > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench_quick.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/bench_quick.json')); print('value', r['value'], 'kernel_ms', r['roofline']['kernel_ms_avg']); [print(k, v['value'], v['kernel_ms_avg']) for k, v in r.get('variants', {}).items()]"
if [ -n "$DIAG" ]; then
  timeout -k 10 300 python scripts/diag_stamps.py 4096 f64 logmap > gpurun_out/diag.log 2>&1 || { echo "diag failed"; tail -20 gpurun_out/diag.log; exit 1; }
  cat gpurun_out/diag.log
fi
