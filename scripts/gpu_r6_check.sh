#!/bin/bash
# Round 6 host-side changes on the GPU: the handle / window suites, then a short config-2 bench
# (placement search with the bounded hold) and a second fresh process for its spread.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_handle.py tests/test_gpu_window.py -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/r6_check_pytest.txt 2>&1
rc=$?; tail -25 gpurun_out/r6_check_pytest.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --cpu-sample 0 --no-variants --dropin-frames 0 \
      > gpurun_out/r6_bench_$r.json 2> gpurun_out/r6_bench_$r.err || { echo "bench $r failed"; tail -20 gpurun_out/r6_bench_$r.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6_bench_$r.json')); p=d['workspace_placement']; print('run $r', d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['sclk_ghz'], p.get('probe_ms'), p.get('kept'), p.get('search_peak_gib_held'), p.get('workspace_gib'), p.get('peak_held_over_workspace'), p.get('launch_over_probe'), p.get('search_wall_ms'))"
done
