#!/bin/bash
# The driver's round-end sequence on one box: the GPU test suite, smoke(), the bench (full variants),
# then a kernel trace of a short bench run; everything under gpurun_out/ (copy what is kept into
# profiles/rNN/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/round_pytest_gpu.txt 2>&1
rc=$?; tail -5 gpurun_out/round_pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/round_pytest_gpu.txt | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round_smoke.txt 2>&1
rc=$?; cat gpurun_out/round_smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/round_bench.json 2> gpurun_out/round_bench.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/round_bench.err; exit $rc; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/round_bench.json"))
r = d["roofline"]
print("config 2", d["value"], d["ms_per_step"], r["kernel_ms_avg"], r["sclk_ghz"], r["latency_floor"]["frac"],
      d["workspace_placement"].get("peak_held_over_workspace"), d["cpu_baseline"]["value"], d["cpu_baseline"]["bits_match_gpu"])
for k, v in d["variants"].items():
    w = v.get("roofline") or {}
    print(" ", k, v.get("value"), v.get("bit_errors"), w.get("binding"), w.get("frac_of_binding"), w.get("lane_valu_per_position"))
print("dropin", d["dropin"].get("ms_per_frame"), d["dropin"].get("window", {}).get("ms_per_frame"))
PY
rm -rf gpurun_out/prof
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o kt --output-format csv -- python3 bench.py --steps 8 --warmup 1 \
    --cpu-sample 0 --no-variants --dropin-frames 0 > gpurun_out/round_prof.log 2>&1
rc=$?; tail -3 gpurun_out/round_prof.log; find gpurun_out/prof -name "*kernel_stats.csv" | head -3; exit $rc
