#!/bin/bash
# Round 6: the windowed schedule's one-read max* table.  Parity of every window test (both max*
# forms against the C restatement), the paired BER curve of both forms against the exact schedule,
# the bench's config-5 lines, then the PMC of the new default (scripts/gpu_window_pmc.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_window.py tests/test_gpu_handle.py tests/test_gpu_decode.py -k "window or graph" \
    -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_win_pytest.txt 2>&1
rc=$?; tail -8 gpurun_out/r6_win_pytest.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r6_win_pytest.txt | head -20; exit $rc; }
timeout -k 10 500 python -u scripts/ber_window_vs_exact.py --frames ${FRAMES:-262144} --out gpurun_out/ber_window_vs_exact.json \
    > gpurun_out/ber_paired.log 2>&1
rc=$?; tail -6 gpurun_out/ber_paired.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 1 --cpu-sample 0 --dropin-frames 8 > gpurun_out/r6_win_bench.json 2> gpurun_out/r6_win_bench.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/r6_win_bench.err; exit $rc; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r6_win_bench.json"))
print("config 2", d["value"], d["roofline"]["kernel_ms_avg"], d["roofline"]["sclk_ghz"])
for k, v in d["variants"].items():
    r = v.get("roofline") or {}
    print(k, v.get("value"), v.get("ms_per_step"), v.get("bit_errors"), r.get("sclk_ghz"), r.get("sclk_td_clock_read_ghz"))
dr = d.get("dropin", {})
print("dropin", dr.get("ms_per_frame"), (dr.get("window") or {}).get("ms_per_frame"), (dr.get("window") or {}).get("bit_errors"))
PY
bash scripts/gpu_window_pmc.sh > gpurun_out/r6_wpmc.txt 2>&1
rc=$?; cat gpurun_out/r6_wpmc.txt; exit $rc
