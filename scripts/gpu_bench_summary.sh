#!/bin/bash
# The driver's bench command (one fresh process) and a summary of its JSON line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SECONDS=0
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b.json 2> gpurun_out/b.err
rc=$?; echo "bench wall ${SECONDS}s rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/b.err; exit $rc; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/b.json"))
r = d["roofline"]
print("config 2", d["value"], d["ms_per_step"], r["kernel_ms_avg"], r["sclk_ghz"], r["latency_floor"]["frac"],
      d["workspace_placement"].get("launch_over_probe"), d["workspace_placement"].get("peak_held_over_workspace"))
for k, v in d["variants"].items():
    if "value" in v:
        w = v.get("roofline") or {}
        print(" ", k, v["value"], v.get("bit_errors"), w.get("binding"), w.get("frac_of_binding"), w.get("sclk_ghz"),
              w.get("sclk_source"))
print("ber gate", json.dumps(d["variants"].get("window_ber_gate")))
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["bits_match_gpu"], "dropin", d["dropin"].get("ms_per_frame"),
      d["dropin"].get("window", {}).get("ms_per_frame"))
PY
