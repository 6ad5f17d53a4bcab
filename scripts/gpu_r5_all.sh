#!/bin/bash
# round 5: windowed parity + config-5 A/B of the libvar_*.so builds (gpu_r5_window_ab.sh), then the
# product library's window PMC (gpu_r5_wpmc.sh); stops at the first failing step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r5_window_ab.sh && bash scripts/gpu_r5_wpmc.sh
