#!/bin/bash
# Round 6: config 5's BER curve against the exact schedule.
#  1. paired: the same frames through both schedules at every point (scripts/ber_window_vs_exact.py)
#  2. main.cpp's own protocol (0..1 dB step 0.1, <= 100000 frames, 50 block errors) for the windowed
#     schedule, result.txt format, beside profiles/r05/ber_K6144_8it_result.txt (the exact one)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
FR=${FRAMES:-262144}
timeout -k 10 400 python -u scripts/ber_window_vs_exact.py --frames $FR --out gpurun_out/ber_window_vs_exact.json \
    > gpurun_out/ber_paired.log 2>&1
rc=$?; cat gpurun_out/ber_paired.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ber_K6144_w64g30_result.txt
timeout -k 10 300 python -u -m turbo_decoder_cuda_amd.ber --K 6144 --iters 8 --ebn0 0 1 0.1 --seed 1 \
    --max-frames 100000 --batch 32768 --window 64 --overlap 30 --out gpurun_out/ber_K6144_w64g30_result.txt \
    > gpurun_out/ber_w64_sweep.log 2> gpurun_out/ber_w64_sweep.err
rc=$?; echo "elapsed ${SECONDS}s"; tail -15 gpurun_out/ber_w64_sweep.err; cat gpurun_out/ber_w64_sweep.log; exit $rc
