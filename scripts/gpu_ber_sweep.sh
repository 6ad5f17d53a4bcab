#!/bin/bash
# BER/BLER sweep on the GPU with the reference's settings (main.cpp:36-41: K=6144, Eb/N0 0..1 step
# 0.1, <= 100000 frames, stop at 50 block errors) at 8 iterations; result.txt format.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
rm -f gpurun_out/ber_K6144_result.txt
timeout -k 10 900 python -m turbo_decoder_cuda_amd.ber --K 6144 --iters 8 --ebn0 0 1 0.1 --seed 1 \
    --max-frames ${MAXF:-100000} --out gpurun_out/ber_K6144_result.txt > gpurun_out/ber_sweep.log 2> gpurun_out/ber_sweep.err
rc=$?; echo "elapsed ${SECONDS}s"; tail -15 gpurun_out/ber_sweep.err; cat gpurun_out/ber_sweep.log; exit $rc
