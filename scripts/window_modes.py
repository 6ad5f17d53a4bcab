"""Windowed-schedule options at config 5 (K=6144, 8 iterations, f64 log-MAP): bit errors against
the exact schedule on the same generator frames, and decode time at B=32768."""
import sys
import time

import torch

sys.path.insert(0, ".")
from turbo_decoder_cuda_amd import TurboCodec  # noqa: E402

MODES = [("exact", 0, 0, False), ("W64 g30", 64, 30, False), ("W64 g0 NII", 64, 0, True),
         ("W64 g12 NII", 64, 12, True), ("W64 g30 NII", 64, 30, True), ("W64 g63", 64, 63, False)]


def main():
    K, it = 6144, 8
    out = []
    with TurboCodec(K, 263, 480, iterations=it) as c:
        frames = {}
        for eb in (0.4, 0.5):
            c.synth_seed(7)
            frames[eb] = c.synth(8192, eb)
        big = torch.cat([frames[0.5][1]] * 4)   # 32768 codewords for timing
        for name, W, g, nii in MODES:
            c.set_window(W, g, 1.0, nii=nii)
            errs = {}
            for eb, (info, llr) in frames.items():
                bits = torch.empty((llr.shape[0], it, K), dtype=torch.uint8, device=llr.device)
                c.decode(llr, bits, all_iters=True)
                e = c.count_errors(bits, info)[:, -1]
                errs[eb] = (int(e.sum()), int((e > 0).sum()))
            bb = torch.empty((big.shape[0], K), dtype=torch.uint8, device=big.device)
            c.decode(big, bb)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(2):
                c.decode(big, bb)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 2
            line = f"{name:14s} errors(bits, blocks) 0.4 dB {errs[0.4]}  0.5 dB {errs[0.5]}   B=32768: {dt * 1e3:.1f} ms = {32768 * K / dt / 1e6:.0f} Mbit/s"
            print(line, flush=True)
            out.append(line)


if __name__ == "__main__":
    main()
