"""Monte-Carlo BER/BLER harness on the MI355X: ITTC/main.cpp:170-315.

Per Eb/N0 point the reference decodes frames of its rand() stream until the last iteration has
`min_block_errors` block errors (main.cpp:239-243) or `max_frames` frames, counting per iteration
the bit errors and the frames with at least one bit error (main.cpp:224-237).  Here the frames
come from the device generator (bit-identical to main.cpp's frames of the same srand seed), are
decoded in batches on the GPU, and the per-frame error counts are replayed in frame order on the
host so the stopping frame -- and therefore every count -- is exactly the reference's.  Frames of
a batch past the stopping frame are discarded and the stream is repositioned after the stopping
frame, so the next Eb/N0 point continues the stream as main.cpp does.

    python -m turbo_decoder_cuda_amd.ber --K 6144 --iters 8 --ebn0 0 1 0.1 --seed 1 --out result.txt
"""
from __future__ import annotations

import argparse
import math
import sys
from dataclasses import dataclass, field

from .decoder import TurboCodec, stream_length


@dataclass
class BerPoint:
    ebn0_db: float
    frames: int = 0
    bit_errors: list = field(default_factory=list)     # per iteration
    block_errors: list = field(default_factory=list)   # per iteration
    K: int = 0

    @property
    def ber(self):
        return [e / (self.frames * self.K) if self.frames else math.nan for e in self.bit_errors]

    @property
    def bler(self):
        return [e / self.frames if self.frames else math.nan for e in self.block_errors]


def ber_point(codec: TurboCodec, ebn0_db: float, max_frames: int, min_block_errors: int = 50, batch: int = 4096,
              stop_iter: int | None = None) -> BerPoint:
    """One Eb/N0 point from the codec's current frame-stream position (codec.synth_seed first)."""
    import torch

    iters = codec.iterations
    stop_it = iters - 1 if stop_iter is None else stop_iter
    dev = torch.device("cuda", codec.device)
    n = stream_length(codec.K)
    info = torch.empty((batch, codec.K), dtype=torch.uint8, device=dev)
    llr64 = torch.empty((batch, n), dtype=torch.float64, device=dev)
    bits = torch.empty((batch, iters, codec.K), dtype=torch.uint8, device=dev)
    pt = BerPoint(ebn0_db, 0, [0] * iters, [0] * iters, codec.K)
    start = _frame_position(codec)
    done = False
    while not done and pt.frames < max_frames:
        B = min(batch, max_frames - pt.frames)
        codec.synth(B, ebn0_db, info[:B], llr64[:B])
        x = llr64[:B] if codec.precision == "f64" else llr64[:B].float()
        codec.decode(x, bits[:B], all_iters=True)
        err = codec.count_errors(bits[:B], info[:B]).cpu().numpy()
        for b in range(B):   # main.cpp's frame loop, in order
            pt.frames += 1
            for it in range(iters):
                pt.bit_errors[it] += int(err[b, it])
                pt.block_errors[it] += int(err[b, it] != 0)
            if min_block_errors > 0 and pt.block_errors[stop_it] >= min_block_errors:
                done = True
                break
    codec.synth_seek(start + pt.frames)   # the stream continues right after the last counted frame
    codec._frame_pos = start + pt.frames
    return pt


def _frame_position(codec: TurboCodec) -> int:
    return getattr(codec, "_frame_pos", 0)


def ber_sweep(codec: TurboCodec, ebn0_list, seed: int, max_frames: int, min_block_errors: int = 50,
              batch: int = 4096, reseed_each_point: bool = False, log=None):
    """main.cpp's sweep: srand(seed) once, then the Eb/N0 points on the continuing stream
    (or srand(seed) per point with reseed_each_point, like oracle/ref_harness's `ber` mode)."""
    codec.synth_seed(seed)
    codec._frame_pos = 0
    points = []
    for e in ebn0_list:
        if reseed_each_point:
            codec.synth_seed(seed)
            codec._frame_pos = 0
        pt = ber_point(codec, float(e), max_frames, min_block_errors, batch)
        points.append(pt)
        if log:
            log(f"Eb/N0 {e:.2f} dB: frames {pt.frames}, BER {pt.ber[-1]:.3e}, BLER {pt.bler[-1]:.3e}")
    return points


def write_result_txt(path: str, points, K: int, ebn0_start: float, ebn0_step: float, ebn0_end: float,
                     modulation: int = 1):
    """Append a block in main.cpp's result.txt format (main.cpp:80-99, 264-315)."""
    n = stream_length(K)
    rate = K / (n // modulation)   # main.cpp:47: source_length / SYMBOL_NUM
    with open(path, "a") as fp:
        fp.write(f"\nMODULATION = {modulation}")
        fp.write(f"\nsource_length = {K}")
        fp.write(f"\nrate_coding = {rate:f}")
        fp.write(f"\nSNR_begin={ebn0_start:f}")
        fp.write(f"\nSNR_step={ebn0_step:f}")
        fp.write("N_ITERATION=1 ")
        fp.write(f"\nSNR_end={ebn0_end:f}")
        factor = 10 * math.log(rate * modulation) / math.log(10)
        fp.write("\nEs/N0:\n")
        for i in range(len(points)):
            fp.write(f"{(ebn0_start + ebn0_step * i) + factor:f} ")
        fp.write("\nBer:\n")
        iters = len(points[0].bit_errors) if points else 0
        for it in range(iters):
            for p in points:
                fp.write(f" {p.ber[it]:.10f} ")
            fp.write("\n")
        fp.write("\nBler:\n")
        for it in range(iters):
            for p in points:
                fp.write(f"{p.bler[it]:.10f} ")
            fp.write("\n")
        fp.write("\nthroughput:\n")
        for p in points:   # main.cpp:309-312 indexes err_block_rate[i1] (iteration 0 of point 0..)
            fp.write(f"{(1 - p.bler[0]) * rate * modulation:.10f} ")
        fp.write("----------------------------------------------------------")


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--K", type=int, default=6144)
    ap.add_argument("--f1", type=int, default=263)
    ap.add_argument("--f2", type=int, default=480)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--ebn0", type=float, nargs=3, default=[0.0, 1.0, 0.1], metavar=("START", "END", "STEP"))
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-frames", type=int, default=100000)
    ap.add_argument("--min-block-errors", type=int, default=50, help="<= 0: decode max-frames per point")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--algo", default="logmap", choices=["logmap", "maxlog"])
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"])
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--modulation", type=int, default=1, choices=[1, 2, 3, 4, 6],
                    help="MODULATION of the frames (bits per symbol, modanddem.cpp)")
    ap.add_argument("--window", type=int, default=0, help="sub-block length (0 = exact schedule)")
    ap.add_argument("--overlap", type=int, default=0)
    ap.add_argument("--nii", action="store_true")
    ap.add_argument("--concurrent", action="store_true")
    ap.add_argument("--ext-scale", type=float, default=1.0)
    ap.add_argument("--reference-gpu", type=int, default=0, metavar="P",
                    help="the reference GPU decoder with P sub-blocks (turboDecoderBianJieZhi.cu): "
                         "Max-Log-MAP fp32, window K/P, NII, concurrent SISOs, extrinsic x0.77")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    start, end, step = a.ebn0
    pts, e = [], start
    while e <= end:   # main.cpp:172 accumulates the Eb/N0 (and so its sigma) exactly this way
        pts.append(e)
        e += step
    if a.reference_gpu:
        a.algo, a.precision = "maxlog", "f32"
        a.window, a.overlap, a.nii, a.concurrent, a.ext_scale = a.K // a.reference_gpu, 0, True, True, 0.77
    with TurboCodec(a.K, a.f1, a.f2, iterations=a.iters, algo=a.algo, precision=a.precision, device=a.device) as c:
        c.synth_modulation(a.modulation)
        if a.window:
            c.set_window(a.window, a.overlap, a.ext_scale, nii=a.nii, concurrent=a.concurrent)
        res = ber_sweep(c, pts, a.seed, a.max_frames, a.min_block_errors, a.batch,
                        log=lambda s: print(s, file=sys.stderr, flush=True))
    for p in res:
        print(f"{p.ebn0_db:.2f} frames {p.frames} " +
              " ".join(f"{be}:{bl}" for be, bl in zip(p.bit_errors, p.block_errors)))
    if a.out:
        write_result_txt(a.out, res, a.K, start, step, end, modulation=a.modulation)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
