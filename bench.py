#!/usr/bin/env python3
"""Benchmark of the MI355X turbo decoder -- BASELINE.json metric:
    decoded info Mbit/s @ K=6144, 8 iter, Eb/N0=1.0 dB; BER match vs CPU log_map

Workload at N=1 = BASELINE config 2: batch 4096 x K=6144, 8 log-MAP (table max*) iterations,
rate 1/3, fp64 parity arithmetic (the reference's precision and operation order).
N>1 = BASELINE config 4: one process per GPU (torchrun), 32768 codewords per GPU (N=8: the
262144-codeword batch; weak scaling), or with --strong the 262144 codewords split over the N
ranks.  The global batch is ONE stream of frames, keyed by global codeword index: codeword j is
frame j of ITTC/main.cpp's srand(seed) frame stream (td_synth_frames, bit-identical to the
reference's frames), and rank r decodes its contiguous slice (shard_layout) -- so the ranks'
bits concatenated are the single-process decode of the same global batch.  No data-path
collective; the only exchange is the max of the step times and the sum of the error counters
(gloo, host scalars).  A "step" = one td_decode_device call on the resident batch (demultiplex +
all iterations + hard decisions).

Extra objects on the JSON line:
  roofline      the turbo kernel against HBM (algorithmic bytes: fp64 LLR in + uint8 bits out
                per codeword) with durations from hipEvents inside the timed region;
                `traffic` from the committed rocprofv3 PMC profile of the same config (or null)
  cpu_baseline  the compiled reference (oracle/_ref/ref_harness: ITTC/log_map.cpp's SISO and loop) on the
                host cores, rank 0, N=1; the C restatement (oracle/) where that binary is absent
  dropin        what the unchanged ITTC/main.cpp caller gets: TurboDecoding one frame per call through
                libturbo_logmap_compat.so (examples/dropin_latency.cpp, 15 iterations = N_ITERATION),
                next to the compiled reference's own per-frame time on one host core
  variants      fp32 log-MAP, fp64/fp32 Max-Log-MAP on the same batch; BASELINE config 5 (sliding
                window 64, overlap 30) at its own batch of 32768 (fewer steps)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "decoded info Mbit/s @ K=6144, 8 iter, Eb/N0=1.0 dB; BER match vs CPU log_map"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_MEASURED_GBS = 6290.0    # MI355X_MICROARCH.md: 6.29 TB/s measured streaming (float4 copy)
SEED = 20261015              # srand() seed of the bench's frame stream
CONFIG4_GLOBAL = 262144      # BASELINE config 4: 262144 codewords over 8 GPUs
CONFIG4_PER_GPU = 32768
CONFIG5_BATCH = 32768        # BASELINE config 5: sliding window 64, batch 32768
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (half the FP32 vector rate, 157.3 TF)
F1, F2 = 263, 480             # QPP for K=6144 (ITTC/main.cpp:36-37)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=0,
                    help="codewords per GPU (0: 4096 = config 2 at N=1, 32768 = config 4 per GPU at N>1)")
    ap.add_argument("--strong", action="store_true",
                    help="config 4 strong scaling: --global-batch codewords split over the N ranks")
    ap.add_argument("--global-batch", type=int, default=CONFIG4_GLOBAL, help="total codewords with --strong")
    ap.add_argument("--dump-bits", default="", help="directory: each rank writes its decoded slice (tests)")
    ap.add_argument("--K", type=int, default=6144)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--ebn0", type=float, default=1.0)
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"])
    ap.add_argument("--algo", default="logmap", choices=["logmap", "maxlog"])
    ap.add_argument("--cpu-sample", type=int, default=4096, help="codewords for the CPU baseline (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the CPUs this process may use (affinity), within the box's CPU share")
    ap.add_argument("--window", type=int, default=0, help="0 = exact schedule; 64 = sliding window (config 5)")
    ap.add_argument("--overlap", type=int, default=30, help="sliding-window warm-up steps")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--no-power", action="store_true",
                    help="no amdsmi sampling thread in the timed region (A/B of its cost: DESIGN.md 5)")
    ap.add_argument("--dropin-frames", type=int, default=8,
                    help="frames for the drop-in per-frame latency (0 = skip; N=1, fp64 log-MAP only)")
    return ap.parse_args(argv)


def shard_layout(world: int, rank: int, batch: int, strong: bool, global_batch: int):
    """(first global codeword, codewords) of rank `rank`.  Weak: `batch` per rank, rank r takes
    codewords [r*batch, (r+1)*batch).  Strong: global_batch split into contiguous slices, the first
    global_batch % world ranks one codeword more.  Codeword j is frame j of the srand(SEED) stream."""
    if strong:
        q, r = divmod(global_batch, world)
        n = q + (1 if rank < r else 0)
        return rank * q + min(rank, r), n
    return rank * batch, batch


def per_gpu_batch(a, world: int) -> int:
    if a.batch:
        return a.batch
    return CONFIG4_PER_GPU if world > 1 else 4096


def qpp_for(K):
    if K == 6144:
        return F1, F2
    if K == 1024:
        return 31, 64
    if K == 40:
        return 3, 10
    raise SystemExit("bench: give K in {40, 1024, 6144}")


def window_steps() -> int:
    """Steps per window of the loaded library's exact-schedule kernel (td_window_steps)."""
    from turbo_decoder_cuda_amd import _native as N
    L = N.lib()
    return int(L.td_window_steps()) if hasattr(L, "td_window_steps") else 15   # older A/B builds: 15


def load_traffic(cfg_key):
    """HBM bytes per turbo-kernel launch from profiles/traffic.json (rocprofv3 PMC, committed)."""
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f).get(cfg_key)
        return int(rec["bytes_per_launch"]) if rec else None
    except (OSError, ValueError, KeyError, TypeError):
        return None


def load_traffic_rec(cfg_key):
    """The whole profiles/traffic.json record of a configuration (None if absent)."""
    try:
        with open(os.path.join(REPO, "profiles", "traffic.json")) as f:
            return json.load(f).get(cfg_key)
    except (OSError, ValueError):
        return None


N_SIMDS = 1024   # 256 CUs x 4 SIMDs (MI355X)
# The VALU issue fraction the windowed kernels' own arithmetic reaches with no memory traffic at their
# occupancy (two waves per SIMD): scripts/ubench_window.hip, beta-position mix (alpha recompute + beta
# step + LLR folds), profiles/r05/ubench_window.jsonl (0.754; the alpha mix 0.762; three waves 0.809).
WINDOW_ISSUE_CEILING = 0.754


def window_roofline(K, B, iters, decode_ms, sclk_ghz=None, sclk_source=None, exact_table=False):
    """Roofline record of the windowed schedule (BASELINE config 5: fp64 log-MAP, window 64, overlap 30)
    from the live decode time and the committed PMC of the same kernels (profiles/traffic.json key
    K6144_B32768_it8_f64_logmap_w64g30: FETCH_SIZE x2 + WRITE_SIZE bytes and SQ_INSTS_VALU per decode,
    scripts/gpu_window_pmc.sh).  Two bounds: VALU issue (a wave64 fp64 VALU instruction occupies its SIMD
    4 cycles; 1024 SIMDs at the shader clock) and HBM (counter bytes against the 8 TB/s spec and the
    6.29 TB/s streaming ceiling).  The algorithmic-bytes fraction is the metric's contract, as for
    the exact kernel."""
    rec = load_traffic_rec(f"K{K}_B{B}_it{iters}_f64_logmap_w64g30" + ("_exacttable" if exact_table else ""))
    clk = sclk_ghz or SCLK_GHZ
    alg = B * (8 * (3 * K + 12) + K)
    out = {"kernels": "sw_demux_kernel + (sw_alpha_kernel + sw_beta_kernel) x 2 SISOs x iterations + bits_transpose",
           "decode_ms": round(decode_ms, 4), "alg_bytes_per_decode": alg,
           "achieved": round(alg / (decode_ms * 1e-3) / 1e9, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(alg / (decode_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6)}
    if rec:
        tb = float(rec["bytes_per_decode"])
        vi = float(rec["valu_instr_per_decode"])
        cap = N_SIMDS * clk * 1e9 / 4.0 * decode_ms * 1e-3   # wave-instructions the SIMDs could issue
        out.update({"traffic": int(tb), "traffic_gbs": round(tb / (decode_ms * 1e-3) / 1e9, 1),
                    "traffic_frac": round(tb / (decode_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "traffic_frac_measured_ceiling": round(tb / (decode_ms * 1e-3) / 1e9 / HBM_MEASURED_GBS, 4),
                    "valu_instr_per_decode": int(vi), "valu_issue_frac": round(vi / cap, 4),
                    # the two resource floors of the decode at this clock: all VALU issue slots busy, or the
                    # counter bytes at the measured streaming ceiling; the kernels overlap the two (two
                    # streams), so the larger floor binds and frac_of_binding = floor / decode time
                    "valu_floor_ms": round(vi * 4.0 / N_SIMDS / (clk * 1e9) * 1e3, 3),
                    "hbm_floor_ms": round(tb / (HBM_MEASURED_GBS * 1e9) * 1e3, 3),
                    "sclk_ghz": round(clk, 4), "sclk_source": (sclk_source or "measured (td_clock_read: one beta workgroup)") if sclk_ghz else "constant",
                    "pmc_source": rec.get("source"), "kernel": rec.get("kernel")})
        floor = max(out["valu_floor_ms"], out["hbm_floor_ms"])
        out.update({"binding": "valu" if out["valu_floor_ms"] >= out["hbm_floor_ms"] else "hbm",
                    "frac_of_binding": round(floor / decode_ms, 4),
                    "lane_valu_per_position": round(vi * 64 / (B * 2 * iters * (K + 3)), 1)})
        if exact_table:   # the issue rate the exact-table mix reaches in the microbenchmark (a measured ceiling)
            out.update({"valu_issue_ceiling": WINDOW_ISSUE_CEILING,
                        "valu_issue_ceiling_source": "scripts/ubench_window.hip, 2 waves/SIMD (profiles/r05/ubench_window.jsonl)",
                        "frac_of_issue_ceiling": round(out["valu_issue_frac"] / WINDOW_ISSUE_CEILING, 4)})
    return out


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    from turbo_decoder_cuda_amd import TurboCodec

    if world > 1:
        dist.init_process_group(backend="gloo")
    # one GPU per rank; more ranks than GPUs (a rehearsal on a smaller box) share them round-robin
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    f1, f2 = qpp_for(a.K)
    first, a.batch = shard_layout(world, rank, per_gpu_batch(a, world), a.strong, a.global_batch)
    a.total = a.global_batch if a.strong else a.batch * world
    if a.batch < 1:
        raise SystemExit(f"bench: rank {rank} has no codewords (--global-batch {a.global_batch} < {world} ranks)")

    codec = TurboCodec(a.K, f1, f2, iterations=a.iters, algo=a.algo, precision=a.precision, device=local)
    # this rank's slice of the global frame stream: frames [first, first + batch) of srand(SEED)
    codec.synth_seed(SEED)
    codec.synth_seek(first)
    u_d, llr64 = codec.synth(a.batch, a.ebn0)
    llr = llr64 if a.precision == "f64" else llr64.float()
    if a.window:
        codec.set_window(a.window, a.overlap)
    codec.reserve(a.batch)   # also picks the workspace placement (td_reserve)
    placement = codec.placement()
    placement_cost = codec.placement_cost() + (codec.workspace_bytes(),)
    bits = torch.empty((a.batch, a.K), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        codec.decode(llr, bits, stream=stream)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)

    power = PowerSampler(local) if rank == 0 and not a.no_power else None
    codec.profile(True)   # hipEvents around each kernel, inside the timed region
    if power is not None:
        power.start()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        codec.decode(llr, bits, stream=stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    power_rec = power.stop() if power is not None else None
    barrier()
    demux_ms, turbo_ms, nlaunch = codec.kernel_ms()
    codec.profile(False)
    clock = None
    # the last launch's sustained shader clock (td_clock_read; windowed: one beta workgroup), outside the timed region
    try:
        clock = codec.clock()
    except Exception:
        clock = None

    errs = int((bits != u_d).sum().item())
    blk = int((bits != u_d).any(dim=1).sum().item())
    if a.dump_bits:
        os.makedirs(a.dump_bits, exist_ok=True)
        np.save(os.path.join(a.dump_bits, f"bits_rank{rank}_first{first}.npy"), bits.cpu().numpy())
    elapsed, errs, blk = reduce_over_ranks(t1 - t0, errs, blk, world)
    out = summarize(a, world, elapsed, errs, blk, demux_ms, turbo_ms, nlaunch, f1, f2, clock)
    out["workspace_placement"] = placement_record(placement, turbo_ms, a.iters, placement_cost)
    if power_rec and power_rec.get("socket_w_mean") and out["value"] > 0:
        # board energy per decoded info bit over the timed region (socket power / throughput of this GPU)
        power_rec["nj_per_info_bit"] = round(power_rec["socket_w_mean"] / (out["value"] / world) * 1e3, 2)
    out["power"] = power_rec

    if rank == 0 and world == 1 and not a.no_variants:
        out["pcie_inclusive"] = pcie_inclusive(a, codec, llr, dev, stream)
    if rank == 0 and world == 1 and a.cpu_sample > 0:
        n = min(a.cpu_sample, a.batch)
        out["cpu_baseline"] = cpu_baseline(a, llr64[:n].cpu().numpy(), bits[:n].cpu().numpy(), f1, f2)
    if rank == 0 and world == 1 and a.dropin_frames > 0 and not a.window and a.precision == "f64" and a.algo == "logmap":
        out["dropin"] = dropin(a, llr64[: a.dropin_frames].cpu().numpy(), f1, f2, local,
                               info=u_d[: a.dropin_frames].cpu().numpy())
    if rank == 0 and world == 1 and not a.no_variants:
        out["variants"] = variants(a, codec, llr64, u_d, f1, f2, dev, stream)
        out["demod"] = demod_rates(a, dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


class PowerSampler:
    """Board power and shader clock of this rank's GPU (amdsmi), sampled every ~10 ms from a host
    thread while the timed region runs.  The config-2 launch sits at the board's power limit
    (1360-1378 W at 2.27-2.30 GHz), so the record says which cap a box's clock met.
    Monitoring only: any amdsmi failure leaves the record null and the bench unchanged."""

    def __init__(self, device: int):
        self.h, self.samples, self.limit, self.smi = None, [], None, None
        try:
            import amdsmi
            import torch
            amdsmi.amdsmi_init()
            self.smi = amdsmi   # initialised: shut down in stop() / close() on every path
            hs = amdsmi.amdsmi_get_processor_handles()
            prop = torch.cuda.get_device_properties(device)
            bus = getattr(prop, "pci_bus_id", None)
            for h in hs:   # the torch device's PCI bus; a single visible GPU otherwise
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)
                if bus is not None and int(bdf.split(":")[1], 16) == int(bus):
                    self.h = h
            if self.h is None and len(hs) == 1:
                self.h = hs[0]
            if self.h is not None:
                lim = amdsmi.amdsmi_get_power_info(self.h).get("power_limit")
                # amdsmi reports the limit in microwatts (1400000000 on MI355X), the socket power in W
                self.limit = (lim / 1e6 if lim > 1e5 else lim) if isinstance(lim, (int, float)) else None
        except Exception:
            self.h = None
        if self.h is None:
            self.close()

    def close(self):
        """amdsmi_shut_down once, whenever amdsmi_init succeeded."""
        if self.smi is not None:
            try:
                self.smi.amdsmi_shut_down()
            except Exception:
                pass
            self.smi = None

    def _read(self):
        p = self.smi.amdsmi_get_power_info(self.h).get("current_socket_power")
        c = self.smi.amdsmi_get_clock_info(self.h, self.smi.AmdSmiClkType.SYS).get("clk")
        return (float(p) if isinstance(p, (int, float)) else None, float(c) if isinstance(c, (int, float)) else None)

    def start(self):
        import threading
        self._stop = threading.Event()

        def loop():
            while not self._stop.is_set():
                try:
                    self.samples.append(self._read())
                except Exception:
                    return
                self._stop.wait(0.01)
        if self.h is not None:
            self._t = threading.Thread(target=loop, daemon=True)
            self._t.start()
        return self

    def stop(self):
        try:
            if self.h is None:
                return None
            self._stop.set()
            self._t.join(timeout=2.0)
        finally:
            self.close()
        pw = [p for p, _ in self.samples if p is not None]
        ck = [c for _, c in self.samples if c is not None]
        if not pw:
            return None
        return {"socket_w_mean": round(sum(pw) / len(pw), 1), "socket_w_max": max(pw),
                "sclk_mhz_mean": round(sum(ck) / len(ck), 1) if ck else None, "samples": len(pw),
                "power_limit_w": self.limit, "source": "amdsmi current_socket_power / SYS clock, ~10 ms apart, timed region",
                "note": "the launch is board-power-capped (DESIGN.md 5): the clock a box reaches at this limit sets its speed"}


def placement_record(placement, turbo_ms: float, iters: int, cost=None) -> dict:
    """td_reserve's workspace placement search beside the full launch it chose for: the kept
    candidate's one-iteration probe time x iterations is what the probe predicts for a launch, so a
    'fast probe, slow launch' box shows as launch_over_probe well above 1."""
    ms, kept = placement
    rec = {"probe_ms": ms, "kept": kept,
           "note": "one-iteration probe per candidate workspace at td_reserve (outside the timed region)"}
    if cost and cost[0] is not None and ms:
        rec["search_wall_ms"] = round(cost[0], 1)
        rec["search_peak_gib_held"] = round(cost[1] / 2**30, 2)
        if len(cost) > 2 and cost[2]:
            rec["workspace_gib"] = round(cost[2] / 2**30, 3)
            rec["peak_held_over_workspace"] = round(cost[1] / cost[2], 3)
    if ms and 0 <= kept < len(ms):
        rec["kept_probe_ms"] = ms[kept]
        rec["probe_x_iters_ms"] = round(ms[kept] * iters, 4)
        rec["launch_ms"] = round(turbo_ms, 4)
        rec["launch_over_probe"] = round(turbo_ms / (ms[kept] * iters), 4) if ms[kept] > 0 else None
    return rec


DROPIN = os.path.join(REPO, "turbo_decoder_cuda_amd", "td_dropin_latency")


DROPIN_WINDOW = {"TD_WINDOW": "64", "TD_OVERLAP": "30"}   # the opt-in low-latency schedule (config 5's)


def dropin(a, flows, f1, f2, device: int, info=None) -> dict:
    """The unchanged reference caller's per-frame latency (ITTC/main.cpp:221: one TurboDecoding per
    frame, 15 iterations = N_ITERATION): examples/dropin_latency.cpp linked against
    libturbo_logmap_compat.so, a child process on this GPU, warm handle after its first frame.  Beside
    it the compiled reference's TurboDecoding loop on one host core at 15 iterations, per frame.
    Bits: the drop-in's last-iteration rows against the reference's on the same frames.
    `window`: the same caller with the compat layer's opt-in sub-block schedule (TD_WINDOW=64,
    TD_OVERLAP=30, read at TurboCodingInit): its per-frame time and its bits against the exact
    schedule's and the source bits (BER-gated, not bit-exact)."""
    import subprocess
    import tempfile

    n = flows.shape[0]
    rec = {"frames": n, "iterations": 15, "K": a.K, "caller": "ITTC/main.cpp:221 TurboDecoding(flow, out, 3K+12)"}
    if not os.access(DROPIN, os.X_OK):
        rec["error"] = "td_dropin_latency not built"
        return rec
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "flows.bin"), os.path.join(td, "bits.bin")
        np.ascontiguousarray(flows, dtype=np.float64).tofile(fin)

        def run(extra):
            env = dict(os.environ, TD_ITERATIONS="15", TD_DEVICE=str(device), **extra)
            for k in DROPIN_WINDOW:
                if k not in extra:
                    env.pop(k, None)
            r = subprocess.run([DROPIN, str(a.K), str(f1), str(f2), str(n), fin, fout], capture_output=True,
                               text=True, env=env, timeout=300)
            if r.returncode:
                return None, (r.stdout + r.stderr)[-400:]
            return (json.loads(r.stdout.strip().splitlines()[-1]),
                    np.fromfile(fout, dtype=np.uint8).reshape(n, a.K)), None

        res, err = run({})
        if err:
            rec["error"] = err
            return rec
        rec.update(res[0])
        gpu_bits = res[1]
        wres, werr = run(DROPIN_WINDOW)
        if werr:
            rec["window"] = {"error": werr}
        else:
            w = {"env": dict(DROPIN_WINDOW), "ms_per_frame": wres[0]["ms_per_frame"], "ms_first": wres[0]["ms_first"],
                 "ms_min": wres[0]["ms_min"], "speedup_vs_exact": round(rec["ms_per_frame"] / wres[0]["ms_per_frame"], 3),
                 "bits_differing_from_exact": int((wres[1] != gpu_bits).sum())}
            if info is not None:
                w["bit_errors"] = int((wres[1] != info).sum())
                rec["bit_errors"] = int((gpu_bits != info).sum())
            rec["window"] = w
        if os.access(REF_HARNESS, os.X_OK):
            nr = min(n, 4)
            rout = os.path.join(td, "rbits.bin")
            np.ascontiguousarray(flows[:nr], dtype=np.float64).tofile(fin)
            rr = subprocess.run([REF_HARNESS, "decode", str(a.K), str(f1), str(f2), "15", "1", fin, rout],
                                capture_output=True, text=True, check=True, timeout=600)
            dt = float(rr.stdout.split()[1])
            ref_bits = np.fromfile(rout, dtype=np.uint8).reshape(nr, a.K)
            rec["reference_ms_per_frame"] = round(dt / nr * 1e3, 3)
            rec["reference"] = f"the compiled reference (ITTC/log_map.cpp, g++ -O2), one host core, {nr} frames"
            rec["bits_match_reference"] = bool(np.array_equal(gpu_bits[:nr], ref_bits))
            rec["speedup_vs_reference"] = round(rec["reference_ms_per_frame"] / rec["ms_per_frame"], 3)
            if isinstance(rec.get("window"), dict) and "ms_per_frame" in rec["window"]:
                rec["window"]["speedup_vs_reference"] = round(rec["reference_ms_per_frame"] / rec["window"]["ms_per_frame"], 3)
    rec["note"] = ("per-frame latency of the batch-of-one path: one codeword group on one CU, so the time is "
                   "the serial alpha / beta chains of 30 SISOs (DESIGN.md 5); throughput callers batch "
                   "(td_decode_device), the headline value; `window` is the opt-in sub-block schedule")
    return rec


def reduce_over_ranks(elapsed: float, errs: int, blk: int, world: int):
    """Max of the timed-region wall time and sum of the error counters over ranks (gloo, host
    scalars: the only cross-rank exchange; the decode itself has no collective)."""
    if world <= 1:
        return elapsed, errs, blk
    import torch
    import torch.distributed as dist

    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    e = torch.tensor([errs, blk], dtype=torch.int64)
    dist.all_reduce(e, op=dist.ReduceOp.SUM)
    return float(t.item()), int(e[0]), int(e[1])


def traffic_model(K: int, B: int, iters: int, esz: int, algo: str, W: int = 15, alpha_raw: bool = True) -> dict:
    """HBM bytes per turbo-kernel launch by stream, from the exact schedule's access pattern
    (groups G = ceil(B/8), L = K+3, windows of W steps (td_window_steps()),
    nT = ceil(L/W), 2*iters SISOs):
      alpha     log-MAP: the F pass writes alpha_raw, one 64-element row per step and row L; the B
                pass DMAs whole W-row windows back, plus the first DMA of the window after the last
                (log_map.cpp:975-1001 alpha, kept for the LLRs; beta's tempmax is the max of the rows).
                Max-Log-MAP: one row in three written, W/3 rows a window read back
      tempmax   Max-Log-MAP only: one 8-element row per step written, whole windows read back (beta's
                :1019 input); log-MAP forms it from the alpha rows on chip (round 4)
      inputs    ys, yp, La tiles (+ the window's write positions) staged once in the F pass, again in
                the B pass
      extrinsic Le written once per SISO (8 B per element, coalesced over a group's 8 codewords)
      sys2      the first SISO forms decoder 2's systematic input (a gather within L2, one write)
    alpha_raw=False models the round-3 (v29) log-MAP kernel: normalised alpha of L rows and the tempmax
    stream.  The sum is checked against the PMC total (FETCH_SIZE x2 + WRITE_SIZE) in profiles/traffic.json."""
    G = (B + 7) // 8
    L = K + 3
    nT = (L + W - 1) // W
    S = 2 * iters
    row = 64 * esz
    if algo == "logmap" and alpha_raw:
        alpha = S * G * ((L + 1) * row + nT * W * row + 1024)
        tm = 0
    elif algo == "logmap":
        alpha = S * G * (L + nT * W) * row
        tm = S * G * (L + nT * W) * 8 * esz
    else:
        alpha = S * G * ((L + 2) // 3 + nT * (W // 3)) * row
        tm = S * G * (L + nT * W) * 8 * esz
    wp_chunks = W // 4 if W % 4 == 0 else (W + 6) // 4   # td_kernels.hip kWpChunks
    tile = 3 * W * 8 * esz + 2 * wp_chunks * 16   # ys, yp, La rows + the window's write positions
    inputs = S * G * 2 * nT * tile
    ext = S * G * K * 8 * esz
    sys2 = G * K * 8 * esz * 2
    bits = B * K
    parts = {"alpha": alpha, "tempmax": tm, "inputs": inputs, "extrinsic": ext, "sys2": sys2, "bits": bits}
    total = sum(parts.values())
    return {"bytes": parts, "total": total, "share": {k: round(v / total, 4) for k, v in parts.items()},
            "scratch_share": round((alpha + tm) / total, 4), "window_steps": W}


# Dependent-chain cycles per trellis step of the two recursions (fp64 log-MAP):
#   isolated   each alone on a SIMD with its operands in registers (scripts/ubench_alpha.hip,
#              scripts/ubench_beta.hip): alpha 218 with its two scratch stores (committed order), beta 148;
#   in_kernel  the chains' own loops inside the production schedule, from the stamps build
#              (profiles/r04/stamps_v31_aspec.txt, slot 4 of waves A and B): alpha 182 (the speculative
#              table-row read of round 4, stores in its shadow), beta 153 (its LDS reads beside the folds).
# The floor is priced at the in-kernel figures (the isolated alpha overstated the
# fraction); the isolated floor rides along.
CHAIN_CYCLES_F64_LOGMAP = {"alpha": 182, "beta": 153}
CHAIN_CYCLES_F64_LOGMAP_ISOLATED = {"alpha": 218, "beta": 148}
SCLK_GHZ = 2.35   # fallback only: the sustained shader clock measured on earlier boxes


def latency_floor(a, turbo_ms, sclk_ghz=None):
    """The exact schedule's own speed of light: every codeword of a dispatch round is in flight at
    once, so a launch cannot beat 2*iters SISOs x L steps x (alpha step + beta step), the two serial
    recursions back to back, at the chains' in-kernel per-step latency, at the launch's own measured
    shader clock (td_clock_read).  frac = floor / measured.  The rest of the launch is the schedule's
    overhead around the chains (window starts, barrier waits, SISO prologues: DESIGN.md 8.5)."""
    if a.window or a.algo != "logmap" or a.precision != "f64" or turbo_ms <= 0:
        return None
    clk = sclk_ghz if sclk_ghz else SCLK_GHZ
    rounds = -(-((a.batch + 7) // 8) // 512)   # dispatch rounds of 512 workgroups (2 per CU)

    def floor(c):
        return rounds * 2 * a.iters * (a.K + 3) * (c["alpha"] + c["beta"]) / (clk * 1e9) * 1e3

    floor_ms, iso_ms = floor(CHAIN_CYCLES_F64_LOGMAP), floor(CHAIN_CYCLES_F64_LOGMAP_ISOLATED)
    per_step = turbo_ms * 1e-3 * clk * 1e9 / (rounds * 2 * a.iters * (a.K + 3))
    return {"floor_ms": round(floor_ms, 3), "frac": round(floor_ms / turbo_ms, 4),
            "chain_cycles_per_step": CHAIN_CYCLES_F64_LOGMAP, "chain_source": "in-kernel (stamps build)",
            "isolated": {"chain_cycles_per_step": CHAIN_CYCLES_F64_LOGMAP_ISOLATED, "floor_ms": round(iso_ms, 3),
                         "frac": round(iso_ms / turbo_ms, 4)},
            "launch_cycles_per_step": round(per_step, 1),
            "overhead_cycles_per_step": round(per_step - sum(CHAIN_CYCLES_F64_LOGMAP.values()), 1),
            "sclk_ghz": round(clk, 4),
            "sclk_source": "measured (td_clock_read)" if sclk_ghz else "constant (no clock sample)",
            "dispatch_rounds": rounds,
            "note": "serial alpha + beta chains at their in-kernel per-step latency, the bound this "
                    "latency-limited kernel is measured against; the overhead is itemised in DESIGN.md 8.5; "
                    "the HBM fraction above is the metric's contract"}


def summarize(a, world, elapsed, errs, blk, demux_ms, turbo_ms, nlaunch, f1, f2, clock=None) -> dict:
    """The bench JSON record.  value = info bits decoded by ALL ranks / max-over-ranks time."""
    ms_step = elapsed / a.steps * 1e3
    total = getattr(a, "total", a.batch * world)   # codewords of all ranks per step
    total_bits = total * a.K * a.steps
    value = total_bits / elapsed / 1e6
    esz = 8 if a.precision == "f64" else 4
    bytes_cw = esz * (3 * a.K + 12) + a.K   # algorithmic: LLR in + uint8 bits out
    alg_bytes = bytes_cw * a.batch
    achieved = alg_bytes / (turbo_ms * 1e-3) / 1e9 if turbo_ms > 0 else 0.0
    cfg_key = f"K{a.K}_B{a.batch}_it{a.iters}_{a.precision}_{a.algo}" + (f"_w{a.window}g{a.overlap}" if a.window else "")
    traffic = load_traffic(cfg_key)
    model = None if a.window else traffic_model(a.K, a.batch, a.iters, esz, a.algo, window_steps())
    sclk = clock[0] if clock else None
    # measured HBM bytes (PMC) per launch over the live kernel time: what the memory system
    # actually moves (the exact kernel streams alpha / tempmax through HBM by design)
    traffic_gbs = traffic / (turbo_ms * 1e-3) / 1e9 if (traffic and turbo_ms > 0) else None
    # fp64 VALU work of the exact schedule (~133 ops per trellis step and SISO,
    # max* counted as one op) over the live kernel time
    valu_tops = a.batch * (a.K + 3) * 2 * a.iters * 133 / (turbo_ms * 1e-3) / 1e12 if turbo_ms > 0 else 0.0
    if a.window:
        cfg_no = "5"
    elif world > 1 or a.batch > 4096 or a.strong:
        cfg_no = "4"
    else:
        cfg_no = "2" if a.algo == "logmap" else "3"
    if cfg_no == "4":
        workload = (f"BASELINE config 4: {total} x K={a.K} over {world} GPU(s), "
                    + (f"strong scaling ({a.batch} on rank 0)" if a.strong else f"{a.batch} per GPU, weak scaling")
                    + f", {a.iters} iterations, {'log-MAP table max*' if a.algo == 'logmap' else 'Max-Log-MAP'}, "
                    f"{a.precision}, Eb/N0={a.ebn0} dB")
    else:
        workload = (f"BASELINE config {cfg_no}: batch {a.batch} x K={a.K} per GPU, "
                    f"{a.iters} iterations, {'log-MAP table max*' if a.algo == 'logmap' else 'Max-Log-MAP'}, "
                    f"{a.precision} {'parity (reference op order)' if a.precision == 'f64' else 'throughput'}, "
                    f"Eb/N0={a.ebn0} dB" + (f", sliding window {a.window} with overlap {a.overlap}" if a.window else ""))
    return {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mbit/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if a.strong else "weak",
        "vs_baseline": None,
        "dtype": a.precision,
        "data": (f"synthetic: ITTC/main.cpp's frames of srand({SEED}) (rand() % 2 info bits, RSC 13/15 + QPP "
                 "turbo encoder, BPSK, mgrns AWGN, LLR = 2y/sigma^2) generated on the GPU by td_synth_frames, "
                 "bit-identical to the reference's; global codeword j = frame j, each rank decodes its slice"),
        "config": {
            "workload": workload,
            "K": a.K, "f1": f1, "f2": f2, "batch_per_gpu": a.batch, "global_batch": total,
            "iterations": a.iters, "algo": a.algo, "precision": a.precision, "ebn0_db": a.ebn0,
            "window": a.window, "overlap": a.overlap if a.window else None,
            "parallelism": f"batch-shard x{world} (no collective on the data path)",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "sw_alpha_kernel + sw_beta_kernel" if a.window else "turbo_decode_kernel",
            "achieved": round(achieved, 3),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6),
            "traffic": traffic,
            "traffic_gbs": round(traffic_gbs, 1) if traffic_gbs else None,
            "traffic_frac": round(traffic_gbs / HBM_PEAK_GBS, 4) if traffic_gbs else None,
            "traffic_frac_measured_ceiling": round(traffic_gbs / HBM_MEASURED_GBS, 4) if traffic_gbs else None,
            "measured_ceiling_gbs": HBM_MEASURED_GBS,
            "traffic_model": model,
            "latency_floor": latency_floor(a, turbo_ms, sclk),
            "sclk_ghz": round(sclk, 4) if sclk else None,
            "clock_span_ms": round(clock[1], 4) if clock else None,
            "limiter": ("latency of the serial alpha / beta recursions (one dependent trellis step at a time "
                        "per codeword; DESIGN.md 3.2): neither HBM nor VALU is saturated") if not a.window else
                       "VALU issue and HBM of the sub-block kernels together (DESIGN.md 8.3; `window`)",
            "valu_top_s": round(valu_tops, 3),
            "alg_bytes_per_launch": alg_bytes,
            "alg_bytes_per_codeword": bytes_cw,
            "kernel_ms_avg": round(turbo_ms, 4),
            "demux_ms_avg": round(demux_ms, 4),
            "launches_timed": nlaunch,
            "window": (window_roofline(a.K, a.batch, a.iters, demux_ms + turbo_ms, sclk)
                       if a.window and a.precision == "f64" and a.algo == "logmap" and turbo_ms > 0 else None),
        },
        "ber": {"bit_errors": errs, "block_errors": blk,
                "ber": errs / (world * a.batch * a.K), "bler": blk / (world * a.batch)},
    }


REF_HARNESS = os.path.join(REPO, "oracle", "_ref", "ref_harness")


def cpu_threads(a) -> dict:
    """Threads for the CPU baseline: every CPU this process may run on (sched_getaffinity), within
    the box's CPU share when the harness sets one (OMP_NUM_THREADS: 16 for a one-GPU lease, whose
    affinity can still list the whole machine).  Physical cores are reported beside it."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS", "")
    share = int(share) if share.isdigit() and int(share) > 0 else 0
    threads = a.cpu_threads or (min(avail, share) if share else avail)
    return {"threads": threads, "affinity_cpus": avail, "cpu_share": share or None,
            "physical_cores": _physical_cores()}


def cpu_baseline(a, llr_h, gpu_bits, f1, f2):
    """The reference's CPU path on the host cores, over the first `cpu_sample` codewords of the
    same batch.  fp64 log-MAP: the compiled reference itself (oracle/_ref/ref_harness, built from
    /root/reference/ITTC/log_map.cpp by `make -C oracle ref`; its `decode` mode runs TurboDecoding's
    loop through the reference's functions, frames spread over threads) -- kind "reference".
    Otherwise, or where that binary was not built: the C restatement (oracle/) -- kind "port"."""
    n = llr_h.shape[0]
    ct = cpu_threads(a)
    threads = ct["threads"]
    if a.precision == "f64" and a.algo == "logmap" and os.access(REF_HARNESS, os.X_OK):
        import subprocess
        import tempfile

        with tempfile.TemporaryDirectory() as td:
            fin, fout = os.path.join(td, "flows.bin"), os.path.join(td, "bits.bin")
            np.ascontiguousarray(llr_h, dtype=np.float64).tofile(fin)
            r = subprocess.run([REF_HARNESS, "decode", str(a.K), str(f1), str(f2), str(a.iters), str(threads), fin, fout],
                               capture_output=True, text=True, check=True)
            dt = float(r.stdout.split()[1])
            cb = np.fromfile(fout, dtype=np.uint8).reshape(n, a.K)
        kind, what = "reference", "the compiled reference (ITTC/log_map.cpp, g++ -O2)"
    else:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import pyoracle

        sample = np.ascontiguousarray(llr_h)
        if a.precision == "f32":
            sample = sample.astype(np.float32)
        algo = pyoracle.ALGO_LOGMAP if a.algo == "logmap" else pyoracle.ALGO_MAXLOG
        t0 = time.perf_counter()
        cb = pyoracle.decode_batch(sample, a.K, f1, f2, a.iters, algo, nthreads=threads)
        dt = time.perf_counter() - t0
        kind, what = "port", "the C restatement (oracle/turbo_oracle.c)"
    value = n * a.K / dt / 1e6
    per_core = value / threads
    return {
        "value": round(value, 4),
        "unit": "Mbit/s",
        "cores": threads,
        "kind": kind,
        "sample": f"{n} codewords of the same batch (K={a.K}, {a.iters} iter, {a.precision} {a.algo}) through {what}, "
                  f"one frame per thread, {threads} threads, {dt:.2f} s",
        "bits_match_gpu": bool(np.array_equal(cb, gpu_bits)),
        "cpu_model": _cpu_model(),
        "affinity_cpus": ct["affinity_cpus"],
        "cpu_share": ct["cpu_share"],
        "physical_cores": ct["physical_cores"],
        "per_core": round(per_core, 4),
        "all_physical_cores_extrapolated": (round(per_core * ct["physical_cores"], 3) if ct["physical_cores"] else None),
        "note": "threads = the CPUs this process may use within the box's CPU share (OMP_NUM_THREADS on a one-GPU "
                "lease); frames are independent, so the rate scales with threads (all_physical_cores_extrapolated "
                "= per_core x physical cores, an extrapolation, not a measurement)",
    }


def pcie_inclusive(a, codec, llr, dev, stream):
    """Host-resident flow (not the headline value): pinned H2D of the LLR batch +
    decode + D2H of the bits per batch.
      serial     one stream, batch after batch;
      pipelined  double-buffered: batch n+1's H2D (copy stream) and batch n-1's D2H (second copy
                 stream) under batch n's decode, ordered by events -- what a host-fed caller of
                 td_decode_device reaches with two device buffers."""
    import torch

    h_llr = llr.cpu().pin_memory()
    h_bits = [torch.empty((a.batch, a.K), dtype=torch.uint8).pin_memory() for _ in range(2)]
    d_llr = [llr, torch.empty_like(llr)]
    d_bits = [torch.empty((a.batch, a.K), dtype=torch.uint8, device=dev) for _ in range(2)]
    steps = max(8, a.steps)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        llr.copy_(h_llr, non_blocking=True)
        codec.decode(llr, d_bits[0], stream=stream)
        h_bits[0].copy_(d_bits[0], non_blocking=True)
    torch.cuda.synchronize(dev)
    serial = (time.perf_counter() - t0) / steps

    s_in, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ev_in = [torch.cuda.Event() for _ in range(2)]     # H2D of the buffer done
    ev_dec = [torch.cuda.Event() for _ in range(2)]    # decode of the buffer done
    ev_out = [torch.cuda.Event() for _ in range(2)]    # D2H of the buffer done (buffer free)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for n in range(steps + 1):
        x = n % 2
        if n < steps:   # H2D of batch n, once batch n-2's decode has released the buffer
            if n >= 2:
                s_in.wait_event(ev_dec[x])
            with torch.cuda.stream(s_in):
                d_llr[x].copy_(h_llr, non_blocking=True)
            ev_in[x].record(s_in)
            stream.wait_event(ev_in[x])
            if n >= 2:
                stream.wait_event(ev_out[x])   # batch n-2's bits have left d_bits[x]
            codec.decode(d_llr[x], d_bits[x], stream=stream)
            ev_dec[x].record(stream)
        if n >= 1:      # D2H of batch n-1
            y = (n - 1) % 2
            s_out.wait_event(ev_dec[y])
            with torch.cuda.stream(s_out):
                h_bits[y].copy_(d_bits[y], non_blocking=True)
            ev_out[y].record(s_out)
    torch.cuda.synchronize(dev)
    piped = (time.perf_counter() - t0) / steps
    gb = llr.numel() * llr.element_size() / 1e9
    return {"value": round(a.batch * a.K / piped / 1e6, 3), "unit": "Mbit/s", "ms_per_step": round(piped * 1e3, 4),
            "serial": {"value": round(a.batch * a.K / serial / 1e6, 3), "ms_per_step": round(serial * 1e3, 4)},
            "h2d_gb_per_batch": round(gb, 4),
            "note": "pinned host LLR batch -> HBM, decode, bits -> pinned host, per batch; value: double-buffered "
                    "pipeline (H2D and D2H on copy streams under the decode); serial: one stream"}


def variants(a, codec, llr64, u_d, f1, f2, dev, stream):
    """Other arithmetic modes on the same batch (configs 3, fp32), BASELINE config 5 (sliding
    window 64 with overlap 30) at its own batch of 32768 codewords, and the exact schedule at config
    4's per-GPU shard (32768; fp32 there runs three or four workgroups per CU): frames
    0..32767 of the same srand(SEED) stream, made on the device by the bench's codec."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec

    res = {}
    cases = [(p, g, 0, False) for p, g in (("f64", "logmap"), ("f32", "logmap"), ("f64", "maxlog"), ("f32", "maxlog"))]
    cases += [(p, g, 64, True) for p, g in (("f64", "logmap"), ("f64", "logmap-exact"), ("f32", "logmap"), ("f32", "maxlog"))]
    if a.batch != CONFIG5_BATCH:
        cases += [(p, g, 0, True) for p, g in (("f64", "logmap"), ("f32", "logmap"), ("f32", "maxlog"))]
    big = None
    for prec, algo_form, win, on_big in cases:
        algo, exact_table = algo_form.split("-")[0], algo_form.endswith("-exact")
        if prec == a.precision and algo == a.algo and win == a.window and not on_big:
            continue
        if on_big:
            if big is None:   # config 5's batch, once for the three windowed modes
                B5 = CONFIG5_BATCH
                codec.synth_seek(0)
                big = codec.synth(B5, a.ebn0)
            ub, xb = big
            B = ub.shape[0]
        else:
            ub, xb, B = u_d, llr64, a.batch
        x = xb if prec == "f64" else xb.float()
        c = TurboCodec(a.K, f1, f2, iterations=a.iters, algo=algo, precision=prec, device=dev.index)
        if win:
            c.set_window_maxstar(exact_table)
            c.set_window(win, a.overlap)
        c.reserve(B)
        b = torch.empty((B, a.K), dtype=torch.uint8, device=dev)
        c.decode(x, b, stream=stream)
        torch.cuda.synchronize(dev)
        steps = max(2, a.steps // 2)
        c.profile(True)
        # config 5's roofline prices VALU issue at the clock: the amdsmi mean over the whole timed
        # region, td_clock_read's one-workgroup sample beside it
        pw = PowerSampler(dev.index) if (win and prec == "f64" and algo == "logmap" and not a.no_power) else None
        if pw is not None:
            pw.start()
        t0 = time.perf_counter()
        for _ in range(steps):
            c.decode(x, b, stream=stream)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        prec_pw = pw.stop() if pw is not None else None
        _, kms, _ = c.kernel_ms()
        try:
            vclk = c.clock()[0]
        except Exception:
            vclk = None
        c.close()
        errs = int((b != ub).sum().item())
        del x
        key = f"{prec}_{algo}" + (f"_window{win}_overlap{a.overlap}" if win else (f"_B{B}" if on_big else "")) + \
            ("_exact_table" if exact_table else "")
        cfg = "5" if win else ("4 (one GPU's shard)" if on_big and prec == "f64" and algo == "logmap"
                               else ("3" if algo == "maxlog" and prec == "f64" else None))
        res[key] = {"value": round(B * a.K * steps / dt / 1e6, 3), "unit": "Mbit/s", "batch": B, "config": cfg,
                    "ms_per_step": round(dt / steps * 1e3, 4), "kernel_ms_avg": round(kms, 4), "bit_errors": errs}
        if win and prec == "f64" and algo == "logmap":
            mean_ghz = (prec_pw["sclk_mhz_mean"] / 1e3) if prec_pw and prec_pw.get("sclk_mhz_mean") else None
            res[key]["roofline"] = window_roofline(a.K, B, a.iters, dt / steps * 1e3, mean_ghz or vclk,
                                                   "amdsmi mean over the timed region" if mean_ghz else None,
                                                   exact_table)
            res[key]["maxstar"] = ("log_map.cpp's E_algorithm (exact three-read table)" if exact_table else
                                   "one-read table: E_algorithm's correction at the midpoint of d's bucket, 8 an octave "
                                   "(td_set_window_maxstar; BER curve in DESIGN.md 8.3)")
            res[key]["roofline"]["sclk_td_clock_read_ghz"] = round(vclk, 4) if vclk else None
            res[key]["power"] = prec_pw
    if big is not None and a.K == 6144:
        res["ref_gpu_schedule_P32_10it"] = ref_gpu_schedule(a, big, f1, f2, dev, stream)
        if a.iters == 8 and a.precision == "f64":
            res["window_ber_gate"] = window_ber_gate(a, f1, f2, dev)
    return res


def window_ber_gate(a, f1, f2, dev, frames=32768, points=(0.35, 0.40), seed=100):
    """Config 5's BER gate measured in this run (north_star: "BER-vs-Eb/N0 within 0.05 dB of the CPU
    reference"): the same generator frames at two waterfall points through the exact schedule (bit-exact
    against the reference) and the windowed one (W = 64, overlap 30, the bench's config-5 line), fp64
    log-MAP, 8 iterations; the window's shift in dB read through the exact curve's local slope.  The
    full paired curve is scripts/ber_window_vs_exact.py (profiles/r06/ber_window_vs_exact.json)."""
    import math

    import torch

    from turbo_decoder_cuda_amd import TurboCodec

    t0 = time.perf_counter()
    rec = {"frames_per_point": frames, "window": 64, "overlap": a.overlap, "points": []}
    with TurboCodec(a.K, f1, f2, iterations=a.iters, device=dev.index) as ex, \
            TurboCodec(a.K, f1, f2, iterations=a.iters, device=dev.index) as win:
        win.set_window(64, a.overlap)
        for k, e in enumerate(points):
            ex.synth_seed(seed + k)
            info, llr = ex.synth(frames, e)
            pt = {"ebn0_db": e}
            for name, c in (("exact", ex), ("window", win)):
                bits = c.decode(llr)
                err = (bits != info)
                pt[f"{name}_bit_errors"] = int(err.sum().item())
                pt[f"{name}_block_errors"] = int(err.any(dim=1).sum().item())
                del bits, err
            rec["points"].append(pt)
            del info, llr
    p0, p1 = rec["points"]
    if min(p0["exact_bit_errors"], p1["exact_bit_errors"], p0["window_bit_errors"], p1["window_bit_errors"]) > 0:
        slope = math.log(p0["exact_bit_errors"] / p1["exact_bit_errors"]) / (points[1] - points[0])   # ln(BER) per dB
        rec["shift_db"] = [round(math.log(p["window_bit_errors"] / p["exact_bit_errors"]) / slope, 5)
                           for p in rec["points"]]
        rec["within_0.05_db"] = all(abs(x) <= 0.05 for x in rec["shift_db"])
    rec["wall_s"] = round(time.perf_counter() - t0, 2)
    return rec


def ref_gpu_schedule(a, big, f1, f2, dev, stream, P=32, iters=10):
    """Context only (not the metric): the reference's own CUDA decoder's schedule
    (ITTC/CUDA/turboDecoderBianJieZhi.cu: Max-Log-MAP fp32, P sub-blocks of 6144/P with NII
    boundaries, both SISOs concurrent, Le x 0.77) at 10 iterations -- the conditions of its
    published throughput, 73.18 Mbit/s at Eb/N0 = 1.0 dB for P = 32 on a GeForce GTX 550 Ti,
    one frame at a time, counting K+3 bits (FinalResult/throughoutput/8_4Blocks_Bian_Max_10000Fs06_20.txt:376).
    Here: td_set_window(6144/P, 0, 0.77, nii, concurrent) on a batch of 32768 of the bench's frames."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec

    ub, xb = big
    B = ub.shape[0]
    x = xb.float()
    c = TurboCodec(a.K, f1, f2, iterations=iters, algo="maxlog", precision="f32", device=dev.index)
    c.set_window(a.K // P, 0, 0.77, nii=True, concurrent=True)
    c.reserve(B)
    b = torch.empty((B, a.K), dtype=torch.uint8, device=dev)
    c.decode(x, b, stream=stream)
    torch.cuda.synchronize(dev)
    steps = max(2, a.steps // 2)
    t0 = time.perf_counter()
    for _ in range(steps):
        c.decode(x, b, stream=stream)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / steps
    c.close()
    errs = int((b != ub).sum().item())
    del x
    return {"value": round(B * a.K / dt / 1e6, 3), "unit": "Mbit/s", "value_k_plus_3": round(B * (a.K + 3) / dt / 1e6, 3),
            "batch": B, "iterations": iters, "P": P, "ms_per_step": round(dt * 1e3, 4), "bit_errors": errs,
            "reference_published": {"value": 73.18, "unit": "Mbit/s (K+3 bits)", "hardware": "GeForce GTX 550 Ti, one frame",
                                    "source": "ITTC/CUDA/FinalResult/throughoutput/8_4Blocks_Bian_Max_10000Fs06_20.txt:376"},
            "note": "context only: a different decoder (max-log fp32, sub-blocks, 0.77 scaling; ~0.5 dB worse BER) "
                    "from the metric's exact log-MAP path"}


def demod_rates(a, dev):
    """td_demodulate (modanddem.cpp:674) over one batch's symbols per
    modulation: HBM roofline with 16 B in + 8 M B out per symbol."""
    import torch

    from turbo_decoder_cuda_amd import demodulate
    res = {}
    g = torch.Generator(device=dev).manual_seed(5)
    for M in (1, 2, 4, 6):
        nsym = a.batch * (3 * a.K + 12) // M
        yi = torch.randn(nsym, dtype=torch.float64, device=dev, generator=g)
        yq = torch.randn(nsym, dtype=torch.float64, device=dev, generator=g)
        out = demodulate(yi, yq, M, 1.3)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 5
        e0.record()
        for _ in range(reps):
            demodulate(yi, yq, M, 1.3)
        e1.record()
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
        gbs = nsym * (16 + 8 * M) / (ms * 1e-3) / 1e9
        res[f"M{M}"] = {"symbols": nsym, "ms": round(ms, 4), "Msym_per_s": round(nsym / ms / 1e3, 1),
                        "GB_per_s": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
        del yi, yq, out
    return res


def _physical_cores():
    """Physical cores of the host (distinct (physical id, core id) pairs of /proc/cpuinfo)."""
    try:
        cores, phys, core = set(), None, None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":", 1)[1].strip()
                elif not line.strip():
                    if core is not None:
                        cores.add((phys, core))
                    phys = core = None
        if core is not None:
            cores.add((phys, core))
        return len(cores) or None
    except OSError:
        return None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
