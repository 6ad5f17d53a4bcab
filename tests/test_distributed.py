"""Multi-rank bench logic on CPU (gloo, world_size 2): each rank decodes its own shard of
codewords, so the only exchange is the max of the timed-region wall time and the sum of the
error counters (bench.reduce_over_ranks); value = all ranks' info bits / max time."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, REPO)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    elapsed = [2.0, 2.5][rank]
    errs, blk = [10, 3][rank], [1, 2][rank]
    e, n, b = bench.reduce_over_ranks(elapsed, errs, blk, world)
    a = bench.parse(["--steps", "4", "--warmup", "1", "--batch", "64", "--K", "1024"])
    rec = bench.summarize(a, world, e, n, b, 0.1, 100.0, 4, 31, 64)
    q.put((rank, e, n, b, rec))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, e, n, b, rec in res:
        assert (e, n, b) == (2.5, 13, 3)
        assert rec["n_gpus"] == 2 and rec["scaling"] == "weak"
        assert rec["value"] == pytest.approx(2 * 64 * 1024 * 4 / 2.5 / 1e6, abs=1e-3)
        assert rec["config"]["global_batch"] == 128
        assert rec["ber"]["bit_errors"] == 13
        assert rec["roofline"]["alg_bytes_per_codeword"] == 8 * (3 * 1024 + 12) + 1024


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_layout_partitions_the_global_batch(world):
    """bench.shard_layout: the ranks' slices of the global frame stream are contiguous, disjoint
    and cover it exactly -- weak (a fixed batch per rank; N=8 x 32768 = config 4's 262144) and
    strong (one global batch split, remainder to the first ranks)."""
    import sys
    sys.path.insert(0, REPO)
    import bench

    for strong, batch, total in ((False, 32768, 32768 * world), (False, 45, 45 * world), (True, 0, 262144),
                                 (True, 0, 91), (True, 0, 7)):
        sl = [bench.shard_layout(world, r, batch, strong, total) for r in range(world)]
        pos = 0
        for first, n in sl:
            assert first == pos and n >= 0
            pos += n
        assert pos == total
        if strong:
            ns = [n for _, n in sl]
            assert max(ns) - min(ns) <= 1
    a = bench.parse([])
    assert bench.per_gpu_batch(a, 1) == 4096 and bench.per_gpu_batch(a, 8) == 32768
    assert 8 * bench.per_gpu_batch(a, 8) == bench.CONFIG4_GLOBAL


def test_traffic_model_matches_the_pmc_total():
    """The per-stream HBM model of the exact kernel (bench.traffic_model) against the PMC bytes
    per launch committed in profiles/traffic.json (config 2): within 2 %, alpha the largest share."""
    import json
    import sys
    sys.path.insert(0, REPO)
    import bench

    pmc = json.load(open(os.path.join(REPO, "profiles", "traffic.json")))["K6144_B4096_it8_f64_logmap"]
    # the record's kernel: v29 (round 3) streamed normalised alpha and tempmax, round 4 alpha_raw only
    m = bench.traffic_model(6144, 4096, 8, 8, "logmap", 15, alpha_raw=not pmc["kernel"].startswith("v29"))
    assert abs(m["total"] / pmc["bytes_per_launch"] - 1) < 0.02
    assert max(m["bytes"], key=m["bytes"].get) == "alpha"


def test_power_sampler_is_inert_without_a_gpu():
    """bench.PowerSampler (board power / clock record of the timed region) never fails a bench:
    with no GPU (or no amdsmi) its record is null."""
    import bench
    s = bench.PowerSampler(0).start()
    assert s.stop() is None


@pytest.mark.parametrize("exact_table", [False, True])
def test_window_roofline_record(exact_table):
    """bench.window_roofline (config 5's roofline object) from the committed PMC record: both floors
    present and consistent with the record (VALU: 4 cycles per wave64 instruction on 1024 SIMDs at the
    given clock; HBM: counter bytes at the measured ceiling), the binding one named, and the fraction
    = the binding floor / the decode time."""
    import json
    import sys
    sys.path.insert(0, REPO)
    import bench

    key = "K6144_B32768_it8_f64_logmap_w64g30" + ("_exacttable" if exact_table else "")
    rec = json.load(open(os.path.join(REPO, "profiles", "traffic.json"))).get(key)
    if rec is None:
        pytest.skip(f"no PMC record {key} committed yet")
    r = bench.window_roofline(6144, 32768, 8, 80.0, 2.2, exact_table=exact_table)
    assert r["traffic"] == rec["bytes_per_decode"] and r["valu_instr_per_decode"] == rec["valu_instr_per_decode"]
    assert abs(r["valu_floor_ms"] - rec["valu_instr_per_decode"] * 4 / 1024 / 2.2e9 * 1e3) < 1e-2
    assert abs(r["hbm_floor_ms"] - rec["bytes_per_decode"] / (bench.HBM_MEASURED_GBS * 1e9) * 1e3) < 1e-2
    floor = max(r["valu_floor_ms"], r["hbm_floor_ms"])
    assert r["binding"] == ("valu" if r["valu_floor_ms"] >= r["hbm_floor_ms"] else "hbm")
    assert abs(r["frac_of_binding"] - floor / 80.0) < 1e-3
    assert 0 < r["valu_issue_frac"] < 1 and 0 < r["traffic_frac"] < 1
    if exact_table:
        assert abs(r["frac_of_issue_ceiling"] - r["valu_issue_frac"] / bench.WINDOW_ISSUE_CEILING) < 1e-3
    assert abs(r["lane_valu_per_position"] - rec["valu_instr_per_decode"] * 64 / (32768 * 16 * 6147)) < 0.1
