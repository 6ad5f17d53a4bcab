"""Handle-level behaviour on the GPU: the workspace placement search of td_reserve and decodes
captured into a hipGraph, both checked against the oracle."""
import os

import time

import numpy as np
import pytest

import pyoracle as O

pytestmark = pytest.mark.gpu


def _dev():
    import torch
    return torch.device("cuda", 0)


def test_reserve_placement_search_decodes_like_the_oracle(monkeypatch):
    """td_reserve with TD_PLACEMENT_TRIALS=3 at B=1024 (the smallest batch it searches at): 1 to
    3 candidates timed, a valid pick, and a decode on the chosen workspace equal to the oracle."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    monkeypatch.setenv("TD_PLACEMENT_TRIALS", "3")
    K, f1, f2, iters, B = 40, 3, 10, 3, 1024
    _, flow = O.synth_batch(K, f1, f2, 0.5, 4242, B)
    x = torch.from_numpy(flow).to(_dev())
    with TurboCodec(K, f1, f2, iterations=iters) as c:
        c.reserve(B)
        ms, pick = c.placement()
        assert 1 <= len(ms) <= 3 and 0 <= pick < len(ms)
        assert all(m > 0 for m in ms) and ms[pick] == min(ms)
        bits = c.decode(x)
        torch.cuda.synchronize()
    ob = O.decode_batch(np.ascontiguousarray(flow), K, f1, f2, iters, nthreads=8)
    assert np.array_equal(bits.cpu().numpy(), ob)


def test_placement_search_holds_at_most_three_workspaces(monkeypatch):
    """Round 6: the search recycles candidates, so however many it probes it
    holds at most three workspaces plus a 48 MiB spacer per recycled candidate; the kept candidate is
    the fastest probed; and the chosen workspace decodes like the oracle."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    monkeypatch.setenv("TD_PLACEMENT_TRIALS", "7")
    monkeypatch.setenv("TD_PLACEMENT_MIN", "100")   # no early stop: all 7 probed
    K, f1, f2, iters, B = 40, 3, 10, 3, 1024
    _, flow = O.synth_batch(K, f1, f2, 0.5, 4343, B)
    x = torch.from_numpy(flow).to(_dev())
    with TurboCodec(K, f1, f2, iterations=iters) as c:
        c.reserve(B)
        ms, pick = c.placement()
        _, held = c.placement_cost()
        ws = c.workspace_bytes()
        assert len(ms) == 7 and ms[pick] == min(ms)
        assert ws > 0 and held <= 3 * ws + 4 * (48 << 20), (held, ws)
        bits = c.decode(x)
        torch.cuda.synchronize()
    ob = O.decode_batch(np.ascontiguousarray(flow), K, f1, f2, iters, nthreads=8)
    assert np.array_equal(bits.cpu().numpy(), ob)


def test_reserve_after_a_growing_decode_keeps_the_workspace(monkeypatch):
    """a decode that grows the workspace (plain allocation), then td_reserve for the
    same batch: the workspace is big enough, so the reserve neither frees it nor searches."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    monkeypatch.setenv("TD_PLACEMENT_TRIALS", "3")
    K, B = 40, 1024
    x = torch.zeros((B, 3 * K + 12), dtype=torch.float64, device=_dev())
    with TurboCodec(K, 3, 10, iterations=2) as c:
        c.decode(x)
        torch.cuda.synchronize()
        ws = c.workspace_bytes()
        c.reserve(B)
        assert c.placement() == ([], -1)
        assert c.workspace_bytes() == ws


def test_set_window_maxstar_rejects_bad_forms():
    from turbo_decoder_cuda_amd import TurboCodec
    from turbo_decoder_cuda_amd import _native as N
    with TurboCodec(40, 3, 10, iterations=2) as c:
        for form in (-1, 2, 7):
            with pytest.raises(N.TurboError):
                N.check(N.lib().td_set_window_maxstar(c._h, form))
        c.set_window_maxstar(True)
        c.set_window_maxstar(False)


def test_plain_allocation_reports_no_placement(monkeypatch):
    from turbo_decoder_cuda_amd import TurboCodec
    monkeypatch.setenv("TD_PLACEMENT_TRIALS", "1")
    with TurboCodec(40, 3, 10, iterations=2) as c:
        c.reserve(2048)
        assert c.placement() == ([], -1)


def test_graph_capture_between_eager_decodes():
    """Eager decode on stream A, capture of a decode on stream B (torch.cuda.graph, hipGraph
    capture), two replays, then an eager decode on stream C: every output equals the oracle.  The
    captured decode neither waits on nor records the handle's workspace event (td_api.cpp), so
    the capture stays isolated and the later eager decode does not wait on a captured event."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    K, f1, f2, iters, B = 1024, 31, 64, 3, 16
    dev = _dev()
    flows = [O.synth_batch(K, f1, f2, 0.2 + 0.1 * k, 500 + k, B)[1] for k in range(3)]
    ref = [O.decode_batch(np.ascontiguousarray(f), K, f1, f2, iters, nthreads=8) for f in flows]
    xs = [torch.from_numpy(f).to(dev) for f in flows]
    sa, sb, sc = (torch.cuda.Stream(dev) for _ in range(3))
    torch.cuda.synchronize()
    with TurboCodec(K, f1, f2, iterations=iters) as c:
        c.reserve(B)   # no workspace growth inside the capture
        with torch.cuda.stream(sa):
            out_a = c.decode(xs[0], stream=sa)
        sa.synchronize()
        assert np.array_equal(out_a.cpu().numpy(), ref[0])

        gin = xs[1].clone()
        gout = torch.empty((B, K), dtype=torch.uint8, device=dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=sb):
            c.decode(gin, gout, stream=sb)
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(gout.cpu().numpy(), ref[1])
        gin.copy_(xs[2])
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(gout.cpu().numpy(), ref[2])

        with torch.cuda.stream(sc):
            out_c = c.decode(xs[0], stream=sc)
        sc.synchronize()
        assert np.array_equal(out_c.cpu().numpy(), ref[0])


def test_launch_clock_and_host_staging_reuse():
    """td_clock_read after an exact-schedule decode: a sustained shader clock in the MI355X's range
    (2.4 GHz peak) over a span no longer than the decode; td_decode_host keeps its device staging
    across calls of different B (1, 5, 1) and every call decodes like the oracle."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    K, f1, f2, iters = 1024, 31, 64, 3
    _, flow = O.synth_batch(K, f1, f2, 0.4, 77, 5)
    with TurboCodec(K, f1, f2, iterations=iters) as c:
        with pytest.raises(Exception):
            c.clock()   # no exact-schedule launch yet
        x = torch.from_numpy(flow).to(torch.device("cuda", 0))
        t0 = time.perf_counter()
        c.decode(x)
        torch.cuda.synchronize()
        wall_ms = (time.perf_counter() - t0) * 1e3
        ghz, span = c.clock()
        assert 0.5 < ghz < 3.0, ghz
        assert 0 < span <= wall_ms + 1.0, (span, wall_ms)
        for rows in (slice(0, 1), slice(0, 5), slice(3, 4)):
            out = c.TurboDecoding(flow[rows])
            for b, fr in enumerate(range(5)[rows]):
                ob, _ = O.turbo_decode(flow[fr], K, f1, f2, iters)
                assert np.array_equal(out[b].astype(np.uint8), ob.astype(np.uint8)), (rows, fr)


def test_graph_capture_windowed_two_streams():
    """A windowed decode large enough to run in two batch parts (two streams, fork / join events)
    captured into a hipGraph: both replays equal the eager decode of the same input bit for bit, and
    sampled codewords of both parts equal the C restatement of the windowed schedule."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    K, f1, f2, iters, W, g = 512, 31, 64, 3, 64, 30
    B = 2 * 64 * 64 + 5                      # 129 waves of 64 codewords: two parts
    dev = _dev()
    flows = [np.tile(O.synth_batch(K, f1, f2, 0.3 + 0.2 * k, 900 + k, 64)[1], (B // 64 + 1, 1))[:B] for k in range(2)]
    xs = [torch.from_numpy(np.ascontiguousarray(f)).to(dev) for f in flows]
    sb = torch.cuda.Stream(dev)
    with TurboCodec(K, f1, f2, iterations=iters) as c:
        # the documented order: set_window (creates the streams), reserve (sizes every buffer), then
        # capture -- no eager decode before it
        c.set_window(W, g)
        c.reserve(B)
        gin = xs[0].clone()
        gout = torch.empty((B, K), dtype=torch.uint8, device=dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=sb):
            c.decode(gin, gout, stream=sb)
        replayed = []
        for k in (0, 1):
            gin.copy_(xs[k])
            graph.replay()
            torch.cuda.synchronize()
            replayed.append(gout.cpu().numpy().copy())
        eager = [c.decode(x).cpu().numpy() for x in xs]
        torch.cuda.synchronize()
        for k in (0, 1):
            assert np.array_equal(replayed[k], eager[k]), k
    for k in (0, 1):
        for b in (3, 64 * 64 + 9, B - 1):
            ob, _ = O.turbo_decode_window(flows[k][b], K, f1, f2, iters, W, g, algo=O.ALGO_LOGMAP_Q)
            assert np.array_equal(eager[k][b], ob[-1]), (k, b)
