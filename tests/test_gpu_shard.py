"""Sharded equals unsharded: bench.py launched as two torchrun ranks (fresh
child processes sharing the one GPU, as bench.py allows), each decoding its slice of the global
frame stream; the slices concatenated must equal a single-process decode of the same global batch
bit for bit -- weak (a batch per rank) and strong (one global batch split, ragged)."""
import glob
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

K, F1, F2, ITERS, EBN0 = 1024, 31, 64, 4, 0.6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(tmp_path, extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--K", str(K), "--iters", str(ITERS), "--ebn0", str(EBN0),
           "--cpu-sample", "0", "--no-variants", "--dump-bits", str(tmp_path), *extra]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", TD_PLACEMENT_TRIALS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


def _single_decode(total):
    import torch

    sys.path.insert(0, REPO)
    import bench
    from turbo_decoder_cuda_amd import TurboCodec
    with TurboCodec(K, F1, F2, iterations=ITERS) as c:
        c.synth_seed(bench.SEED)
        _, llr = c.synth(total, EBN0)
        bits = c.decode(llr)
        torch.cuda.synchronize()
        return bits.cpu().numpy()


def _gathered(tmp_path):
    parts = []
    for f in glob.glob(os.path.join(str(tmp_path), "bits_rank*_first*.npy")):
        first = int(f.rsplit("_first", 1)[1].split(".")[0])
        parts.append((first, np.load(f)))
    parts.sort(key=lambda x: x[0])
    pos = 0
    for first, b in parts:
        assert first == pos
        pos += b.shape[0]
    return np.concatenate([b for _, b in parts])


@pytest.mark.timeout(300)
def test_weak_shards_equal_single_process_decode(tmp_path):
    rec = _run_ranks(tmp_path, ["--batch", "45"])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 90 and rec["scaling"] == "weak"
    assert np.array_equal(_gathered(tmp_path), _single_decode(90))


@pytest.mark.timeout(300)
def test_strong_shards_equal_single_process_decode(tmp_path):
    rec = _run_ranks(tmp_path, ["--strong", "--global-batch", "91"])
    assert rec["config"]["global_batch"] == 91 and rec["scaling"] == "strong"
    got = _gathered(tmp_path)
    assert got.shape[0] == 91
    assert np.array_equal(got, _single_decode(91))
