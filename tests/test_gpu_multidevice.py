"""The C++ multi-device caller (examples/multi_gpu_decode.cpp): one td_handle, one
host thread and one HIP stream per device ordinal, each decoding a contiguous slice of one batch.
On a one-GPU box the ordinals repeat (0 0 0): three handles on one device from three threads,
each with its own workspace.  The bits must equal the oracle's for every codeword."""
import os
import subprocess

import numpy as np
import pytest

import pyoracle as O
from conftest import REPO

pytestmark = pytest.mark.gpu

PKG = os.path.join(REPO, "turbo_decoder_cuda_amd")


@pytest.fixture(scope="module")
def prog(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("mgd") / "multi_gpu_decode")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", f"-I{REPO}/include",
                           "-I/opt/rocm/include", os.path.join(REPO, "examples", "multi_gpu_decode.cpp"),
                           f"-L{PKG}", "-lturbo_mi355x", "-L/opt/rocm/lib", "-lamdhip64", "-lpthread",
                           f"-Wl,-rpath,{PKG}", "-Wl,-rpath,/opt/rocm/lib", "-o", out])
    return out


@pytest.mark.parametrize("ordinals", [["0"], ["0", "0"], ["0", "0", "0"]])
def test_multi_handle_threads_equal_oracle(prog, tmp_path, ordinals):
    import torch
    K, f1, f2, iters, B = 1024, 31, 64, 4, 21
    _, flow = O.synth_batch(K, f1, f2, 0.5, 77, B)
    flow.astype(np.float64).tofile(tmp_path / "flows.bin")
    ordinals = [str(int(o) % max(1, torch.cuda.device_count())) for o in ordinals]
    r = subprocess.run([prog, str(K), str(f1), str(f2), str(iters), str(tmp_path / "flows.bin"),
                        str(tmp_path / "bits.bin"), *ordinals], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    bits = np.fromfile(tmp_path / "bits.bin", dtype=np.uint8).reshape(B, K)
    ob = O.decode_batch(np.ascontiguousarray(flow), K, f1, f2, iters, nthreads=8)
    assert np.array_equal(bits, ob)
