"""The C ABI (include/turbo_mi355x.h) on a host without a GPU: the library loads, exports every
declared symbol, its host-side tables equal the oracle's / the reference's, argument errors
come back as status codes, and the compat layer (libturbo_logmap_compat.so) links where
ITTC/main.cpp expects log_map.o.  No GPU compute here."""
import ctypes as C
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

import pyoracle as O
from conftest import GOLD, REPO

from turbo_decoder_cuda_amd import _native as N

HEADER = os.path.join(REPO, "include", "turbo_mi355x.h")
PKG = os.path.join(REPO, "turbo_decoder_cuda_amd")
COMPAT = os.path.join(PKG, "libturbo_logmap_compat.so")
REF = "/root/reference/ITTC"


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(td_[a-z0-9_]+)\s*\(", text)))


def test_header_and_exports_agree():
    decl = declared_functions()
    assert set(decl) == set(N.EXPORTS), "EXPORTS and include/turbo_mi355x.h disagree"
    L = N.lib()
    for s in decl:
        assert hasattr(L, s), f"libturbo_mi355x.so does not export {s}"


def test_placement_probe_has_its_own_kernel_symbol():
    """td_reserve's one-iteration placement probes launch turbo_placement_probe_kernel, not
    turbo_decode_kernel, so kernel traces and PMC passes of a decode average the decode's own
    launches only (workspace placement).  Both names are in the gfx950 code object."""
    blob = open(N.LIB_PATH, "rb").read()
    for algo in (b"0", b"1"):
        for t in (b"d", b"f"):
            assert b"turbo_decode_kernelI" + t + b"Li" + algo in blob
            assert b"turbo_placement_probe_kernelI" + t + b"Li" + algo in blob


def test_abi_version_and_device_count():
    L = N.lib()
    assert L.td_abi_version() == 1
    assert L.td_device_count() >= 0


def test_trellis_tables_match_oracle():
    ns, ls, no = (np.zeros(n, dtype=np.int32) for n in (16, 16, 32))
    assert N.lib().td_trellis_tables(ns.ctypes.data, ls.ctypes.data, no.ctypes.data) == 0
    t = O.trellis()
    assert ns.tolist() == list(np.array(t.nextstat).ravel())
    assert ls.tolist() == list(np.array(t.laststat).ravel())
    assert no.tolist() == list(np.array(t.nextout).ravel())


@pytest.mark.parametrize("K,f1,f2", [(40, 3, 10), (1024, 31, 64), (6144, 263, 480), (10000, 1, 0)])
def test_qpp_table_matches_oracle(K, f1, f2):
    pi = np.zeros(K, dtype=np.int32)
    assert N.lib().td_qpp_table(K, f1, f2, pi.ctypes.data) == 0
    assert np.array_equal(pi, O.qpp(K, f1, f2))


def test_maxstar_lut_equals_reference_table():
    """The bucket LUT the kernels read (td_tables.h) reproduces E_algorithm
    (log_map.cpp:779-801) on the reference's own outputs, incl. every threshold edge."""
    d = np.load(os.path.join(GOLD, "maxstar.npz"))
    f = N.lib().td_maxstar_host_f64
    got = np.array([f(x, y, N.TD_ALGO_LOGMAP) for x, y in zip(d["x"], d["y"])])
    assert np.array_equal(got, d["r"])


def test_maxstar_lut_random_and_edges():
    rng = np.random.default_rng(1)
    f = N.lib().td_maxstar_host_f64
    g = N.lib().td_maxstar_host_f32
    xs = np.concatenate([rng.normal(0, 3, 20000), rng.uniform(-1e3, 1e3, 2000)])
    ys = xs + np.concatenate([rng.exponential(1.5, 20000) * rng.choice([-1, 1], 20000),
                              rng.uniform(-1e3, 1e3, 2000)])
    idx = [0.0, 0.08824, 0.19587, 0.31026, 0.43275, 0.56508, 0.70963, 0.86972,
           1.0502, 1.2587, 1.5078, 1.8212, 2.2522, 2.9706, 3.6764, 4.3758]
    edges = [v for t in idx for v in (np.nextafter(t, -1), t, np.nextafter(t, 9))]
    xs = np.concatenate([xs, np.full(len(edges), -1.5)])
    ys = np.concatenate([ys, -1.5 + np.array(edges)])
    for x, y in zip(xs, ys):
        assert f(x, y, N.TD_ALGO_LOGMAP) == O.maxstar(x, y)
        assert f(x, y, N.TD_ALGO_MAXLOG) == max(x, y)
    for x, y in zip(xs[:4000].astype(np.float32), ys[:4000].astype(np.float32)):
        assert g(x, y, N.TD_ALGO_LOGMAP) == np.float32(O.maxstar_f32(float(x), float(y)))


def test_window_one_read_maxstar():
    """The windowed schedule's one-read max* (td_set_window_maxstar TD_WMAXSTAR_FAST, td_tables.h
    build_qlut): the library's host evaluation equals the C restatement (TDO_ALGO_LOGMAP_Q, restated
    from the definition) on random pairs, every bucket edge of the 8-an-octave grid and the
    reference's thresholds, in fp64 and fp32; and it equals E_algorithm (log_map.cpp:779-801) except
    where |y - x| lies in a bucket that holds one of the reference's thresholds, where the two differ
    by exactly one table step."""
    f = N.lib().td_maxstar_host_f64
    g = N.lib().td_maxstar_host_f32
    rng = np.random.default_rng(7)
    xs = rng.normal(0, 3, 20000)
    ys = xs + rng.exponential(1.5, 20000) * rng.choice([-1, 1], 20000)
    grid = [np.ldexp(1 + m / 8, e) for e in range(-6, 5) for m in range(8)]
    idx = [0.08824, 0.19587, 0.31026, 0.43275, 0.56508, 0.70963, 0.86972,
           1.0502, 1.2587, 1.5078, 1.8212, 2.2522, 2.9706, 3.6764, 4.3758]
    edges = [v for t in grid + idx for v in (np.nextafter(t, -1), t, np.nextafter(t, 99))] + [0.0, 1e-300, 7.99, 8.0, 1e6]
    xs = np.concatenate([xs, np.full(len(edges), 2.25), np.full(len(edges), -7.0)])
    ys = np.concatenate([ys, 2.25 - np.array(edges), -7.0 + np.array(edges)])
    # the buckets (of the 8-an-octave grid) that hold a reference threshold
    def bucket(d):   # octave e, eighth m of it: [2^e (1 + m/8), 2^e (1 + (m+1)/8))
        if d <= 0:
            return -10**9
        m, e = np.frexp(d)   # d = m 2^e, m in [0.5, 1)
        return (int(e) - 1) * 8 + int((2 * m - 1) * 8)
    mixed = {bucket(t) for t in idx}
    tab = [0.69315, 0.65, 0.6, 0.55, 0.5, 0.45, 0.4, 0.35, 0.3, 0.25, 0.2, 0.15, 0.1, 0.05, 0.025, 0.0125]
    steps = {round(abs(a - b), 12) for a, b in zip(tab, tab[1:] + [0.0])}
    for x, y in zip(xs, ys):
        q = f(x, y, N.TD_MAXSTAR_WINDOW_FAST)
        assert q == O.maxstar_q(x, y), (x, y)
        d = abs(y - x)
        if q != O.maxstar(x, y):
            assert bucket(d) in mixed, (x, y, d)
            assert round(abs(q - O.maxstar(x, y)), 12) in steps, (x, y)
    for x, y in zip(xs[:4000].astype(np.float32), ys[:4000].astype(np.float32)):
        assert g(x, y, N.TD_MAXSTAR_WINDOW_FAST) == np.float32(O.maxstar_q_f32(float(x), float(y)))


def test_create_rejects_bad_arguments():
    L = N.lib()
    h = C.c_void_p()
    for K, f1, f2, it, algo, prec in ((0, 3, 10, 4, 0, 0), (10001, 1, 0, 4, 0, 0), (40, 3, 10, 0, 0, 0),
                                      (40, 3, 10, 65, 0, 0), (40, 3, 10, 4, 7, 0), (40, 3, 10, 4, 0, 9),
                                      (40, 2, 10, 4, 0, 0)):   # f1=2: not a permutation of 40
        p = N.TdParams(K, f1, f2, it, algo, prec, 0)
        assert L.td_create(C.byref(h), C.byref(p)) == N.TD_EINVAL
        assert L.td_last_error()
    with pytest.raises(N.TurboError):
        N.check(L.td_create(None, None))


def test_create_without_gpu_fails_loudly():
    from turbo_decoder_cuda_amd import TurboCodec, device_count
    if device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(N.TurboError) as e:
        TurboCodec(1024, 31, 64, iterations=4)
    assert e.value.code == N.TD_ENODEV


def test_null_handle_calls_are_errors():
    L = N.lib()
    assert L.td_reserve(None, 8) == N.TD_EINVAL
    assert L.td_decode_device(None, None, 1, None, 0, None, None) == N.TD_EINVAL
    assert L.td_destroy(None) == 0
    assert L.td_clock_read(None, None, None) == N.TD_EINVAL
    assert L.td_set_window_maxstar(None, 0) == N.TD_EINVAL
    assert L.td_debug_window_layout(None, 0, 0, 0) == N.TD_EINVAL
    assert L.td_debug_workspace_bytes(None, None) == N.TD_EINVAL


def test_window_steps_is_the_kernel_window():
    """td_window_steps: the exact kernel's window length (td_kernels.hip kW = 15), which
    bench.traffic_model takes; a multiple of the rotating labels' period 3."""
    W = N.lib().td_window_steps()
    assert W == 15 and W % 3 == 0


def test_dropin_latency_driver_built_and_linked():
    """examples/dropin_latency.cpp (bench.py `dropin`) is built in-tree by build() against the compat
    layer, i.e. it resolves the reference's C++ entry points from libturbo_logmap_compat.so."""
    exe = os.path.join(PKG, "td_dropin_latency")
    assert os.access(exe, os.X_OK), "run __graft_entry__.build()"
    und = subprocess.run(["nm", "-D", "--undefined-only", exe], check=True, capture_output=True, text=True).stdout
    for sym in ("_Z15TurboCodingInitv", "_Z13TurboDecodingPdPii", "_Z18TurboCodingReleasev"):
        assert sym in und


# ---------------------------------------------------------------- compat layer (C++ entry points)
@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not os.path.exists(COMPAT):
        pytest.fail("libturbo_logmap_compat.so missing: run python turbo_decoder_cuda_amd/build.py")
    out = str(tmp_path_factory.mktemp("compat") / "compat_driver")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", out, os.path.join(REPO, "tests", "compat_driver.cpp"),
                           f"-L{PKG}", "-lturbo_logmap_compat", "-lturbo_mi355x", f"-Wl,-rpath,{PKG}"])
    return out


def test_compat_exports_reference_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", COMPAT], check=True, capture_output=True, text=True).stdout
    for sym in ("_Z15TurboCodingInitv", "_Z13TurboEnCodingPiS_i", "_Z13TurboDecodingPdPii",
                "_Z18TurboCodingReleasev", "_Z4AWGNPdS_di", "_Z15Log_MAP_decoderPdS_iS_i", "M_num_reg"):
        assert re.search(rf"\b{sym}\b", out), sym
    undef = subprocess.run(["nm", "-D", "--undefined-only", COMPAT], check=True, capture_output=True,
                           text=True).stdout
    for g in ("source_length", "f1", "f2"):   # owned by the caller (ITTC/main.h:6-11)
        assert re.search(rf"\b{g}\b", undef), g


@pytest.mark.parametrize("K,f1,f2", [(40, 3, 10), (1024, 31, 64), (6144, 263, 480)])
def test_compat_encoder_matches_oracle(driver, tmp_path, K, f1, f2):
    src = np.random.default_rng(K).integers(0, 2, K).astype(np.int32)
    src.tofile(tmp_path / "s.bin")
    subprocess.check_call([driver, "encode", str(K), str(f1), str(f2), str(tmp_path / "s.bin"),
                           str(tmp_path / "c.bin")])
    coded = np.fromfile(tmp_path / "c.bin", dtype=np.int32)
    assert np.array_equal(coded, O.encode(src, f1, f2))


def test_compat_awgn_matches_oracle(driver, tmp_path):
    """AWGN: seed from the process's rand() after srand(seed), then mgrns (log_map.cpp:1359-1400)."""
    n, sigma, seed = 3084, 1.2, 17
    send = np.random.default_rng(0).choice([-1.0, 1.0], n)
    send.tofile(tmp_path / "x.bin")
    subprocess.check_call([driver, "awgn", str(n), repr(sigma), str(seed), str(tmp_path / "x.bin"),
                           str(tmp_path / "r.bin")])
    r = np.fromfile(tmp_path / "r.bin", dtype=np.float64)
    rnd = int(O.glibc_rand_stream(seed, 1)[0])
    s = 3.0 - (rnd / 2147483647.0) / 10e6
    noise = np.zeros(n)
    O.lib().tdo_mgrns(0.0, sigma, s, n, noise.ctypes.data_as(C.c_void_p))
    assert np.array_equal(r, send + noise)


@pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("make") is None, reason="needs /root/reference")
def test_reference_main_links_against_compat():
    """ITTC/main.cpp + modanddem.cpp (the reference caller) link against the compat layer in
    place of log_map.cpp, with no other change (oracle/Makefile target compat-link)."""
    subprocess.check_call(["make", "-s", "-B", "-C", os.path.join(REPO, "oracle"), "compat-link"])
    exe = os.path.join(REPO, "oracle", "_ref", "main_compat")
    ldd = subprocess.run(["ldd", exe], check=True, capture_output=True, text=True).stdout
    assert "libturbo_logmap_compat.so" in ldd and "libturbo_mi355x.so" in ldd


def test_rand_window_jump_matches_glibc_stream():
    """The generator's jump-ahead (td_rand_window: srand(seed) window advanced by a power of the
    lagged-Fibonacci companion matrix) continues glibc's rand() stream exactly (the oracle's
    glibc restatement, itself pinned by the reference's golden frames)."""
    for seed in (1, 11, 2026):
        ref = O.glibc_rand_stream(seed, 2600)
        for d in (0, 1, 30, 31, 100, 2500):
            w = np.zeros(31, dtype=np.uint32)
            assert N.lib().td_rand_window(seed, d, w.ctypes.data) == 0
            x = [int(v) for v in w]
            outs = []
            for _ in range(40):
                v = (x[-31] + x[-3]) & 0xFFFFFFFF
                x.append(v)
                outs.append(v >> 1)
            assert outs == list(ref[d:d + 40])


def test_compat_rejects_more_iterations_than_flow_decoded_rows(driver, tmp_path):
    """main.cpp sizes flow_decoded as N_ITERATION (15) rows (main.cpp:153): TD_ITERATIONS above 15
    would make TurboDecoding write past the caller's buffer, so TurboCodingInit refuses it
    (exit 1, like the reference's init failures) before any device work."""
    K = 40
    np.zeros(3 * K + 12).tofile(tmp_path / "flow.bin")
    for bad in ("16", "0"):
        r = subprocess.run([driver, "decode", str(K), "3", "10", "1", str(tmp_path / "flow.bin"),
                            str(tmp_path / "out.bin")], env={**os.environ, "TD_ITERATIONS": bad},
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 1 and "TD_ITERATIONS" in r.stdout, (bad, r.stdout, r.stderr)


def test_decode_output_buffer_checks():
    """TurboCodec.decode validates caller-supplied output buffers before the kernels write
    B*iterations*K bits / B*iterations*2*(K+3) Le into them (dtype, shape, device, layout)."""
    import torch

    from turbo_decoder_cuda_amd import TurboCodec
    chk = TurboCodec._check_out
    dev = torch.device("cpu")
    chk("bits", torch.empty((4, 8), dtype=torch.uint8), torch.uint8, (4, 8), dev)
    bad = [torch.empty((4, 8), dtype=torch.int32),          # dtype
           torch.empty((4, 3, 8), dtype=torch.uint8),       # all_iters shape given to a final-only decode
           torch.empty((8, 4), dtype=torch.uint8).t(),      # not contiguous
           torch.empty((3, 8), dtype=torch.uint8)]          # too few rows
    for t in bad:
        with pytest.raises(ValueError):
            chk("bits", t, torch.uint8, (4, 8), dev)


def test_multi_gpu_example_builds(tmp_path):
    """examples/multi_gpu_decode.cpp (one handle + thread + stream per device ordinal) compiles and
    links against the C ABI with plain g++ and the HIP runtime headers (run: tests/test_gpu_multidevice.py)."""
    pkg = os.path.join(REPO, "turbo_decoder_cuda_amd")
    out = str(tmp_path / "mgd")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", f"-I{REPO}/include",
                           "-I/opt/rocm/include", os.path.join(REPO, "examples", "multi_gpu_decode.cpp"),
                           f"-L{pkg}", "-lturbo_mi355x", "-L/opt/rocm/lib", "-lamdhip64", "-lpthread",
                           f"-Wl,-rpath,{pkg}", "-Wl,-rpath,/opt/rocm/lib", "-o", out])
    r = subprocess.run([out], capture_output=True, text=True)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.parametrize("ms,stop", [
    ([2.3898, 2.3797, 2.3829, 2.378, 2.3972, 2.3827, 2.4883], 0),   # round 2's driver box: all slow + a straggler
    ([2.3898, 2.3797], 0),                                          # two candidates never decide
    ([2.3898, 2.3797, 2.2212], 1),                                  # a fast one below the median
    ([2.2812, 2.3907, 2.4039], 1),                                  # fast first, then two slow
    ([2.2895, 2.2386, 2.2215, 2.2343, 2.2303], 0),                  # fast mode only: keep looking
    ([2.2895, 2.2386, 2.2215, 2.2343, 2.3797, 2.4022, 2.3166], 1),  # ... until the slow mode shows thrice
])
def test_placement_stop_rule(ms, stop, monkeypatch):
    """td_reserve's placement search stops only once the fast mode is evident (td_api.cpp
    placement_fast_seen): never on a slow straggler.  (The mode rule alone: TD_PLACEMENT_MIN=3.)"""
    import ctypes as C
    monkeypatch.setenv("TD_PLACEMENT_MIN", "3")
    arr = (C.c_float * len(ms))(*ms)
    assert N.lib().td_debug_placement_rule(arr, len(ms)) == stop


@pytest.mark.parametrize("ms,stop", [
    ([2.3927, 2.3856, 2.2803], 0),                                  # round 3: a middle level, 3 probed
    ([2.3927, 2.3856, 2.2803, 2.4011, 2.3902, 2.2876, 2.3957], 0),  # seven: not yet
    ([2.3927, 2.3856, 2.2803, 2.4011, 2.3902, 2.2876, 2.3957, 2.2308], 1),
    ([2.3927] * 7 + [2.4883], 0),                                   # all slow + a straggler: keep looking
])
def test_placement_stop_rule_min_candidates(ms, stop, monkeypatch):
    """By default the search probes at least eight candidates before either stop rule applies, so
    a middle-level candidate (4 % below a slow median, 2 % above the fastest level) does not end it."""
    import ctypes as C
    monkeypatch.delenv("TD_PLACEMENT_MIN", raising=False)
    arr = (C.c_float * len(ms))(*ms)
    assert N.lib().td_debug_placement_rule(arr, len(ms)) == stop


@pytest.mark.parametrize("name", ["libturbo_mi355x_redo.so", "libturbo_mi355x_stamps.so"])
def test_test_builds_load_and_export_the_abi(name):
    """build() also makes the redo-forced build (tests/test_gpu_decode.py, the α speculation's exact
    redo on every window) and the stamps build (scripts/diag_stamps.py): both load without a GPU and
    export every declared entry point, so a TD_LIB_PATH swap is a drop-in (checked in a child
    process: one process, one copy of the HIP runtime's kernel registrations)."""
    path = os.path.join(PKG, name)
    assert os.path.exists(path), f"build() makes {name}"
    code = ("import ctypes, sys; L = ctypes.CDLL(sys.argv[1]); "
            "missing = [s for s in sys.argv[2:] if not hasattr(L, s)]; print(missing); sys.exit(1 if missing else 0)")
    r = subprocess.run(["python", "-c", code, path, *declared_functions()], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
