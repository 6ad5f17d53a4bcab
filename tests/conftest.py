import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))   # pyoracle: the CPU checker (test infrastructure)

GOLD = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libturbo_mi355x.so")


def gpu_available() -> bool:
    try:
        from turbo_decoder_cuda_amd import device_count
        return device_count() > 0
    except Exception:
        return False
