"""Test configuration.  `-m gpu` tests need a HIP device (MI355X); everything else runs on CPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

LIB = os.path.join(ROOT, "ray_tracer_fragment_shader_amd", "lib", "librt_amd.so")
ORACLE = os.path.join(ROOT, "oracle", "librt_oracle.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "ref: needs /root/reference (the reference build, build container only)")
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "ray_tracer_fragment_shader_amd", "csrc"), "-j8"],
                       check=True, stdout=subprocess.DEVNULL)
    if not os.path.exists(ORACLE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "all"], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
