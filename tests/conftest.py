"""Shared fixtures.  `-m "not gpu"` runs the oracle, golden-vector, host-logic and ABI
tests on CPU; `-m gpu` runs the HIP parity tests (they call libsph_hip.so through its C
ABI and compare with the oracle)."""
import importlib.util
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import pyoracle  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests of the HIP path")
    config.addinivalue_line("markers", "ref: needs the reference oracle build (oracle/_ref)")


def load_sph_amd():
    spec = importlib.util.spec_from_file_location(
        "sph_amd", os.path.join(ROOT, "lammps-sph-multiphase_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["sph_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def sph_amd():
    return load_sph_amd()


@pytest.fixture(scope="session")
def po():
    pyoracle.build_oracle()
    return pyoracle


@pytest.fixture(scope="session")
def ref(po):
    """The reference's own compute code; built on demand where /root/reference exists."""
    if not po.ref_available() and os.path.isdir("/root/reference/src"):
        import subprocess
        subprocess.run([os.path.join(ROOT, "oracle", "build_ref.sh")], check=True,
                       stdout=subprocess.DEVNULL)
    if not po.ref_available():
        pytest.skip("reference oracle (oracle/_ref) not available on this machine")
    return po.ref()


@pytest.fixture(scope="session")
def gpu(sph_amd):
    """A usable HIP device, or a hard failure (GPU tests must not silently pass)."""
    n = sph_amd.device_count()
    assert n > 0, "no HIP device visible: -m gpu tests need an MI355X"
    return 0


def rel_err(a, b):
    """Normwise relative error ||a-b||_inf / ||b||_inf (SURVEY.md 8(d) parity metric)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.abs(b).max() if b.size else 0.0
    if den == 0.0:
        return float(np.abs(a - b).max()) if a.size else 0.0
    return float(np.abs(a - b).max() / den)


def elem_rel_err(a, b, floor=1e-6):
    """Elementwise relative error where |b| > floor*||b||_inf."""
    a = np.asarray(a, dtype=np.float64).ravel()
    b = np.asarray(b, dtype=np.float64).ravel()
    if not b.size:
        return 0.0
    m = np.abs(b) > floor * np.abs(b).max()
    if not m.any():
        return 0.0
    return float((np.abs(a[m] - b[m]) / np.abs(b[m])).max())
