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


SPREAD_K = 16.0  # elementwise bar: |a_i - b_i| <= max(1e-10 |b_i|, SPREAD_K * spread_i)


def elem_ratio(a, b, spread=None, tol=1e-10, k=SPREAD_K, floor=1e-6):
    """SURVEY.md 8(d)'s elementwise bar as a ratio (<= 1 passes): the worst
    |a_i - b_i| / max(tol |b_i|, k s_i) over the elements with |b_i| > floor ||b||_inf, where
    s_i is how far the reference's own result for element i moves under changes that leave
    its mathematics alone (pyoracle RefRun / MpRefRun spread=True, the _Spread shadow runs:
    every list row reversed, every row rotated, the inputs moved by one ulp, and for the
    multiphase stack the quintic dW evaluated factored instead of expanded).  Without a
    spread it is the plain elementwise relative error / tol.  Where an element's sum nearly
    cancels, or its terms carry the expanded quintic's cancellation (the reference's own
    colour gradient is up to ~8e-11 off the exact value there, where the engine is within
    1e-14: tools/cg_probe.py, profiles/r05/README.md), its relative error under any of these
    is that large.  k = 16 (the round-4 verdict's recipe with the factor committed here)."""
    a = np.asarray(a, dtype=np.float64).ravel()
    b = np.asarray(b, dtype=np.float64).ravel()
    if not b.size:
        return 0.0
    m = np.abs(b) > floor * np.abs(b).max()
    if not m.any():
        return 0.0
    den = tol * np.abs(b[m])
    if spread is not None:
        den = np.maximum(den, k * np.asarray(spread, dtype=np.float64).ravel()[m])
    return float((np.abs(a[m] - b[m]) / den).max())


def check_fields(got, ref, fields, tol=1e-10, where=""):
    """normwise (||a-b||_inf / ||b||_inf <= tol) and elementwise (elem_ratio <= 1) parity of
    the named fields of an engine state against an oracle run (RefRun / MpRefRun)"""
    for k in fields:
        want = ref.field(k)
        if np.abs(np.asarray(want)).max() == 0:
            assert rel_err(got[k], want) == 0.0, (where, k)
            continue
        sp = ref.spread(k)
        # normwise: 1e-10, or k x the oracle's own normwise reordering spread where that is
        # larger (perfect lattices, whose force sums cancel: test_c5_bricks)
        ntol = tol if sp is None else max(tol, SPREAD_K * float(np.abs(sp).max()) /
                                          float(np.abs(np.asarray(want)).max()))
        assert rel_err(got[k], want) < ntol, (where, k, "normwise", rel_err(got[k], want))
        r = elem_ratio(got[k], want, sp, tol=tol)
        if r > 1.0:  # (the worst element, for the record)
            a = np.asarray(got[k], dtype=np.float64).ravel()
            b = np.asarray(want, dtype=np.float64).ravel()
            m = np.abs(b) > 1e-6 * np.abs(b).max()
            den = tol * np.abs(b)
            if sp is not None:
                den = np.maximum(den, SPREAD_K * np.asarray(sp, dtype=np.float64).ravel())
            q = np.where(m, np.abs(a - b) / np.where(den > 0, den, 1.0), 0.0)
            i = int(np.argmax(q))
            detail = dict(i=i, got=a[i], want=b[i], spread=None if sp is None else
                          float(np.asarray(sp).ravel()[i]), maxabs=float(np.abs(b).max()))
        assert r <= 1.0, (where, k, "elementwise", r, detail if r > 1.0 else None)
