"""Elementwise parity probe (rel <= 1e-10 where |b| > 1e-6 ||b||_inf): the
engine against the oracle, and the oracle against itself with every list row reversed (its
own reordering spread), per field, for C2 / C3 at edge^3 over a few steps.
Usage: python tools/elem_probe.py c2|c3 EDGE STEPS"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pyoracle as po  # noqa: E402
from conftest import load_sph_amd  # noqa: E402
from scenarios import c2_system, c3_system  # noqa: E402
from test_gpu_engine import engine_for  # noqa: E402


def elem(a, b, floor=1e-6):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    m = np.abs(b) > floor * np.abs(b).max()
    r = np.zeros_like(b)
    r[m] = np.abs(a[m] - b[m]) / np.abs(b[m])
    return r, m


def main(wl, edge, steps):
    sph = load_sph_amd()
    s = (c2_system if wl == "c2" else c3_system)(edge)
    ph = po.c2_physics() if wl == "c2" else po.c3_physics()
    eng = engine_for(sph, s, ph)
    eng.setup()
    ref = po.RefRun(s, ph)
    alt = po.RefRun(s, ph)
    alt.rev = True
    ref.setup()
    alt.setup()
    for k in range(steps + 1):
        if k:
            eng.run(1)
            ref.run(1)
            alt.run(1)
        got = eng.get_atoms()
        for f, want, other in (("rho", ref.s.rho, alt.s.rho), ("f", ref.f, alt.f),
                               ("drho", ref.drho, alt.drho), ("de", ref.de, alt.de),
                               ("e", ref.s.e, alt.s.e), ("x", ref.s.x, alt.s.x),
                               ("v", ref.s.v, alt.s.v)):
            if np.abs(want).max() == 0:
                continue
            r, m = elem(got[f], want)
            sp, _ = elem(other, want)
            tol = np.maximum(1e-10, 4.0 * sp)
            i = int(np.argmax(r))
            print(f"step {k} {f:5s} elem max {r.max():.3e} (spread there {sp.ravel()[i]:.2e}) "
                  f"oracle spread max {sp.max():.3e}  n>1e-10 {(r > 1e-10).sum()}  "
                  f"worst err/tol {(r / tol).max():.3f}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))
