"""C5 colour-gradient accuracy probe (10^3 bubble at setup): engine and oracle against the
colour gradient evaluated in long double from the oracle's inputs, for the worst elements.
pair_sph_colorgradient.cpp:130-181."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pyoracle as po  # noqa: E402
from c5_util import mp_engine, mp_state  # noqa: E402
from conftest import load_sph_amd  # noqa: E402
from scenarios import bubble_physics, bubble_system  # noqa: E402


def dwq3(s):
    """the quintic's dW/ds, factored (exact up to long double rounding)"""
    s = np.asarray(s, dtype=np.longdouble)
    a = np.maximum(3 - s, 0)
    b = np.maximum(2 - s, 0)
    c = np.maximum(1 - s, 0)
    return -5 * a ** 4 + 30 * b ** 4 - 75 * c ** 4


def dwq3_ref(s):
    """sph_kernel_quintic.cpp:43-57 in double: the expanded polynomials"""
    s = float(s)
    if s < 1:
        return -50 * s ** 4 + 120 * s ** 3 - 120 * s
    if s < 2:
        return 25 * s ** 4 - 180 * s ** 3 + 450 * s ** 2 - 420 * s + 75
    if s < 3.0:
        return -5 * s ** 4 + 60 * s ** 3 - 270 * s ** 2 + 540 * s - 405
    return 0.0


def main(nx=10):
    s = bubble_system(nx)
    ph = bubble_physics(nx, prob=0.5, Tt=-1.0)
    ref = po.MpRefRun(s, ph)
    ref.setup()
    g = ref.g
    L = np.longdouble
    n = s.n
    x = g.x.astype(L)
    sig = (ref.rho_all / ref.rm_all).astype(L)
    cut = ref.tabs["cg_cut"]
    alpha = ref.tabs["cg_alpha"]
    cg = np.zeros((n, 3), dtype=L)
    cgr = np.zeros((n, 3), dtype=L)  # (the terms with the reference's expanded dW in double)
    for i in range(n):
        js = ref.fnb[ref.foff[i]:ref.foff[i + 1]]
        ti = g.type[i]
        for j in js:
            tj = g.type[j]
            d = x[i] - x[j]
            rsq = (d * d).sum()
            h = L(cut[ti, tj])
            if not (float(rsq) < cut[ti, tj] ** 2) or alpha[ti, tj] == 0:
                continue
            r = np.sqrt(rsq)
            nrm = L(3.0 * 0.0716197243913529) * (L(1) / h) ** 4
            for out, dw in ((cg, dwq3(3 * r / h)), (cgr, L(dwq3_ref(3 * float(r) / float(h))))):
                dphi = -(dw * nrm) * L(alpha[ti, tj]) / (sig[j] * sig[j]) * sig[i]
                out[i] += dphi * d / r
    cgo = ref.cg
    sph = load_sph_amd()
    eng = mp_engine(sph, s, ph)
    eng.setup()
    cge = mp_state(eng)["cg"]
    t = cg.astype(np.float64)
    m = np.abs(t) > 1e-6 * np.abs(t).max()
    eo = np.where(m, np.abs(cgo - t) / np.where(m, np.abs(t), 1), 0)
    ee = np.where(m, np.abs(cge - t) / np.where(m, np.abs(t), 1), 0)
    print("max |cg| %.4g  oracle vs long double: max elem rel %.3e; engine: %.3e" %
          (np.abs(t).max(), eo.max(), ee.max()))
    tr = cgr.astype(np.float64)
    eor = np.where(m, np.abs(cgo - tr) / np.where(m, np.abs(t), 1), 0)
    print("oracle vs the expanded-dW long double sum: max elem rel %.3e" % eor.max())
    for idx in np.argsort(ee.ravel())[::-1][:6]:
        i, k = divmod(int(idx), 3)
        print(f"atom {i} comp {k}: exact {float(cg[i, k]):.17g} expanded {tr[i, k]:.17g} "
              f"oracle {cgo[i, k]:.17g} engine {cge[i, k]:.17g} rel(orc) {eo[i, k]:.2e} "
              f"rel(eng) {ee[i, k]:.2e}")


if __name__ == "__main__":
    main()
