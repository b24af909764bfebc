"""The reference's own known-answer tests, restated.

examples/USER/sph/multiphase_two_atoms/ pairs a 2-3 atom LAMMPS input with a Maxima script
(*.mac) that evaluates the same quantity symbolically from scripts/sph-kernel.mac.  No
expected outputs are committed there and Maxima is not installed, so the .mac formulas
are restated below in closed form (numpy, independent of the C code) and the oracle's
multiphase styles must reproduce them on the .lmp geometries.  These are the "parity
unpinned by outputs, pinned by the reference's own formulas" cases of SURVEY.md section 4.
"""
import numpy as np
import pytest

import pyoracle as po

NORM3 = 9.0 / (40.0 * np.pi)          # sph-kernel.mac quintic norm[3]


def fsim(s):                           # quintic shape, sph-kernel.mac (s = 3r/h)
    if s < 1:
        return (3 - s) ** 5 - 6 * (2 - s) ** 5 + 15 * (1 - s) ** 5
    if s < 2:
        return (3 - s) ** 5 - 6 * (2 - s) ** 5
    if s < 3:
        return (3 - s) ** 5
    return 0.0


def dfsim(s):                          # factor(diff(fsim, s))
    if s < 1:
        return -5 * (3 - s) ** 4 + 30 * (2 - s) ** 4 - 75 * (1 - s) ** 4
    if s < 2:
        return -5 * (3 - s) ** 4 + 30 * (2 - s) ** 4
    if s < 3:
        return -5 * (3 - s) ** 4
    return 0.0


def w(r, h):                           # define_kernel(3, h, 'quintic, w, dw)
    return NORM3 * fsim(3 * r / h) / h ** 3


def dw(r, h):
    return 3 * NORM3 / h * dfsim(3 * r / h) / h ** 3


X3 = np.array([[5, 5, 5], [5.5, 5, 5], [5, 5, 4.8]], dtype=np.float64)
T3 = np.array([1, 2, 2], dtype=np.int32)
M3 = np.array([2.0, 1.0, 1.0])          # set type 1 mass 2 / type 2 mass 1
H = 1.0


def lists(n):
    """All-pairs full list and the i<j half list (newton on) for n isolated atoms."""
    foff = np.arange(n + 1, dtype=np.int64) * (n - 1)
    fnb = np.array([j for i in range(n) for j in range(n) if j != i], dtype=np.int32)
    hrows = [[j for j in range(i + 1, n)] for i in range(n)]
    hoff = np.zeros(n + 1, dtype=np.int64)
    hoff[1:] = np.cumsum([len(r) for r in hrows])
    hnb = np.array([j for r in hrows for j in r], dtype=np.int32)
    return foff, fnb, hoff, hnb


def table(v):
    t = np.zeros((3, 3))
    t[1:, 1:] = v
    return t


def test_sph_rhosum_multiphase_kat(po):
    """sph_rhosum_multiphase.mac: rho_i = sum_j m_i w(x_i - x_j) (self term included)."""
    want = np.array([sum(M3[i] * w(np.linalg.norm(X3[i] - X3[j]), H) for j in range(3))
                     for i in range(3)])
    foff, fnb, _, _ = lists(3)
    cut = table(H)
    rho = np.ones(3)
    po.lib().orc_rhosum_multiphase(3, 3, np.ascontiguousarray(X3), T3, 2, M3, cut, cut * cut,
                                   foff, fnb, rho)
    assert np.allclose(rho, want, rtol=1e-13, atol=0)


def test_sph_taitwater_multiphase_kat(po):
    """sph_taitwater_multiphase.mac: gamma 1, c 1, eta 0, rbackground 0.5, rho0 1;
    F_i = sum_j -(V_i^2+V_j^2) p~_ij dw(x_i-x_j),  p~ = (rho_j P_i + rho_i P_j)/(rho_i+rho_j)."""
    gamma, c, rbg, rho0 = 1.0, 1.0, 0.5, 1.0
    rho = np.ones(3)
    B = c * c * rho0 / gamma
    P = B * (rho / rho0) ** gamma - rbg
    V = M3 / rho
    want = np.zeros((3, 3))
    for i in range(3):
        for j in range(3):
            if i == j:
                continue
            d = X3[i] - X3[j]
            r = np.linalg.norm(d)
            pij = (rho[j] * P[i] + rho[i] * P[j]) / (rho[i] + rho[j])
            want[i] += -(V[i] ** 2 + V[j] ** 2) * pij * d / r * dw(r, H)
    _, _, hoff, hnb = lists(3)
    cut = table(H)
    f = np.zeros((3, 3))
    t = np.array([0.0, 1.0, 1.0])
    po.lib().orc_taitwater_multiphase(3, 3, 1, np.ascontiguousarray(X3), np.zeros((3, 3)), rho,
                                      T3, 2, M3, t * rho0, t * c, t * B, t * gamma, t * rbg,
                                      table(0.0), cut, cut * cut, hoff, hnb, f)
    assert np.allclose(f, want, rtol=1e-12, atol=1e-14 * np.abs(want).max())


def test_heatconduction_phase_change_kat(po):
    """heatconduction_phase_change.mac: 2 atoms, E=(1,2), cv=(3,1), m=(1,2), rho=1, k=1;
    dE_i = sum_j 4 m_j/(rho_i rho_j) k_i k_j/(k_i+k_j) (T_i - T_j) dw(r)/r."""
    x = np.array([[5, 5, 5], [5.6, 5, 5]], dtype=np.float64)
    t = np.array([1, 2], dtype=np.int32)
    e = np.array([1.0, 2.0])
    cv = np.array([3.0, 1.0])
    m = np.array([1.0, 2.0])
    rho = np.ones(2)
    T = e / cv
    r = 0.6
    want = np.array([4 * m[1] * 0.5 * (T[0] - T[1]) * dw(r, H) / r,
                     4 * m[0] * 0.5 * (T[1] - T[0]) * dw(r, H) / r])
    _, _, hoff, hnb = lists(2)
    cut = table(H)
    de = np.zeros(2)
    po.lib().orc_heatconduction_phasechange(3, 2, 1, x, e, cv, rho, m, t, 2, table(1.0), None,
                                            None, cut, cut * cut, hoff, hnb, de)
    assert np.allclose(de, want, rtol=1e-12, atol=0)


def test_colorgradient_kat(po):
    """colorgradient.mac: |dC_i| with dC_i = sum_{j: type_j != type_i} sigma_i/sigma_j^2
    dw(x_i - x_j), sigma = rho/m; alpha(1,2) = 1, alpha(1,1) = alpha(2,2) = 0."""
    rho = np.ones(3)
    sig = rho / M3
    want = np.zeros((3, 3))
    for i in range(3):
        for j in range(3):
            if i == j or T3[i] == T3[j]:
                continue
            d = X3[i] - X3[j]
            r = np.linalg.norm(d)
            want[i] += sig[i] / sig[j] ** 2 * d / r * dw(r, H)
    foff, fnb, _, _ = lists(3)
    cut = table(H)
    alpha = np.zeros((3, 3))
    alpha[1, 2] = alpha[2, 1] = 1.0
    cg = np.zeros((3, 3))
    po.lib().orc_colorgradient(3, 3, np.ascontiguousarray(X3), rho, M3, T3, 2, alpha, cut,
                               cut * cut, foff, fnb, cg)
    # the script prints |dC_i| for i = 1, 2
    got = np.linalg.norm(cg, axis=1)
    assert np.allclose(got[:2], np.linalg.norm(want, axis=1)[:2], rtol=1e-12, atol=0)


def test_surfacetension_kat(po):
    """surfacetension.mac (with surfacetension.lmp): 3 atoms, m = rho = 1, types (1, 2, 2),
    h = 1, colorgradient alpha(1,2) = 1.  dC_i = sum_{j: type_j != type_i}
    sigma_i (C_l(i)/sigma_i^2 + C_l(j)/sigma_j^2) dw(x_i - x_j);
    Pm_i = (|dC_i|^2/3 I - dC_i dC_i^T)/|dC_i|;
    Fs_i = sum_{j != i} alpha(k,l) dw(x_i - x_j) . (Pm_i/sigma_i^2 + Pm_j/sigma_j^2).
    The script prints Fs[1] (atom 1's neighbours are both of the other type, so the
    alpha(k,l) factor of the .mac is 1 for every pair the LAMMPS style sums for it); Pm is
    even in dC, so the colorgradient's sign convention does not enter."""
    X = np.array([[4.6, 5.3, 5.0], [5.5, 5.0, 5.2], [5.0, 5.0, 5.0]])
    T = np.array([1, 2, 2], dtype=np.int32)
    m = np.ones(3)
    rho = np.ones(3)
    sig = rho / m

    def dwv(d):
        r = np.linalg.norm(d)
        return d / r * dw(r, H)

    dC = np.zeros((3, 3))
    for i in range(3):
        for j in range(3):
            if i != j and T[i] != T[j]:
                dC[i] += sig[i] * (0.0 / sig[i] ** 2 + 1.0 / sig[j] ** 2) * dwv(X[i] - X[j])
    Pm = [(np.dot(c, c) / 3 * np.eye(3) - np.outer(c, c)) / np.linalg.norm(c) for c in dC]
    want1 = sum(dwv(X[0] - X[j]) @ (Pm[0] / sig[0] ** 2 + Pm[j] / sig[j] ** 2) for j in (1, 2))
    # the LAMMPS side: colorgradient (full list) then surfacetension (half list, newton on)
    foff, fnb, hoff, hnb = lists(3)
    cut = table(H)
    alpha = np.zeros((3, 3))
    alpha[1, 2] = alpha[2, 1] = 1.0
    cg = np.zeros((3, 3))
    L = po.lib()
    L.orc_colorgradient(3, 3, np.ascontiguousarray(X), rho, m, T, 2, alpha, cut, cut * cut,
                        foff, fnb, cg)
    # (atom 2's gradient is a near-cancellation ~1e-5 of atom 1's: normwise bar)
    assert np.allclose(np.abs(cg), np.abs(dC), rtol=0, atol=1e-12 * np.abs(dC).max())
    f = np.zeros((3, 3))
    L.orc_surfacetension(3, 3, 1, np.ascontiguousarray(X), rho, m, T, 2, cg, cut, cut * cut,
                         hoff, hnb, f)
    assert np.allclose(f[0], want1, rtol=1e-12, atol=1e-14 * np.abs(want1).max())
