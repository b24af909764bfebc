"""GPU parity of the multiphase styles (sph_hip_*_multiphase, _phasechange, colorgradient,
surfacetension):

* the golden vectors the reference's own code wrote (tests/golden/multiphase_n5.npz):
  rhosum/multiphase and colorgradient on the reference's full list, taitwater/multiphase,
  heatconduction/phasechange and surfacetension on its half list with newton on (ghost
  slots included);
* the oracle on a larger two-phase box (fresh seed), same lists;
* the 2-3 atom KAT geometries of examples/USER/sph/multiphase_two_atoms.
Tolerance 1e-10 normwise (north_star)."""
import os

import numpy as np
import pytest

import pyoracle as po
from conftest import rel_err
from scenarios import c3_system

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TOL = 1e-10


def mp_context(sph_amd, d):
    n, ng = int(d["nlocal"]), int(d["nghost"])
    ctx = sph_amd.PairContext(int(d["dim"]), int(d["ntypes"]), 1)
    ctx.atoms(n, ng, d["x"], d["type"], vest=d["vest"], rho=d["rho"], e=d["e"])
    ctx.atoms_multiphase(d["rmass"], d["cv"])
    return ctx


def test_golden_multiphase(gpu, sph_amd):
    d = dict(np.load(os.path.join(GOLD, "multiphase_n5.npz")))
    n, ng = int(d["nlocal"]), int(d["nghost"])
    nall = n + ng
    ctx = mp_context(sph_amd, d)
    ctx.list_csr(sph_amd.SPH_LIST_FULL, d["full_off"], d["full_nbr"])
    ctx.rhosum_multiphase_coeff(d["cut"])
    rho = ctx.rhosum_multiphase(np.zeros(nall))[:n]
    assert rel_err(rho, d["out_rho"]) < 1e-13
    ctx.colorgradient_coeff(d["cg_alpha"], d["cut"])
    cg = ctx.colorgradient(np.zeros((nall, 3)))[:n]
    assert rel_err(cg, d["out_cg"]) < TOL
    ctx.list_csr(sph_amd.SPH_LIST_HALF, d["half_off"], d["half_nbr"])
    ctx.taitwater_multiphase_coeff(d["rho0"], d["c0"], d["gamma"], d["rbg"], d["visc"], d["cut"])
    f = np.zeros((nall, 3))
    ctx.taitwater_multiphase(f)
    assert rel_err(f, d["out_f"]) < TOL
    ctx.heatconduction_phasechange_coeff(d["alpha"], d["cut"], fixflag=d["fixflag"], tc=d["tc"])
    de = np.zeros(nall)
    ctx.heatconduction_phasechange(de)
    assert rel_err(de, d["out_de"]) < TOL
    ctx.surfacetension_coeff(d["st_cut"])
    f = np.zeros((nall, 3))
    ctx.surfacetension(d["cg_all"], f)
    assert rel_err(f, d["out_f_st"]) < TOL


def two_phase(nside=8, seed=4321):
    s = c3_system(nside, seed=seed)
    nt = 2
    cut = np.zeros((3, 3))
    cut[1:, 1:] = 2.1
    cns, cmax = po.cutneighsq(nt, cut, 0.25)
    g = po.borders(s, cmax)
    foff, fnb = po.neigh_full(3, g, nt, cns)
    hoff, hnb = po.half_from_full(g, foff, fnb)
    rng = np.random.default_rng(seed)
    liq = s.type == 1
    own = dict(rmass=np.where(liq, 1.0, 0.1) * (1 + 0.05 * rng.uniform(-1, 1, s.n)),
               rho=np.where(liq, 1.0, 0.1) * (1 + 0.02 * rng.uniform(-1, 1, s.n)),
               e=np.where(liq, 0.04, 0.12) * (1 + 0.3 * rng.uniform(-1, 1, s.n)),
               cv=np.where(liq, 0.04, 0.06), vest=s.v + 0.05 * rng.normal(size=s.v.shape))
    d = {k: g.gather(v) for k, v in own.items()}
    d.update(dim=3, ntypes=nt, nlocal=g.nlocal, nghost=g.nghost, x=g.x, type=g.type, cut=cut,
             full_off=foff, full_nbr=fnb, half_off=hoff, half_nbr=hnb, owner=g.owner)
    return d


def test_multiphase_vs_oracle(gpu, sph_amd):
    d = two_phase()
    L = po.lib()
    n, nall = d["nlocal"], d["nlocal"] + d["nghost"]
    cut = d["cut"]
    ctx = mp_context(sph_amd, d)
    ctx.list_csr(sph_amd.SPH_LIST_FULL, d["full_off"], d["full_nbr"])
    ctx.rhosum_multiphase_coeff(cut)
    rho = ctx.rhosum_multiphase(np.zeros(nall))[:n]
    want = d["rho"].copy()
    L.orc_rhosum_multiphase(3, n, d["x"], d["type"], 2, d["rmass"], cut, cut * cut,
                            d["full_off"], d["full_nbr"], want)
    assert rel_err(rho, want[:n]) < 1e-13
    # unequal gamma: the reference's asymmetric p_j must be reproduced on the half list
    rho0 = np.array([0.0, 1.0, 0.1])
    c0 = np.array([0.0, 10.0, 8.0])
    gamma = np.array([0.0, 7.0, 1.4])
    rbg = np.array([0.0, 0.5, 0.2])
    visc = np.zeros((3, 3))
    visc[1:, 1:] = 0.05
    ctx.list_csr(sph_amd.SPH_LIST_HALF, d["half_off"], d["half_nbr"])
    ctx.taitwater_multiphase_coeff(rho0, c0, gamma, rbg, visc, cut)
    f = np.zeros((nall, 3))
    ctx.taitwater_multiphase(f)
    fw = np.zeros((nall, 3))
    L.orc_taitwater_multiphase(3, n, 1, d["x"], d["vest"], d["rho"], d["type"], 2, d["rmass"],
                               rho0, c0, c0 ** 2 * rho0 / np.where(gamma > 0, gamma, 1), gamma,
                               rbg, visc, cut, cut * cut, d["half_off"], d["half_nbr"], fw)
    assert rel_err(f, fw) < TOL
    alpha = np.zeros((3, 3))
    alpha[1:, 1:] = 0.1
    ff = np.zeros((3, 3), dtype=np.int32)
    ff[1, 2] = ff[2, 1] = 2
    tc = np.zeros((3, 3))
    tc[1, 2] = tc[2, 1] = 2.5
    ctx.heatconduction_phasechange_coeff(alpha, cut, fixflag=ff, tc=tc)
    de = np.zeros(nall)
    ctx.heatconduction_phasechange(de)
    dw = np.zeros(nall)
    L.orc_heatconduction_phasechange(3, n, 1, d["x"], d["e"], d["cv"], d["rho"], d["rmass"],
                                     d["type"], 2, alpha, ff.ctypes.data, tc.ctypes.data, cut,
                                     cut * cut, d["half_off"], d["half_nbr"], dw)
    assert rel_err(de, dw) < TOL
    # surfacetension: colorgradient of every atom (ghosts copy their owner), half list
    cga = np.zeros((3, 3))
    cga[1, 2] = cga[2, 1] = 1.0
    cg = np.zeros((nall, 3))
    L.orc_colorgradient(3, n, d["x"], d["rho"], d["rmass"], d["type"], 2, cga, cut, cut * cut,
                        d["full_off"], d["full_nbr"], cg)
    cg_all = np.ascontiguousarray(np.concatenate([cg[:n], cg[:n][d["owner"]]]))
    ctx.surfacetension_coeff(cut)
    f = np.zeros((nall, 3))
    ctx.surfacetension(cg_all, f)
    fw = np.zeros((nall, 3))
    L.orc_surfacetension(3, n, 1, d["x"], d["rho"], d["rmass"], d["type"], 2, cg_all, cut,
                         cut * cut, d["half_off"], d["half_nbr"], fw)
    assert rel_err(f, fw) < TOL
    # ... and on the full list (gather only, owned rows) = the half-list result with the
    # ghost slots folded into their owners (reverse comm; the pair force is antisymmetric)
    ctx.list_csr(sph_amd.SPH_LIST_FULL, d["full_off"], d["full_nbr"])
    f = np.zeros((nall, 3))
    ctx.surfacetension(cg_all, f)
    want = fw[:n].copy()
    np.add.at(want, d["owner"], fw[n:])
    assert rel_err(f[:n], want) < TOL


def test_kat_geometry(gpu, sph_amd):
    """multiphase_two_atoms: 3 isolated atoms (no ghosts), h = 1."""
    x = np.array([[5, 5, 5], [5.5, 5, 5], [5, 5, 4.8]], dtype=np.float64)
    t = np.array([1, 2, 2], dtype=np.int32)
    m = np.array([2.0, 1.0, 1.0])
    off = np.array([0, 2, 4, 6], dtype=np.int64)
    nb = np.array([1, 2, 0, 2, 0, 1], dtype=np.int32)
    cut = np.zeros((3, 3))
    cut[1:, 1:] = 1.0
    ctx = sph_amd.PairContext(3, 2, 1)
    ctx.atoms(3, 0, x, t, vest=np.zeros((3, 3)), rho=np.ones(3), e=np.zeros(3))
    ctx.atoms_multiphase(m, np.ones(3))
    ctx.list_csr(sph_amd.SPH_LIST_FULL, off, nb)
    ctx.rhosum_multiphase_coeff(cut)
    rho = ctx.rhosum_multiphase(np.zeros(3))
    want = np.ones(3)
    po.lib().orc_rhosum_multiphase(3, 3, x, t, 2, m, cut, cut * cut, off, nb, want)
    assert rel_err(rho, want) < 1e-13
