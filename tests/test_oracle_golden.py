"""Pin the CPU restatement (oracle/sph_oracle.c) to the reference.

* golden vectors (tests/golden/*.npz, written by make_golden.py from the reference's own
  compute code in oracle/_ref): list membership per row, half-list derivation (order
  included), rho, f, drho, de, colour gradient and quintic kernels must come out
  bit-identical from the restatement;
* where oracle/_ref exists (this container), the same comparison on fresh seeds.
"""
import glob
import os

import numpy as np
import pytest

import pyoracle as po
from scenarios import c2_system, c3_system, prepared

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SINGLE = ["c2_n6", "c2_n7_h2.2", "c3_n6", "c2_2d_n14"]


def load(name):
    return dict(np.load(os.path.join(GOLD, name + ".npz")))


def ghosted(d):
    return po.Ghosted(int(d["nlocal"]), int(d["nghost"]), np.ascontiguousarray(d["x"]),
                      np.ascontiguousarray(d["type"]), d.get("owner"), d.get("image"))


def test_golden_files_present():
    have = {os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "*.npz"))}
    assert set(SINGLE + ["multiphase_n5", "quintic"]) <= have


@pytest.mark.parametrize("name", SINGLE)
def test_borders_match_fixture(po, name):
    """The restated CommBrick::borders yields the ghost set the fixture was built on."""
    d = load(name)
    dim = int(d["dim"])
    s = po.System(dim, d["boxlo"], d["boxhi"], tuple(int(p) for p in d["periodic"]),
                  d["x"][:int(d["nlocal"])].copy(), np.zeros((int(d["nlocal"]), 3)),
                  d["type"][:int(d["nlocal"])].copy(), np.zeros(int(d["nlocal"])),
                  np.zeros(int(d["nlocal"])), np.zeros(int(d["nlocal"])), int(d["ntypes"]),
                  d["mass"])
    g = po.borders(s, float(d["cutghost"]))
    assert g.nghost == int(d["nghost"])
    assert np.array_equal(g.x, d["x"])
    assert np.array_equal(g.owner, d["owner"])


@pytest.mark.parametrize("name", SINGLE)
def test_neighbor_lists_bit_exact(po, name):
    d = load(name)
    g = ghosted(d)
    foff, fnb = po.neigh_full(int(d["dim"]), g, int(d["ntypes"]), d["cutneighsq"])
    # same members per row, bit-exact (the restatement bins differently from
    # Neighbor::bin_atoms, so the order inside a row may differ -- see DESIGN.md)
    assert np.array_equal(foff, d["full_off"])
    assert np.array_equal(sorted_rows(foff, fnb), sorted_rows(foff, d["full_nbr"]))
    # half_from_full_newton keeps the full list's order: on the reference's full list the
    # restatement must reproduce the reference's half list exactly, order included
    hoff, hnb = po.half_from_full(g, d["full_off"], d["full_nbr"])
    assert np.array_equal(hoff, d["half_off"])
    assert np.array_equal(hnb, d["half_nbr"])


def sorted_rows(off, nb):
    out = nb.copy()
    for i in range(off.size - 1):
        out[off[i]:off[i + 1]].sort()
    return out


@pytest.mark.parametrize("name", SINGLE)
def test_oracle_own_lists_match_golden(po, name):
    """End to end through the restatement's own lists: equal up to summation order."""
    d = load(name)
    g = ghosted(d)
    dim, nt = int(d["dim"]), int(d["ntypes"])
    foff, fnb = po.neigh_full(dim, g, nt, d["cutneighsq"])
    hoff, hnb = po.half_from_full(g, foff, fnb)
    if "out_rho" in d:
        rho = po.rhosum(dim, g, nt, d["mass"], d["rhosum_cut"], foff, fnb)
        assert np.abs(rho - d["out_rho"]).max() <= 1e-14 * np.abs(d["out_rho"]).max()
    if "out_f" in d:
        f, drho, de = po.taitwater(dim, g, nt, 1, d["vest"], d["rho"], d["mass"], d["rho0"],
                                   d["c0"], d["visc"], d["tait_cut"], hoff, hnb,
                                   morris=bool(d["morris"]))
        for a, b in ((f, d["out_f"]), (drho, d["out_drho"]), (de, d["out_de_tait"])):
            assert np.abs(a - b).max() <= 1e-13 * np.abs(b).max()


@pytest.mark.parametrize("name", SINGLE)
def test_pair_styles_bit_exact(po, name):
    d = load(name)
    g = ghosted(d)
    dim, nt = int(d["dim"]), int(d["ntypes"])
    if "out_rho" in d:
        rho = po.rhosum(dim, g, nt, d["mass"], d["rhosum_cut"], d["full_off"], d["full_nbr"])
        assert np.array_equal(rho, d["out_rho"])
    if "out_f" in d:
        f, drho, de = po.taitwater(dim, g, nt, 1, d["vest"], d["rho"], d["mass"], d["rho0"],
                                   d["c0"], d["visc"], d["tait_cut"], d["half_off"],
                                   d["half_nbr"], morris=bool(d["morris"]))
        assert np.array_equal(f, d["out_f"])
        assert np.array_equal(drho, d["out_drho"])
        assert np.array_equal(de, d["out_de_tait"])
    if "out_de_heat" in d:
        de = po.heatconduction(dim, g, nt, 1, d["e"], d["rho"], d["mass"], d["alpha"],
                               d["heat_cut"], d["half_off"], d["half_nbr"])
        assert np.array_equal(de, d["out_de_heat"])


def test_multiphase_bit_exact(po):
    d = load("multiphase_n5")
    L = po.lib()
    n, ng = int(d["nlocal"]), int(d["nghost"])
    nall = n + ng
    x, ty, rm = d["x"], d["type"], d["rmass"]
    cut = d["cut"]
    cutsq = cut * cut
    rho = d["rho"].copy()
    L.orc_rhosum_multiphase(3, n, x, ty, 2, rm, cut, cutsq, d["full_off"], d["full_nbr"], rho)
    assert np.array_equal(rho[:n], d["out_rho"])
    f = np.zeros((nall, 3))
    B = d["c0"] ** 2 * d["rho0"] / np.where(d["gamma"] > 0, d["gamma"], 1.0)
    L.orc_taitwater_multiphase(3, n, 1, x, d["vest"], d["rho"], ty, 2, rm, d["rho0"], d["c0"],
                               B, d["gamma"], d["rbg"], d["visc"], cut, cutsq, d["half_off"],
                               d["half_nbr"], f)
    assert np.array_equal(f, d["out_f"])
    de = np.zeros(nall)
    # the fixture holds coeff()'s upper triangle; init_one mirrors it
    # (pair_sph_heatconduction_phasechange.cpp:231-240), the restatement takes full tables
    ff = np.ascontiguousarray(np.triu(d["fixflag"]) + np.triu(d["fixflag"], 1).T, dtype=np.int32)
    tc = np.ascontiguousarray(np.triu(d["tc"]) + np.triu(d["tc"], 1).T)
    L.orc_heatconduction_phasechange(3, n, 1, x, d["e"], d["cv"], d["rho"], rm, ty, 2,
                                     d["alpha"], ff.ctypes.data, tc.ctypes.data, cut, cutsq,
                                     d["half_off"], d["half_nbr"], de)
    assert np.array_equal(de, d["out_de"])
    cg = np.zeros((nall, 3))
    L.orc_colorgradient(3, n, x, d["rho"], rm, ty, 2, d["cg_alpha"], cut, cutsq, d["full_off"],
                        d["full_nbr"], cg)
    assert np.array_equal(cg[:n], d["out_cg"])
    # surfacetension (half list, Newton-3 onto owned and ghost j)
    st_cut = d["st_cut"]
    f = np.zeros((nall, 3))
    L.orc_surfacetension(3, n, 1, x, d["rho"], rm, ty, 2, d["cg_all"], st_cut, st_cut * st_cut,
                         d["half_off"], d["half_nbr"], f)
    assert np.array_equal(f, d["out_f_st"])


def test_quintic_kernels(po):
    d = load("quintic")
    L = po.lib()
    for fn in ("kernel_quintic2d", "kernel_quintic3d", "dw_quintic2d", "dw_quintic3d"):
        got = np.array([getattr(L, "orc_" + fn)(float(r)) for r in d["r"]])
        assert np.array_equal(got, d[fn]), fn


# ---- against the live reference build (this container only) ---------------------------
@pytest.mark.ref
@pytest.mark.parametrize("case", ["c2", "c3", "2d", "nonperiodic"])
def test_oracle_vs_reference_fresh_seed(po, ref, case):
    if case == "c2":
        s, ph = c2_system(7, seed=777), po.c2_physics()
    elif case == "c3":
        s, ph = c3_system(7, seed=778), po.c3_physics()
    elif case == "2d":
        s, ph = c2_system(16, seed=779, dim=2), po.c2_physics(2.0)
    else:
        s, ph = c2_system(8, seed=780), po.c2_physics(2.5)
        s.periodic = (0, 1, 0)
        s.boxlo = s.boxlo - 1.5
        s.boxhi = s.boxhi + 1.5
    P = prepared(s, ph)
    g = P["g"]
    nt = s.ntypes
    off = np.zeros(g.nlocal + 1, dtype=np.int64)
    args = (s.dim, nt, g.nlocal, g.nghost, np.ascontiguousarray(g.x), g.type, s.boxlo, s.boxhi,
            s.boxlo, s.boxhi, P["cmax"], np.ascontiguousarray(P["cns"]))
    tot = ref.ref_neigh_full(*args, off, None, 0)
    nb = np.zeros(max(tot, 1), dtype=np.int32)
    ref.ref_neigh_full(*args, off, nb.ctypes.data, tot)
    assert np.array_equal(off, P["foff"])
    assert np.array_equal(sorted_rows(off, nb[:tot]), sorted_rows(off, P["fnb"]))
    if ph.rhosum_nstep:
        rr = P["rho_all"].copy()
        ref.ref_rhosum(s.dim, nt, g.nlocal, g.nghost, g.x, g.type, s.mass,
                       np.ascontiguousarray(ph.rhosum_cut), P["foff"], P["fnb"], rr)
        ro = po.rhosum(s.dim, g, nt, s.mass, ph.rhosum_cut, P["foff"], P["fnb"])
        assert np.array_equal(rr[:g.nlocal], ro)
    f = np.zeros((g.nall, 3))
    drho = np.zeros(g.nall)
    de = np.zeros(g.nall)
    fn = ref.ref_taitwater_morris if ph.morris else ref.ref_taitwater
    fn(s.dim, nt, g.nlocal, g.nghost, 1, g.x, P["vest_all"], P["rho_all"], g.type, s.mass,
       ph.rho0, ph.c0, np.ascontiguousarray(ph.visc), np.ascontiguousarray(ph.tait_cut),
       P["hoff"], P["hnb"], f, drho, de)
    fo, dro, deo = po.taitwater(s.dim, g, nt, 1, P["vest_all"], P["rho_all"], s.mass, ph.rho0,
                                ph.c0, ph.visc, ph.tait_cut, P["hoff"], P["hnb"],
                                morris=ph.morris)
    assert np.array_equal(f, fo) and np.array_equal(drho, dro) and np.array_equal(de, deo)


@pytest.mark.ref
@pytest.mark.parametrize("nx,dim", [(10, 3), (16, 2), (7, 3)])
def test_oracle_vs_reference_lattice_ties(po, ref, nx, dim):
    """On the C5 bubble lattice ~30 pairs per atom sit exactly at the cutoff (skin 0): the
    reference's Neighbor::full_bin keeps every one with rsq <= cutneighsq, and so must the
    restatement's builder (whose bins are a hair wider than the cutoff so that no such pair
    is ever two bins apart)."""
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import ref_full
    from scenarios import bubble_physics, bubble_system
    s = bubble_system(nx, dim=dim)
    ph = bubble_physics(nx, dim=dim)
    r = po.MpRefRun(s, ph)
    r.setup()
    foff, fnb = ref_full(ref, r.s, r.g, r.cns, r.cutneighmax)
    assert np.array_equal(foff, r.foff)
    assert np.array_equal(sorted_rows(foff, fnb), sorted_rows(r.foff, r.fnb))
