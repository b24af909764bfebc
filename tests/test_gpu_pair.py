"""GPU parity of the pair-style layer (sph_hip_* C ABI): the kernels run on LAMMPS-shaped
inputs (owned+ghost arrays and a NeighList) and must reproduce the reference loops
(pair_sph_rhosum.cpp:66-204, pair_sph_taitwater.cpp:53-200,
pair_sph_taitwater_morris.cpp:52-200, pair_sph_heatconduction.cpp:47-134) as restated in
oracle/sph_oracle.c.  Tolerance: 1e-10 normwise relative (BASELINE.json north_star);
the FULL-list path changes only the summation order, the HALF path adds atomic ordering."""
import copy

import numpy as np
import pytest

import pyoracle as po
from conftest import elem_rel_err, rel_err
from scenarios import c2_system, c3_system, oracle_forces, prepared

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _ctx(sph_amd, sysm, ph, P, newton=1):
    ctx = sph_amd.PairContext(sysm.dim, sysm.ntypes, newton)
    g = P["g"]
    ctx.atoms(g.nlocal, g.nghost, g.x, g.type, vest=P["vest_all"], rho=P["rho_all"], e=P["e_all"])
    if ph.rhosum_nstep > 0:
        ctx.rhosum_coeff(ph.rhosum_cut, sysm.mass)
    if ph.tait:
        ctx.taitwater_coeff(ph.rho0, ph.c0, ph.c0 * ph.c0 * ph.rho0 / 7.0, ph.visc, ph.tait_cut,
                            sysm.mass, morris=ph.morris)
    if ph.heat:
        ctx.heatconduction_coeff(ph.alpha, ph.heat_cut, sysm.mass)
    return ctx


@pytest.mark.parametrize("dim", [3, 2])
def test_rhosum_full_list(gpu, sph_amd, dim):
    s = c2_system(8 if dim == 3 else 24, dim=dim)
    ph = po.c2_physics(3.0)
    P = prepared(s, ph)
    ctx = _ctx(sph_amd, s, ph, P)
    ctx.list_csr(sph_amd.SPH_LIST_FULL, P["foff"], P["fnb"])
    rho = ctx.rhosum(np.zeros(P["g"].nall))[:s.n]
    want = po.rhosum(dim, P["g"], 1, s.mass, ph.rhosum_cut, P["foff"], P["fnb"])
    assert rel_err(rho, want) < 1e-13
    assert elem_rel_err(rho, want) < 1e-13


@pytest.mark.parametrize("dim", [3, 2])
def test_taitwater_full_list(gpu, sph_amd, dim):
    s = c2_system(8 if dim == 3 else 24, dim=dim)
    ph = po.c2_physics(3.0)
    P = prepared(s, ph)
    ctx = _ctx(sph_amd, s, ph, P)
    ctx.list_csr(sph_amd.SPH_LIST_FULL, P["foff"], P["fnb"])
    nall = P["g"].nall
    f, drho, de = np.zeros((nall, 3)), np.zeros(nall), np.zeros(nall)
    ctx.taitwater(f, drho, de)
    wf, wd, we = oracle_forces(s, ph, P)
    n = s.n
    assert rel_err(f[:n], wf[:n]) < TOL
    assert rel_err(drho[:n], wd[:n]) < TOL
    assert rel_err(de[:n], we[:n]) < TOL
    # full list: ghosts untouched
    assert not f[n:].any() and not drho[n:].any() and not de[n:].any()


def test_taitwater_half_list_newton_scatter(gpu, sph_amd):
    """HALF list (LAMMPS' default request): ghosts receive their Newton-3 share exactly as
    in the reference, before reverse comm."""
    s = c2_system(8)
    ph = po.c2_physics(3.0)
    P = prepared(s, ph)
    ctx = _ctx(sph_amd, s, ph, P)
    ctx.list_csr(sph_amd.SPH_LIST_HALF, P["hoff"], P["hnb"])
    nall = P["g"].nall
    f, drho, de = np.zeros((nall, 3)), np.zeros(nall), np.zeros(nall)
    vir = np.zeros(6)
    ctx.taitwater(f, drho, de, virial=vir)
    wf, wd, we = oracle_forces(s, ph, P, reverse=False)
    assert rel_err(f, wf) < TOL
    assert rel_err(drho, wd) < TOL
    assert rel_err(de, we) < TOL
    _, _, _, wvir = po.taitwater(3, P["g"], 1, 1, P["vest_all"], P["rho_all"], s.mass, ph.rho0,
                                 ph.c0, ph.visc, ph.tait_cut, P["hoff"], P["hnb"], virial=True)
    assert rel_err(vir, wvir) < TOL


def test_morris_heat_two_types(gpu, sph_amd):
    s = c3_system(8)
    ph = po.c3_physics(3.0)
    P = prepared(s, ph)
    ctx = _ctx(sph_amd, s, ph, P)
    ctx.list_csr(sph_amd.SPH_LIST_FULL, P["foff"], P["fnb"])
    nall = P["g"].nall
    f, drho, de = np.zeros((nall, 3)), np.zeros(nall), np.zeros(nall)
    ctx.taitwater(f, drho, de)
    ctx.heatconduction(de)
    wf, wd, we = oracle_forces(s, ph, P)
    n = s.n
    assert rel_err(f[:n], wf[:n]) < TOL
    assert rel_err(drho[:n], wd[:n]) < TOL
    assert rel_err(de[:n], we[:n]) < TOL


def test_heat_half_list(gpu, sph_amd):
    s = c3_system(7)
    ph = po.c3_physics(3.0)
    P = prepared(s, ph)
    ctx = _ctx(sph_amd, s, ph, P)
    ctx.list_csr(sph_amd.SPH_LIST_HALF, P["hoff"], P["hnb"])
    nall = P["g"].nall
    de = np.zeros(nall)
    ctx.heatconduction(de)
    want = po.heatconduction(3, P["g"], 2, 1, P["e_all"], P["rho_all"], s.mass, ph.alpha,
                             ph.heat_cut, P["hoff"], P["hnb"])
    assert rel_err(de, want) < TOL


def test_lammps_neighlist_form(gpu, sph_amd):
    """sph_hip_list with ilist/numneigh/firstneigh (+ NEIGHMASK bits set) == CSR path."""
    s = c2_system(6)
    ph = po.c2_physics(3.0)
    P = prepared(s, ph)
    foff, fnb = P["foff"], P["fnb"]
    n = s.n
    ilist = np.arange(n - 1, -1, -1, dtype=np.int32)  # non-identity ilist
    numneigh = np.diff(foff).astype(np.int32)
    rows = [(fnb[foff[i]:foff[i + 1]] | (1 << 30)).astype(np.int32) for i in range(n)]
    ctx = _ctx(sph_amd, s, ph, P)
    ctx.list_lammps(sph_amd.SPH_LIST_FULL, ilist, numneigh, rows)
    rho = ctx.rhosum(np.zeros(P["g"].nall))[:n]
    want = po.rhosum(3, P["g"], 1, s.mass, ph.rhosum_cut, foff, fnb)
    assert rel_err(rho, want) < 1e-13


def test_edge_cases(gpu, sph_amd):
    ph = po.c2_physics(3.0)
    ctx = sph_amd.PairContext(3, 1, 1)
    # empty system
    ctx.atoms(0, 0, np.zeros((0, 3)), np.zeros(0, np.int32))
    ctx.rhosum_coeff(ph.rhosum_cut, np.array([0.0, 1.0]))
    ctx.list_csr(sph_amd.SPH_LIST_FULL, np.zeros(1, np.int64), np.zeros(0, np.int32))
    ctx.rhosum(np.zeros(1))
    # isolated atoms: rho = self term only, zero forces
    x = np.array([[0.0, 0.0, 0.0], [50.0, 0.0, 0.0]])
    ctx.atoms(2, 0, x, np.ones(2, np.int32), vest=np.zeros((2, 3)), rho=np.ones(2), e=np.zeros(2))
    ctx.list_csr(sph_amd.SPH_LIST_FULL, np.zeros(3, np.int64), np.zeros(0, np.int32))
    rho = ctx.rhosum(np.zeros(2))
    assert np.allclose(rho, 2.1541870227086614782 / 27.0, rtol=1e-15)
    # bad inputs fail loudly with EINVAL
    with pytest.raises(sph_amd.HipError) as ei:
        ctx.atoms(1, 0, np.zeros((1, 3)), np.array([5], np.int32))
    assert ei.value.code == -1
    with pytest.raises(sph_amd.HipError):
        ctx.list_csr(sph_amd.SPH_LIST_FULL, np.array([0, 1], np.int64), np.array([7], np.int32))


def test_keyed_list_reuse(gpu, sph_amd):
    """sph_hip_list_keyed (the LAMMPS shim's call, key = neighbor->ncalls): a FULL and a HALF
    list of one build are both kept; calls with a known key skip the host rows entirely
    (corrupted rows give bit-identical results), a new key re-uploads, and restaging atoms
    with another ghost count drops every staged list (SURVEY 8(b) device mirrors)."""
    s = c2_system(6)
    ph = po.c2_physics(3.0)
    P = prepared(s, ph)
    n, nall = s.n, P["g"].nall

    def rows_of(off, nb, bad=False):
        numneigh = np.diff(off).astype(np.int32)
        rows = [np.zeros(int(numneigh[i]), np.int32) if bad else nb[off[i]:off[i + 1]].astype(np.int32)
                for i in range(n)]
        return np.arange(n, dtype=np.int32), numneigh, rows

    def rho_full(key, bad=False):
        ctx.list_lammps(sph_amd.SPH_LIST_FULL, *rows_of(P["foff"], P["fnb"], bad), key=key)
        return ctx.rhosum(np.zeros(nall)).copy()

    def tait_half(key, bad=False):
        ctx.list_lammps(sph_amd.SPH_LIST_HALF, *rows_of(P["hoff"], P["hnb"], bad), key=key)
        f, drho, de = np.zeros((nall, 3)), np.zeros(nall), np.zeros(nall)
        ctx.taitwater(f, drho, de)
        return f

    ctx = _ctx(sph_amd, s, ph, P)
    rho1 = rho_full(5)
    f1 = tait_half(5)
    assert rel_err(rho1[:n], po.rhosum(3, P["g"], 1, s.mass, ph.rhosum_cut, P["foff"], P["fnb"])) < 1e-13
    wf, _, _ = oracle_forces(s, ph, P, reverse=False)
    assert rel_err(f1, wf) < TOL
    # same build: both kinds reused, the (corrupted) host rows are never read
    assert np.array_equal(rho_full(5, bad=True), rho1)
    assert np.array_equal(tait_half(5, bad=True), f1)
    # a new build re-uploads
    assert np.array_equal(rho_full(6), rho1)
    with pytest.raises(sph_amd.HipError):
        ctx.list_lammps(sph_amd.SPH_LIST_FULL, np.arange(n, dtype=np.int32),
                        np.ones(n, np.int32), [np.array([nall + 3], np.int32)] * n, key=7)
    # rho-only restage (the later computes of one step): equal to a full restage
    g = P["g"]
    rho2 = P["rho_all"] * (1.0 + 0.01 * np.sin(np.arange(nall)))
    ctx.atoms_rho(rho2)
    f_rho = tait_half(5)
    ref = sph_amd.PairContext(s.dim, s.ntypes, 1)
    ref.atoms(g.nlocal, g.nghost, g.x, g.type, vest=P["vest_all"], rho=rho2, e=P["e_all"])
    ref.taitwater_coeff(ph.rho0, ph.c0, ph.c0 * ph.c0 * ph.rho0 / 7.0, ph.visc, ph.tait_cut,
                        s.mass, morris=ph.morris)
    ref.list_csr(sph_amd.SPH_LIST_HALF, P["hoff"], P["hnb"])
    f_ref, d_ref, e_ref = np.zeros((nall, 3)), np.zeros(nall), np.zeros(nall)
    ref.taitwater(f_ref, d_ref, e_ref)
    assert rel_err(f_rho, f_ref) < 1e-14 and not np.array_equal(f_rho, f1)
    ref.close()
    # another atom count drops the staged lists: a style call needs a restaged list
    ctx.atoms(g.nlocal, g.nghost - 1, g.x[:-1], g.type[:-1], vest=P["vest_all"][:-1],
              rho=P["rho_all"][:-1], e=P["e_all"][:-1])
    with pytest.raises(sph_amd.HipError):
        ctx.rhosum(np.zeros(nall))


@pytest.mark.parametrize("system,dim", [("c2", 3), ("c2", 2), ("c3", 3)])
def test_device_built_lists(gpu, sph_amd, system, dim):
    """sph_hip_build_list (the device-list path of the shim): from the staged owned + ghost
    atoms, the FULL list has Neighbor::full_bin's membership and the HALF list
    half_from_full_newton's -- row lengths bit-exact against the oracle's lists -- and the
    styles on them match the oracle (rhosum 1e-13; taitwater Newton-3 scatter incl. the
    ghosts' shares, heat conduction 1e-10)."""
    s = (c2_system(8 if dim == 3 else 24, dim=dim) if system == "c2" else c3_system(8))
    ph = po.c2_physics(3.0) if system == "c2" else po.c3_physics(3.0)
    P = prepared(s, ph)
    g, n, nall = P["g"], s.n, P["g"].nall
    cns = np.asarray(P["cns"], dtype=np.float64).reshape(s.ntypes + 1, s.ntypes + 1)
    ctx = _ctx(sph_amd, s, ph, P)
    ctx.build_list(sph_amd.SPH_LIST_FULL, cns, key=1)
    assert np.array_equal(ctx.numneigh(n), np.diff(P["foff"]).astype(np.int32))
    if ph.rhosum_nstep > 0:
        rho = ctx.rhosum(np.zeros(nall))[:n]
        want = po.rhosum(dim, g, s.ntypes, s.mass, ph.rhosum_cut, P["foff"], P["fnb"])
        assert rel_err(rho, want) < 1e-13
    ctx.build_list(sph_amd.SPH_LIST_HALF, cns, key=1)
    assert np.array_equal(ctx.numneigh(n), np.diff(P["hoff"]).astype(np.int32))
    f, drho, de = np.zeros((nall, 3)), np.zeros(nall), np.zeros(nall)
    ctx.taitwater(f, drho, de)
    if ph.heat:
        ctx.heatconduction(de)
    wf, wd, we = oracle_forces(s, ph, P, reverse=False)
    assert rel_err(f, wf) < TOL
    assert rel_err(drho, wd) < TOL
    assert rel_err(de, we) < TOL
    # the same key again: the staged device list is reused (no rebuild), same results
    ctx.build_list(sph_amd.SPH_LIST_HALF, cns, key=1)
    f2, d2, e2 = np.zeros((nall, 3)), np.zeros(nall), np.zeros(nall)
    ctx.taitwater(f2, d2, e2)
    assert rel_err(f2, wf) < TOL


def test_device_list_with_a_far_away_ghost(gpu, sph_amd):
    """A stray ghost far from the rank (here 1e4 box lengths along every axis) stretches the
    bounding box of the binned build past 2^26 half-size bins: the build coarsens the bins
    along the longest axes (membership unchanged) instead of failing; the owned rows are the
    oracle's, the stray ghost's row is never built (ghost) and it is nobody's neighbour."""
    s = c2_system(8)
    ph = po.c2_physics(3.0)
    P = prepared(s, ph)
    g, n = P["g"], s.n
    cns = np.asarray(P["cns"], dtype=np.float64).reshape(s.ntypes + 1, s.ntypes + 1)
    ctx = _ctx(sph_amd, s, ph, P)
    far = np.asarray(s.boxhi, dtype=np.float64) * 1.0e4
    x = np.concatenate([g.x, far[None, :]])
    ty = np.concatenate([g.type, g.type[:1]])
    ext = lambda a: np.concatenate([a, a[:1]])
    ctx.atoms(g.nlocal, g.nghost + 1, np.ascontiguousarray(x), ty, vest=ext(P["vest_all"]),
              rho=ext(P["rho_all"]), e=ext(P["e_all"]))
    ctx.build_list(sph_amd.SPH_LIST_FULL, cns, key=7)
    assert np.array_equal(ctx.numneigh(n), np.diff(P["foff"]).astype(np.int32))
    rho = ctx.rhosum(np.zeros(g.nall + 1))[:n]
    want = po.rhosum(s.dim, g, s.ntypes, s.mass, ph.rhosum_cut, P["foff"], P["fnb"])
    assert rel_err(rho, want) < 1e-13


def test_mapped_host_arrays_and_update(gpu, sph_amd):
    """sph_hip_host_arrays (the shim registers LAMMPS' arrays): the staging kernels read x /
    vest / rho / e straight from mapped host memory, rhosum writes rho and taitwater / heat
    add f / drho / de in place -- the same results as the copy path, added (not assigned) to
    what the arrays held; sph_hip_atoms_update restages a moved atom set without types."""
    s = c3_system(8)
    ph = po.c3_physics(3.0)
    P = prepared(s, ph)
    g, n, nall = P["g"], s.n, P["g"].nall
    cns = np.asarray(P["cns"], dtype=np.float64)
    x = np.ascontiguousarray(g.x).copy()
    vest, rho, e = (np.ascontiguousarray(P[k]).copy() for k in ("vest_all", "rho_all", "e_all"))
    f, drho, de = np.full((nall, 3), 0.25), np.full(nall, -0.5), np.full(nall, 2.0)
    ctx = sph_amd.PairContext(3, 2, 1)
    ctx.host_arrays(nall, x=x, vest=vest, rho=rho, e=e, f=f, drho=drho, de=de)
    ctx.atoms(g.nlocal, g.nghost, x, g.type, vest=vest, rho=rho, e=e)
    ctx.taitwater_coeff(ph.rho0, ph.c0, ph.c0 * ph.c0 * ph.rho0 / 7.0, ph.visc, ph.tait_cut,
                        s.mass, morris=ph.morris)
    ctx.heatconduction_coeff(ph.alpha, ph.heat_cut, s.mass)
    ctx.build_list(sph_amd.SPH_LIST_HALF, cns, key=3)
    ctx.taitwater(f, drho, de)
    ctx.heatconduction(de)
    wf, wd, we = oracle_forces(s, ph, P, reverse=False)
    assert rel_err(f - 0.25, wf) < TOL
    assert rel_err(drho + 0.5, wd) < TOL
    assert rel_err(de - 2.0, we) < TOL
    # move the atoms (same set, ghosts too): update, rebuild the list, oracle on the moved set
    x += 0.01 * np.sin(np.arange(x.size)).reshape(x.shape)
    ctx.atoms_update(x, vest=vest, rho=rho, e=e)
    ctx.build_list(sph_amd.SPH_LIST_HALF, cns, key=4)
    f[:], drho[:], de[:] = 0.0, 0.0, 0.0
    ctx.taitwater(f, drho, de)
    g2 = copy.copy(g)
    g2.x = x
    foff, fnb = po.neigh_full(3, g2, s.ntypes, cns)
    hoff, hnb = po.half_from_full(g2, foff, fnb)
    assert np.array_equal(ctx.numneigh(n), np.diff(hoff).astype(np.int32))
    wf2, wd2, _ = po.taitwater(3, g2, s.ntypes, 1, vest, rho, s.mass, ph.rho0, ph.c0, ph.visc,
                               ph.tait_cut, hoff, hnb, morris=ph.morris,
                               B=ph.c0 * ph.c0 * ph.rho0 / 7.0)
    assert rel_err(f, wf2) < TOL
    assert rel_err(drho, wd2) < TOL
    ctx.host_arrays(0)
    ctx.close()


def test_device_lists_edge_cases(gpu, sph_amd):
    """sph_hip_build_list on an empty system, on isolated atoms (no neighbour, the self term
    only), with ghosts only beside one owned atom, and a key reused with another
    cutneighsq (rebuilt, not reused); a non-finite cutoff fails with EINVAL."""
    ph = po.c2_physics(3.0)
    mass = np.array([0.0, 1.0])
    cns = np.array([[0.0, 0.0], [0.0, 3.3 * 3.3]])
    ctx = sph_amd.PairContext(3, 1, 1)
    ctx.rhosum_coeff(ph.rhosum_cut, mass)
    ctx.atoms(0, 0, np.zeros((0, 3)), np.zeros(0, np.int32))
    ctx.build_list(sph_amd.SPH_LIST_FULL, cns, key=1)
    ctx.rhosum(np.zeros(1))
    # isolated atoms
    x = np.array([[0.0, 0.0, 0.0], [50.0, 0.0, 0.0]])
    ctx.atoms(2, 0, x, np.ones(2, np.int32), vest=np.zeros((2, 3)), rho=np.ones(2), e=np.zeros(2))
    ctx.build_list(sph_amd.SPH_LIST_FULL, cns, key=2)
    assert np.array_equal(ctx.numneigh(2), [0, 0])
    rho = ctx.rhosum(np.zeros(2))
    assert np.allclose(rho, 2.1541870227086614782 / 27.0, rtol=1e-15)
    # one owned atom, its neighbours all ghosts (owned rows only; ghosts are never rows)
    xg = np.array([[0.0, 0.0, 0.0], [1.0, 0.0, 0.0], [0.0, 2.0, 0.0], [0.0, 0.0, 3.2],
                   [3.0, 3.0, 0.0]])
    t = np.ones(5, np.int32)
    ctx.atoms(1, 4, xg, t, vest=np.zeros((5, 3)), rho=np.ones(5), e=np.zeros(5))
    ctx.build_list(sph_amd.SPH_LIST_FULL, cns, key=3)
    assert np.array_equal(ctx.numneigh(1), [3])      # 4.24 > 3.3 is out
    ctx.build_list(sph_amd.SPH_LIST_HALF, cns, key=3)
    assert np.array_equal(ctx.numneigh(1), [3])      # ghosts above in z / y / x all kept
    # the same key with another cutneighsq: built again
    ctx.build_list(sph_amd.SPH_LIST_FULL, cns * (1.5 / 3.3) ** 2, key=3)
    assert np.array_equal(ctx.numneigh(1), [1])
    with pytest.raises(sph_amd.HipError):
        ctx.build_list(sph_amd.SPH_LIST_FULL, np.array([[0.0, 0.0], [0.0, np.inf]]), key=4)
    ctx.close()
