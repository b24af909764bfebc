"""Generate the golden vectors in tests/golden/*.npz from the REFERENCE's own compute code.

The generator drives oracle/_ref/libsph_ref.so -- the USER-SPH pair styles and the
Neighbor::full_bin / half_from_full_newton builders compiled from /root/reference/src by
oracle/build_ref.sh -- on small jittered-lattice systems, and stores inputs and outputs as
plain arrays (np.savez_compressed, no pickles).  Only the ghost atoms themselves come from
the C restatement (orc_borders, CommBrick::borders semantics), because the harness runs the
reference with nswap = 0; every number that the GPU path must reproduce -- list membership
and order, rho, f, drho, de, colour gradient -- is produced by reference code.

Run here (where /root/reference exists):  python tests/golden/make_golden.py
The fixtures are small (a few hundred owned atoms) and are committed; the tests that use
them never touch /root/reference.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pyoracle as po  # noqa: E402
from scenarios import c2_system, c3_system, prepared  # noqa: E402


def ref_full(R, s, g, cns, cmax):
    nt = s.ntypes
    off = np.zeros(g.nlocal + 1, dtype=np.int64)
    args = (s.dim, nt, g.nlocal, g.nghost, np.ascontiguousarray(g.x), g.type, s.boxlo, s.boxhi,
            s.boxlo, s.boxhi, cmax, np.ascontiguousarray(cns))
    tot = R.ref_neigh_full(*args, off, None, 0)
    nb = np.zeros(max(tot, 1), dtype=np.int32)
    assert R.ref_neigh_full(*args, off, nb.ctypes.data, tot) == tot
    return off, nb[:tot]


def ref_half(R, g, foff, fnb):
    hoff = np.zeros(g.nlocal + 1, dtype=np.int64)
    fn = fnb if fnb.size else np.zeros(1, np.int32)
    tot = R.ref_neigh_half_from_full(g.nlocal, g.nghost, np.ascontiguousarray(g.x), foff, fn,
                                     hoff, None)
    hn = np.zeros(max(tot, 1), dtype=np.int32)
    R.ref_neigh_half_from_full(g.nlocal, g.nghost, np.ascontiguousarray(g.x), foff, fn, hoff,
                               hn.ctypes.data)
    return hoff, hn[:tot]


def nz(a):
    return a if a.size else np.zeros(1, dtype=a.dtype)


def single_phase_case(name, s, ph, out):
    R = po.ref()
    P = prepared(s, ph)
    g = P["g"]
    nt = s.ntypes
    foff, fnb = ref_full(R, s, g, P["cns"], P["cmax"])
    hoff, hnb = ref_half(R, g, foff, fnb)
    d = dict(dim=s.dim, ntypes=nt, nlocal=g.nlocal, nghost=g.nghost, boxlo=s.boxlo,
             boxhi=s.boxhi, periodic=np.array(s.periodic, np.int32), skin=ph.skin,
             mass=s.mass, cutneighsq=P["cns"], cutghost=P["cmax"], x=g.x, type=g.type,
             owner=g.owner, image=g.image, vest=P["vest_all"], rho=P["rho_all"], e=P["e_all"],
             full_off=foff, full_nbr=fnb, half_off=hoff, half_nbr=hnb)
    if ph.rhosum_nstep > 0:
        rc = np.ascontiguousarray(ph.rhosum_cut, dtype=np.float64)
        rho = P["rho_all"].copy()
        R.ref_rhosum(s.dim, nt, g.nlocal, g.nghost, g.x, g.type, s.mass, rc, foff, nz(fnb), rho)
        d.update(rhosum_cut=rc, out_rho=rho[:g.nlocal])
    if ph.tait:
        f = np.zeros((g.nall, 3))
        drho = np.zeros(g.nall)
        de = np.zeros(g.nall)
        fn = R.ref_taitwater_morris if ph.morris else R.ref_taitwater
        visc = np.ascontiguousarray(ph.visc, dtype=np.float64)
        cut = np.ascontiguousarray(ph.tait_cut, dtype=np.float64)
        fn(s.dim, nt, g.nlocal, g.nghost, 1, g.x, P["vest_all"], P["rho_all"], g.type, s.mass,
           ph.rho0, ph.c0, visc, cut, hoff, nz(hnb), f, drho, de)
        d.update(morris=int(ph.morris), rho0=ph.rho0, c0=ph.c0, visc=visc, tait_cut=cut,
                 out_f=f, out_drho=drho, out_de_tait=de)
    if ph.heat:
        de = np.zeros(g.nall)
        alpha = np.ascontiguousarray(ph.alpha, dtype=np.float64)
        cut = np.ascontiguousarray(ph.heat_cut, dtype=np.float64)
        R.ref_heatconduction(s.dim, nt, g.nlocal, g.nghost, 1, g.x, P["e_all"], P["rho_all"],
                             g.type, s.mass, alpha, cut, hoff, nz(hnb), de)
        d.update(alpha=alpha, heat_cut=cut, out_de_heat=de)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    out.append((name, g.nlocal, g.nghost, int(foff[-1])))


def multiphase_case(name, out):
    """Two-phase system with per-atom rmass (atom_style meso/multiphase) through the
    reference's rhosum/multiphase, taitwater/multiphase, heatconduction/phasechange,
    colorgradient and surfacetension."""
    R = po.ref()
    s = c3_system(5)
    nt = 2
    h = 1.6
    cut = np.zeros((3, 3))
    cut[1:, 1:] = h
    skin = 0.2
    cns, cmax = po.cutneighsq(nt, cut, skin)
    g = po.borders(s, cmax)
    foff, fnb = ref_full(R, s, g, cns, cmax)
    hoff, hnb = ref_half(R, g, foff, fnb)
    rng = np.random.default_rng(99)
    rmass = g.gather(np.where(s.type == 1, 1.0, 0.1) * (1 + 0.05 * rng.uniform(-1, 1, s.n)))
    rho = g.gather(np.where(s.type == 1, 1.0, 0.1) * (1 + 0.02 * rng.uniform(-1, 1, s.n)))
    e = g.gather(np.where(s.type == 1, 0.04, 0.12) * (1 + 0.3 * rng.uniform(-1, 1, s.n)))
    cv = g.gather(np.where(s.type == 1, 0.04, 0.06))
    vest = g.gather(s.v + 0.05 * rng.normal(size=s.v.shape))
    # rhosum/multiphase
    rho_mp = rho.copy()
    R.ref_rhosum_multiphase(3, nt, g.nlocal, g.nghost, g.x, g.type, rmass, cut, foff, nz(fnb),
                            rho_mp)
    # taitwater/multiphase (gamma[itype] quirk)
    rho0 = np.array([0.0, 1.0, 0.1])
    c0 = np.array([0.0, 10.0, 10.0])
    gamma = np.array([0.0, 7.0, 1.4])
    rbg = np.array([0.0, 0.5, 0.5])
    visc = np.zeros((3, 3))
    visc[1:, 1:] = 0.05
    f = np.zeros((g.nall, 3))
    R.ref_taitwater_multiphase(3, nt, g.nlocal, g.nghost, 1, g.x, vest, rho, g.type, rmass,
                               rho0, c0, gamma, rbg, visc, cut, hoff, nz(hnb), f)
    # heatconduction/phasechange with a clamp on the (1,2) pair
    alpha = np.zeros((3, 3))
    alpha[1:, 1:] = 0.1
    fixflag = np.zeros((3, 3), dtype=np.int32)
    fixflag[1, 2] = 1
    tc = np.zeros((3, 3))
    tc[1, 2] = 1.0
    de = np.zeros(g.nall)
    R.ref_heatconduction_phasechange(3, nt, g.nlocal, g.nghost, 1, g.x, e, cv, rho, rmass,
                                     g.type, alpha, fixflag.ctypes.data, tc.ctypes.data, cut,
                                     hoff, nz(hnb), de)
    # colorgradient
    cga = np.zeros((3, 3))
    cga[1:, 1:] = 1.0
    cg = np.zeros((g.nall, 3))
    R.ref_colorgradient(3, nt, g.nlocal, g.nghost, g.x, rho, rmass, g.type, cga, cut, foff,
                        nz(fnb), cg)
    # surfacetension on the half list, colorgradient of every atom (ghosts copy their owner:
    # the gradient is translation invariant)
    cg_all = g.gather(cg[:g.nlocal])
    st_cut = np.zeros((3, 3))
    st_cut[1:, 1:] = h
    f_st = np.zeros((g.nall, 3))
    R.ref_surfacetension(3, nt, g.nlocal, g.nghost, 1, g.x, rho, rmass, g.type, cg_all, st_cut,
                         hoff, nz(hnb), f_st)
    np.savez_compressed(
        os.path.join(HERE, name + ".npz"), dim=3, ntypes=nt, nlocal=g.nlocal, nghost=g.nghost,
        x=g.x, type=g.type, rmass=rmass, rho=rho, e=e, cv=cv, vest=vest, cut=cut,
        full_off=foff, full_nbr=fnb, half_off=hoff, half_nbr=hnb, rho0=rho0, c0=c0,
        gamma=gamma, rbg=rbg, visc=visc, alpha=alpha, fixflag=fixflag, tc=tc, cg_alpha=cga,
        out_rho=rho_mp[:g.nlocal], out_f=f, out_de=de, out_cg=cg[:g.nlocal], cg_all=cg_all,
        st_cut=st_cut, out_f_st=f_st)
    out.append((name, g.nlocal, g.nghost, int(foff[-1])))


def quintic_case(name, out):
    r = np.linspace(0.0, 3.2, 257)
    R = po.ref()
    d = {"r": r}
    for fn in ("kernel_quintic2d", "kernel_quintic3d", "dw_quintic2d", "dw_quintic3d"):
        d[fn] = np.array([getattr(R, "ref_" + fn)(float(v)) for v in r])
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    out.append((name, r.size, 0, 0))


def main():
    assert po.ref_available(), "build oracle/_ref first (oracle/build_ref.sh)"
    out = []
    single_phase_case("c2_n6", c2_system(6), po.c2_physics(), out)
    c2b = po.c2_physics(2.2)
    single_phase_case("c2_n7_h2.2", c2_system(7, seed=4242), c2b, out)
    single_phase_case("c3_n6", c3_system(6), po.c3_physics(), out)
    p2 = po.c2_physics(2.5)
    single_phase_case("c2_2d_n14", c2_system(14, dim=2), p2, out)
    multiphase_case("multiphase_n5", out)
    quintic_case("quintic", out)
    for row in out:
        print("%-14s nlocal=%-5d nghost=%-6d full=%d" % row)


if __name__ == "__main__":
    main()
