"""Standard systems of the parity tests (shrunk to sizes the oracle
finishes in seconds) and the oracle evaluations the HIP path is compared against."""
from __future__ import annotations

import os

import numpy as np

import pyoracle as po


def c2_system(n=8, seed=12345, dim=3):
    return po.cubic_lattice(n, seed=seed, dim=dim)


def c3_system(n=8, seed=12345):
    return po.cubic_lattice(n, seed=seed, ntypes=2, type2_frac=0.5, mass=(1.0, 0.5),
                            rho=(1.0, 0.5), e=(1.0, 2.0))


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def water_collapse_system():
    """C1: the reference's examples/USER/sph/water_collapse/data.initial (fixture
    golden/water_collapse.npz, made by golden/make_water_collapse.py): 15,702 atoms, 2-D,
    boundary f f p, atom_style meso."""
    d = np.load(os.path.join(GOLDEN, "water_collapse.npz"))
    return po.System(2, d["boxlo"].copy(), d["boxhi"].copy(), (0, 0, 1), d["x"].copy(),
                     d["v"].copy(), d["type"].astype(np.int32), d["rho"].copy(), d["e"].copy(),
                     d["cv"].copy(), 2, d["mass"].copy())


def water_collapse_physics(h=0.03, c=10.0):
    """water_collapse.lmp: pair_style hybrid/overlay sph/rhosum 1 sph/taitwater;
    pair_coeff * * sph/taitwater 1000 c 1.0 h (rho0, soundspeed, viscosity, cut);
    pair_coeff 1 1 sph/rhosum h; fix gravity -9.81 vector 0 1 0 on water (type 1); fix meso
    on water, meso/stationary on bc (type 2); neighbor 0.3 h bin, every 5; dt = 0.1 h / c."""
    rc = np.zeros((3, 3))
    rc[1, 1] = h
    tc = np.zeros((3, 3))
    tc[1:, 1:] = h
    visc = np.zeros((3, 3))
    visc[1:, 1:] = 1.0
    return po.Physics(skin=0.3 * h, dt=0.1 * h / c, every=5, rhosum_nstep=1, rhosum_cut=rc,
                      rho0=np.array([0.0, 1000.0, 1000.0]), c0=np.array([0.0, c, c]),
                      visc=visc, tait_cut=tc, stationary_mask=1 << 2,
                      gravity=(0.0, -9.81, 0.0), gravity_mask=1 << 1)


def prepared(sysm, ph: po.Physics, rho_jitter=0.02, vseed=7):
    """Owned+ghost atoms, full and half lists, and per-atom fields with some spread in rho
    and e (so the EOS / heat terms are exercised), as the pair styles see them."""
    nt = sysm.ntypes
    cns, cmax = po.cutneighsq(nt, ph.cutmax(nt), ph.skin)
    g = po.borders(sysm, cmax)
    foff, fnb = po.neigh_full(sysm.dim, g, nt, cns)
    hoff, hnb = po.half_from_full(g, foff, fnb)
    rng = np.random.default_rng(vseed)
    rho = sysm.rho * (1.0 + rho_jitter * rng.uniform(-1, 1, sysm.n))
    e = sysm.e + 0.1 * rng.uniform(-1, 1, sysm.n)
    vest = sysm.v + 0.05 * rng.normal(size=sysm.v.shape)
    if sysm.dim == 2:
        vest[:, 2] = 0.0
    return dict(g=g, foff=foff, fnb=fnb, hoff=hoff, hnb=hnb, cns=cns, cmax=cmax,
                rho_all=g.gather(rho), e_all=g.gather(e), vest_all=g.gather(vest))


def oracle_forces(sysm, ph: po.Physics, P, newton=1, reverse=True):
    """Reference semantics: half list, Newton-3 scatter, then reverse comm into owners."""
    g = P["g"]
    nt = sysm.ntypes
    B = ph.c0 * ph.c0 * ph.rho0 / 7.0
    f = np.zeros((g.nall, 3))
    drho = np.zeros(g.nall)
    de = np.zeros(g.nall)
    if ph.tait:
        f, drho, de = po.taitwater(sysm.dim, g, nt, newton, P["vest_all"], P["rho_all"],
                                   sysm.mass, ph.rho0, ph.c0, ph.visc, ph.tait_cut, P["hoff"],
                                   P["hnb"], morris=ph.morris, B=B)
    if ph.heat:
        de = de + po.heatconduction(sysm.dim, g, nt, newton, P["e_all"], P["rho_all"], sysm.mass,
                                    ph.alpha, ph.heat_cut, P["hoff"], P["hnb"])
    if reverse:
        po.reverse_comm(g, f, drho, de)
    return f, drho, de


def bubble_system(nx=10, dim=3, rv=None, slab=False):
    """C5 geometry (examples/USER/sph/bubble_growth/bubble.lmp, vars.lmp, in.phases): unit box,
    lattice sc (sq) dx = 1/nx with origin 0.5, liquid (type 1) everywhere, vapour (type 2)
    inside a sphere at the centre (radius rv, default 1.01 dx: the 8 (4) central sites);
    rho_l 1, rho_v 0.1, cv_l 0.04, cv_v 0.06, e = cv T with T_l = Tinf = 1, T_v = Tc = 0,
    per-atom mass = dx^dim rho."""
    dx = 1.0 / nx
    nz = nx if dim == 3 else 1
    g = np.stack(np.meshgrid(np.arange(nx), np.arange(nx), np.arange(nz), indexing="ij"),
                 -1).reshape(-1, 3)
    g = g[np.lexsort((g[:, 0], g[:, 1], g[:, 2]))]      # create_atoms: x fastest
    x = (g + 0.5) * dx
    if slab:   # jittered (a perfect lattice makes the colour gradient's transverse components
        # cancel exactly or not depending on summation order, and create_newpos' b2 = 0/0)
        x += np.random.default_rng(1234).uniform(-0.1, 0.1, size=x.shape) * dx
    if dim == 2:
        x[:, 2] = 0.0
    c = np.array([0.5, 0.5, 0.5 if dim == 3 else 0.0])
    rv = 1.01 * dx if rv is None else rv
    vap = ((x - c) ** 2).sum(1) < rv * rv
    if slab:   # vapour in the last x layer: its rows meet LAMMPS' first ghost slots (the
        vap = x[:, 0] > 1.0 - dx   # x-low layer imaged past x = 1), see sph_pc.h
    t = np.where(vap, 2, 1).astype(np.int32)
    rho = np.where(vap, 0.1, 1.0)
    cv = np.where(vap, 0.06, 0.04)
    e = np.where(vap, 0.06 * 0.0, 0.04 * 1.0)
    boxhi = np.array([1.0, 1.0, 1.0 if dim == 3 else dx])
    s = po.System(dim, np.zeros(3), boxhi, (1, 1, 1 if dim == 3 else 0), x, np.zeros_like(x), t,
                  rho, e, cv, 2, np.zeros(3), rmass=rho * dx ** dim)
    return s


def bubble_physics(nx=10, dim=3, dt=None, prob=0.01, Tt=0.1, pc=True, nevery=1, seed=123456):
    """bubble.lmp:57-73 pair stack with vars.lmp values (h = 3 dx, neighbor 0 bin, every 1)
    and fix phase_change Tc Tt Hwv dr mass_v cutoff 1 2 nevery seed prob (:105-109).
    dt defaults to a small multiple of the script's stability limits."""
    dx = 1.0 / nx
    h = 3.0 * dx
    rho_l, rho_v = 1.0, 0.1
    c_l, c_v = 200.0 / np.sqrt(rho_l), 200.0 / np.sqrt(rho_v)
    eta_l, eta_v = 1.0, 0.69
    eta_ld = 2 * eta_l * eta_v / (eta_v + eta_l)
    D_l, D_v = 0.2, 0.6
    D_ld = 2 * D_l * D_v / (D_v + D_l)
    alpha = 500.0
    hh = np.zeros((3, 3))
    hh[1:, 1:] = h
    cga = np.zeros((3, 3))
    cga[1, 2] = alpha
    visc = np.zeros((3, 3))
    visc[1, 1], visc[1, 2], visc[2, 2] = eta_l, eta_ld, eta_v
    hal = np.zeros((3, 3))
    hal[1, 1], hal[1, 2], hal[2, 2] = D_l, D_ld, D_v
    ff = np.zeros((3, 3), dtype=np.int32)
    ff[1, 2] = 2                       # "1 2 ... NULL Tc": type 2 held at Tc
    tc = np.zeros((3, 3))
    if dt is None:
        dt = 0.25 * 0.25 * dx / c_v
    pcd = None
    if pc:
        pcd = dict(Tc=0.0, Tt=Tt, Hwv=8.0, dr=0.5 * dx, to_mass=dx ** dim * rho_v, cutoff=h,
                   from_type=1, to_type=2, nevery=nevery, seed=seed, prob=prob)
    return po.MpPhysics(skin=0.0, dt=dt, every=1, rhosum_cut=hh.copy(), cg_alpha=cga,
                        cg_cut=hh.copy(), rho0=np.array([0.0, rho_l, rho_v]),
                        c0=np.array([0.0, c_l, c_v]), gamma=np.array([0.0, 1.0, 1.0]),
                        rbg=np.zeros(3), visc=visc, tait_cut=hh.copy(), st_cut=hh.copy(),
                        heat_alpha=hal, heat_cut=hh.copy(), heat_fixflag=ff, heat_tc=tc,
                        pc=pcd)


def skip_list_case(n=7, h=3.0, skin=0.3):
    """water_collapse.lmp's rhosum under hybrid/overlay (`pair_coeff 1 1 sph/rhosum`) on a
    two-type jittered box: the sub-style's SKIP list (pair_hybrid.cpp:428-485) holds the
    type-1 rows and their type-1 neighbours only.  Returns the inputs of ref_rhosum_skip and
    the oracle's result (type-1 rows summed over that list, type-2 rho untouched)."""
    s = po.cubic_lattice(n, ntypes=2, type2_frac=0.4, rho=(1.0, 0.7))
    nt = 2
    cut = np.zeros((nt + 1, nt + 1))
    cut[1, 1] = h
    cns, cmax = po.cutneighsq(nt, cut, skin)
    g = po.borders(s, cmax)
    off, nb = po.neigh_full(s.dim, g, nt, cns)
    rows = np.nonzero(s.type == 1)[0].astype(np.int32)
    soff = [0]
    snb = []
    moff = np.zeros(s.n + 1, dtype=np.int64)  # (the oracle's CSR: type-2 rows empty)
    for i in range(s.n):
        js = nb[off[i]:off[i + 1]]
        keep = js[g.type[js] == 1] if s.type[i] == 1 else js[:0]
        if s.type[i] == 1:
            snb.append(keep)
            soff.append(soff[-1] + len(keep))
        moff[i + 1] = moff[i] + len(keep)
    snb = np.concatenate(snb).astype(np.int32) if snb else np.zeros(0, np.int32)
    iskip = np.array([0, 0, 1], dtype=np.int32)
    ijskip = np.ones((nt + 1, nt + 1), dtype=np.int32)
    ijskip[1, 1] = 0
    rho0 = g.gather(s.rho)
    want = s.rho.copy()
    got = po.rhosum(s.dim, g, nt, s.mass, cut, moff, snb)
    want[rows] = got[rows]
    return dict(dim=s.dim, nt=nt, nlocal=s.n, nghost=g.nghost, x=np.ascontiguousarray(g.x),
                type=np.ascontiguousarray(g.type, dtype=np.int32), mass=s.mass, cut=cut,
                rows=rows, off=np.asarray(soff, dtype=np.int64), nb=snb, iskip=iskip,
                ijskip=np.ascontiguousarray(ijskip.ravel()), rho0=rho0, want=want)


def run_rhosum_skip(R, c):
    """R.ref_rhosum_skip on a case of skip_list_case; returns the owned rho"""
    rho = c["rho0"].copy()
    R.ref_rhosum_skip(c["dim"], c["nt"], c["nlocal"], c["nghost"], c["x"], c["type"],
                      c["mass"], np.ascontiguousarray(c["cut"].ravel()), len(c["rows"]),
                      c["rows"], c["off"], c["nb"] if c["nb"].size else np.zeros(1, np.int32),
                      c["iskip"], c["ijskip"], rho)
    return rho[:c["nlocal"]]


def shuffled(s, seed):
    """The same atoms read in another order (a data file's line order = the tags)."""
    p = np.random.default_rng(seed).permutation(s.n)
    s = s.copy()
    for k in ("x", "v", "type", "rho", "e", "cv", "rmass"):
        if getattr(s, k) is not None:
            setattr(s, k, np.ascontiguousarray(getattr(s, k)[p]))
    return s


def drifting(s, vx, dx0):
    """s moving as a whole along x at vx, shifted by dx0 (wrapped into the box): atoms cross
    brick faces every few steps (CommBrick::exchange), the flow itself unchanged."""
    s = s.copy()
    lo, hi = s.boxlo[0], s.boxhi[0]
    x = s.x[:, 0] + dx0
    s.x[:, 0] = np.where(x >= hi, x - (hi - lo), x)
    s.v[:, 0] += vx
    return s
