"""Golden vectors for fix phase_change from the REFERENCE's own FixPhaseChange.

oracle/_ref/libsph_ref.so holds fix_phase_change.cpp, random_park.cpp, region.cpp and
region_block.cpp compiled from /root/reference/src (oracle/build_ref.sh).  The harness
(oracle/ref_harness.cpp: ref_pc_new / ref_pc_pre_exchange) constructs FixPhaseChange from its
own argument list (so the reference parses "... seed prob|ENERGY rate region box units box"),
keeps it alive across calls (one RanPark stream, as in a LAMMPS run), and calls
pre_exchange() on atoms + ghosts given in LAMMPS index order with CommBrick's self swaps set up
for reverse_comm_fix.  Every output -- which atoms change phase, the created atoms (written by
AtomVecMesoMultiPhase::create_atom over the ghost slots right after the owned atoms), donor
rmass and energies -- is produced by reference code.  The inputs (ghosts from the restated
CommBrick::borders, the full list from the reference's own Neighbor::full_bin, colour
gradients from the reference's PairSPHColorGradient) are stored with them.

Cases:
  kat          examples/USER/sph/multiphase_two_atoms/phase_change.lmp (2 atoms, prob 1)
  slab         6^3 two-phase box, vapour slab at the x-high face: several insertions per call,
               ghost donors, and created atoms landing on ghost slots that later candidates'
               lists still name (the reference then loses those ghosts' donations: mass is
               not conserved -- this fixture pins that behaviour); two consecutive calls
  bubble       7^3 box with a vapour core (bubble_growth-like), ENERGY-rate variant, two calls
  slab2d       2-D version of slab (create_newpos' 2-D branch)

Run here (where /root/reference exists):  python tests/golden/make_phase_change.py
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)
import pyoracle as po  # noqa: E402
from make_golden import ref_full  # noqa: E402

FIELDS3 = ("x", "v", "vest", "cg")
FIELDS1 = ("e", "rmass", "rho", "cv")


def two_phase(n, dx, h, skin, vap, dim=3, seed=5, cga=1.0):
    """jittered lattice of liquid (type 1) with vapour (type 2) where vap(x); per-atom fields
    with spread; colour gradient from the reference's own style; full list from the
    reference's own builder."""
    R = po.ref()
    s = po.cubic_lattice(n, dx=dx, jitter=0.1, seed=seed, ntypes=2, dim=dim)
    s.type = np.where(vap(s.x), 2, 1).astype(np.int32)
    rng = np.random.default_rng(seed + 1)
    liq = s.type == 1
    own = dict(rmass=np.where(liq, 1.0, 0.3) * (1 + 0.05 * rng.uniform(-1, 1, s.n)),
               rho=np.where(liq, 1.0, 0.3) * (1 + 0.02 * rng.uniform(-1, 1, s.n)),
               cv=np.where(liq, 1.0, 0.5),
               e=np.where(liq, 1.0, 2.0) * (1 + 0.5 * rng.uniform(-1, 1, s.n)),
               v=s.v, vest=s.v + 0.01 * rng.normal(size=s.v.shape))
    if dim == 2:
        own["vest"][:, 2] = 0.0
    s.rmass = own["rmass"]
    return s, own, h, skin, cga


def ghosts_and_list(s, own, h, skin, cga):
    R = po.ref()
    nt = 2
    cut = np.zeros((3, 3))
    cut[1:, 1:] = h
    cns, cmax = po.cutneighsq(nt, cut, skin)
    g = po.borders(s, cmax)
    foff, fnb = ref_full(R, s, g, cns, cmax)
    d = {k: np.ascontiguousarray(g.gather(v)) for k, v in own.items()}
    alpha = np.zeros((3, 3))
    alpha[1, 2] = alpha[2, 1] = cga
    cg = np.zeros((g.nall, 3))
    R.ref_colorgradient(s.dim, nt, g.nlocal, g.nghost, g.x, d["rho"], d["rmass"], g.type, alpha,
                        cut, foff, fnb if fnb.size else np.zeros(1, np.int32), cg)
    cg[g.nlocal:] = cg[g.owner]          # forward comm of the colour gradient
    d.update(x=np.ascontiguousarray(g.x), type=np.ascontiguousarray(g.type), cg=cg)
    return g, d, foff, fnb


def ref_call(R, hnd, step, g, d, foff, fnb, extra=256):
    nmax = g.nall + extra
    A = {}
    for k in FIELDS3:
        b = np.zeros((nmax, 3))
        b[:g.nall] = d[k]
        A[k] = b
    for k in FIELDS1:
        b = np.zeros(nmax)
        b[:g.nall] = d[k]
        A[k] = b
    t = np.zeros(nmax, np.int32)
    t[:g.nall] = d["type"]
    A["type"] = t
    nr = C.c_long(0)
    n = R.ref_pc_pre_exchange(hnd, step, g.nlocal, g.nghost, nmax, A["x"], A["v"], A["vest"],
                              A["cg"], A["e"], A["rmass"], A["rho"], A["cv"], A["type"], foff,
                              fnb if fnb.size else np.zeros(1, np.int32),
                              len(g.swap_first) - 1, g.swap_first,
                              g.src if g.src.size else np.zeros(1, np.int32), C.byref(nr))
    return n, {k: v[:n].copy() for k, v in A.items()}, nr.value


def run_case(name, s, own, h, skin, cga, args, ncalls, out, dt=1e-3):
    R = po.ref()
    av = (C.c_char_p * len(args))(*[a.encode() for a in args])
    hnd = R.ref_pc_new(s.dim, 2, s.boxlo, s.boxhi, 0, dt, len(args), av)
    d_out = dict(args=np.array(args), dim=s.dim, boxlo=s.boxlo, boxhi=s.boxhi,
                 periodic=np.array(s.periodic, np.int32), ncalls=ncalls, dt=dt)
    owned = {k: np.array(v) for k, v in own.items()}
    owned["x"] = s.x.copy()
    owned["type"] = s.type.copy()
    summary = []
    for c in range(ncalls):
        s.x = owned["x"]
        s.type = owned["type"]
        s.rmass = owned["rmass"]
        ownf = {k: owned[k] for k in ("rmass", "rho", "cv", "e", "v", "vest")}
        g, d, foff, fnb = ghosts_and_list(s, ownf, h, skin, cga)
        n, A, nr = ref_call(R, hnd, c + 1, g, d, foff, fnb)
        p = f"c{c}_"
        for k in FIELDS3 + FIELDS1 + ("type",):
            d_out[p + "in_" + k] = d[k]
            d_out[p + "out_" + k] = A[k]
        d_out.update({p + "nlocal": g.nlocal, p + "nghost": g.nghost, p + "full_off": foff,
                      p + "full_nbr": fnb, p + "swap_first": g.swap_first, p + "src": g.src,
                      p + "owner": g.owner, p + "out_nlocal": n, p + "next_reneighbor": nr})
        m0 = d["rmass"][:g.nlocal].sum()
        m1 = A["rmass"].sum()
        summary.append(f"call {c}: nlocal {g.nlocal} nghost {g.nghost} created {n - g.nlocal}"
                       f" mass {m0:.12f} -> {m1:.12f}")
        # next call: the owned atoms after this one (created atoms appended, tag order)
        owned = {k: A[k].copy() for k in FIELDS3 + FIELDS1 + ("type",)}
    np.savez_compressed(os.path.join(HERE, f"pc_{name}.npz"), **d_out)
    out.append((name, summary))


def fix_args(Tc, Tt, Hwv, dr, to_mass, pcut, nfreq, seed, chance=None, rate=None,
             extra=("region", "box", "units", "box")):
    a = ["fdep", "all", "phase_change", repr(Tc), repr(Tt), repr(Hwv), repr(dr), repr(to_mass),
         repr(pcut), "1", "2", str(nfreq), str(seed)]
    a += ["ENERGY", repr(rate)] if rate is not None else [repr(chance)]
    return a + list(extra)


def kat_case(out):
    """phase_change.lmp: box 0..10 x 0..10 x -10..10, create_atoms from phase_change.mac
    (x = (5,5,5) type 1 and (5.6,5,5) type 2), m = (10, 2), rho 1, e = (10, 2),
    cv = (3, 1), colorgradient h = 1 with alpha(1,2) = 1, neighbor 0, Tc = Tt = Hwv = dr =
    to_mass = pcutoff = 1, seed 123456, prob 1."""
    s = po.System(3, np.array([0.0, 0.0, -10.0]), np.array([10.0, 10.0, 10.0]), (1, 1, 1),
                  np.array([[5.0, 5.0, 5.0], [5.6, 5.0, 5.0]]), np.zeros((2, 3)),
                  np.array([1, 2], np.int32), np.ones(2), np.array([10.0, 2.0]),
                  np.array([3.0, 1.0]), 2, np.zeros(3), np.array([10.0, 2.0]))
    own = dict(rmass=np.array([10.0, 2.0]), rho=np.ones(2), cv=np.array([3.0, 1.0]),
               e=np.array([10.0, 2.0]), v=np.zeros((2, 3)), vest=np.zeros((2, 3)))
    run_case("kat", s, own, 1.0, 0.0, 1.0,
             fix_args(1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1, 123456, chance=1.0), 1, out, dt=0.0)


def main():
    assert po.ref_available(), "build oracle/_ref first (oracle/build_ref.sh)"
    out = []
    kat_case(out)
    # bubble_growth scales: pcutoff = h with r*h < 1 everywhere in the list (quirk A.6-3)
    s, own, h, skin, cga = two_phase(6, 0.1, 0.15, 0.01, lambda x: x[:, 0] > 0.42)
    run_case("slab", s, own, h, skin, cga,
             fix_args(1.0, 1.2, 0.5, 0.05, 0.05, h, 1, 123456, chance=0.3), 2, out)
    c = 0.35
    s, own, h, skin, cga = two_phase(
        7, 0.1, 0.3, 0.0, lambda x: ((x - c) ** 2).sum(1) < 0.2 ** 2, seed=11)
    run_case("bubble", s, own, h, skin, cga,
             fix_args(1.0, 1.1, 8.0, 0.05, 0.03, h, 1, 7777, rate=400.0), 2, out, dt=1e-3)
    s, own, h, skin, cga = two_phase(12, 0.1, 0.25, 0.01, lambda x: x[:, 1] > 0.85, dim=2,
                                     seed=21)
    run_case("slab2d", s, own, h, skin, cga,
             fix_args(1.0, 1.2, 0.5, 0.05, 0.05, h, 1, 4242, chance=0.4), 2, out)
    for name, summ in out:
        print(name)
        for line in summ:
            print("   ", line)


if __name__ == "__main__":
    main()
