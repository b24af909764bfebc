"""C5 (bubble_growth) helpers shared by the multiphase-engine tests and the bench."""
import threading

import numpy as np


def mp_engine(sph, s, ph, path=0, procgrid=(1, 1, 1), rank=0, sel=None):
    """A multiphase engine for System s and MpPhysics ph (atoms set, phase change armed).
    procgrid/rank/sel: one brick of a decomposition holding the atoms s.x[sel] (tags = sel)."""
    mp = dict(rhosum_nstep=ph.rhosum_nstep, rhosum_cut=ph.rhosum_cut, cg_nstep=ph.cg_nstep,
              cg_alpha=ph.cg_alpha, cg_cut=ph.cg_cut)
    if ph.tait:
        mp.update(rho0=ph.rho0, c0=ph.c0, gamma=ph.gamma, rbg=ph.rbg, visc=ph.visc,
                  tait_cut=ph.tait_cut)
    if ph.st:
        mp.update(st_cut=ph.st_cut)
    if ph.heat:
        mp.update(heat_alpha=ph.heat_alpha, heat_cut=ph.heat_cut, heat_fixflag=ph.heat_fixflag,
                  heat_tc=ph.heat_tc)
    mass = np.where(s.mass > 0, s.mass, 1.0)
    cfg = sph.make_config(s.dim, s.ntypes, s.boxlo, s.boxhi, s.periodic, mass, ph.skin, ph.dt,
                          neigh_every=ph.every, kernel_path=path, mp=mp, procgrid=procgrid,
                          rank=rank)
    eng = sph.Engine(cfg)
    if sel is None:
        eng.set_atoms(s.x, s.v, s.type, s.rho, s.e, s.cv)
        eng.set_atoms_multiphase(s.rmass, s.cv)
    else:
        eng.set_atoms(s.x[sel], s.v[sel], s.type[sel], s.rho[sel], s.e[sel], s.cv[sel])
        eng.set_atoms_multiphase(s.rmass[sel], s.cv[sel])
        eng.set_tags(np.asarray(sel, dtype=np.int32))
    if ph.pc:
        p = ph.pc
        eng.phase_change(p["Tc"], p["Tt"], p["Hwv"], p["dr"], p["to_mass"], p["cutoff"],
                         p["from_type"], p["to_type"], nevery=p.get("nevery", 1),
                         seed=p["seed"], prob=p.get("prob", 0.0))
        eng.atom_sort(getattr(ph, "sortfreq", 1000), getattr(ph, "sort_binsize", 0.0))
    return eng


def mp_state(eng):
    g = eng.get_atoms()
    g.update(eng.get_atoms_multiphase())
    return g


def mp_bricks(sph, s, ph, pg, owner):
    """One engine per brick of procgrid pg over a LocalWorld (one host thread each when
    stepping, see bricks_step); owner[i] = the rank holding atom i."""
    P = int(np.prod(pg))
    world = sph.LocalWorld(P)
    engines = []
    for r in range(P):
        sel = np.nonzero(owner == r)[0]
        eng = mp_engine(sph, s, ph, procgrid=pg, rank=r, sel=sel)
        eng.comm_local(world, r)
        engines.append(eng)
    return world, engines


def bricks_step(engines, fn):
    """fn(eng) on every brick at once (the bricks exchange through the LocalWorld)."""
    errors = []

    def work(e):
        try:
            fn(e)
        except Exception as ex:  # surfaced below
            errors.append(ex)

    th = [threading.Thread(target=work, args=(e,)) for e in engines]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "brick threads hung"
    assert not errors, errors


def mp_collect(engines, n):
    """The bricks' atoms by tag (tags 0..n-1): every atom owned exactly once."""
    out, seen, counts = {}, np.zeros(n, dtype=np.int64), np.zeros(n, dtype=np.int32)
    ninserted = 0
    for eng in engines:
        g = mp_state(eng)
        tags = g["tag"]
        assert tags.size == 0 or (tags.min() >= 0 and tags.max() < n), "tag outside [0, n)"
        seen[tags] += 1
        for k, v in g.items():
            if k in ("tag", "ninserted") or not isinstance(v, np.ndarray) or v.shape[:1] != tags.shape:
                continue
            if k not in out:
                out[k] = np.zeros((n,) + v.shape[1:], dtype=v.dtype)
            out[k][tags] = v
        counts[tags] = eng.neighbor_counts()
        ninserted += int(g["ninserted"])
    assert (seen == 1).all(), "every atom owned by exactly one brick"
    out["ninserted"] = ninserted
    out["counts"] = counts
    return out


def unexplained_count_diffs(got, want, x, boxlo, boxhi, cutsq, rtol=1e-13):
    """The atoms whose neighbour counts differ (got vs want) by more than the number of their
    pairs within rtol of the cutoff (rsq vs cutneighsq, minimum image): on the bubble's exact
    binary lattice (32^3: dx = 1/32) ~30 pairs per atom sit exactly at the cutoff, and once
    the atoms have moved, a last-bit difference in a position flips such a pair in or out
    (the reference's own builds disagree on 8-35 atoms' counts at 32^3 after two steps,
    tools/c5_bricks_diag.py / DESIGN.md 3).  Returns the tags whose difference no near-tie
    explains."""
    got = np.asarray(got)
    want = np.asarray(want)
    bad = np.nonzero(got != want)[0]
    x = np.asarray(x, dtype=np.float64)
    prd = np.asarray(boxhi, dtype=np.float64) - np.asarray(boxlo, dtype=np.float64)
    out = []
    for t in bad:
        d = x - x[t]
        d -= prd * np.rint(d / prd)
        rsq = (d * d).sum(axis=1)
        rsq[t] = np.inf
        ties = int((np.abs(rsq - cutsq) <= rtol * cutsq).sum())
        if abs(int(got[t]) - int(want[t])) > ties:
            out.append(int(t))
    return out
