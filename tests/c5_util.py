"""C5 (bubble_growth) helpers shared by the multiphase-engine tests and the bench."""
import numpy as np


def mp_engine(sph, s, ph, path=0):
    """A multiphase engine for System s and MpPhysics ph (atoms set, phase change armed)."""
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
                          neigh_every=ph.every, kernel_path=path, mp=mp)
    eng = sph.Engine(cfg)
    eng.set_atoms(s.x, s.v, s.type, s.rho, s.e, s.cv)
    eng.set_atoms_multiphase(s.rmass, s.cv)
    if ph.pc:
        p = ph.pc
        eng.phase_change(p["Tc"], p["Tt"], p["Hwv"], p["dr"], p["to_mass"], p["cutoff"],
                         p["from_type"], p["to_type"], nevery=p.get("nevery", 1),
                         seed=p["seed"], prob=p.get("prob", 0.0))
    return eng


def mp_state(eng):
    g = eng.get_atoms()
    g.update(eng.get_atoms_multiphase())
    return g
