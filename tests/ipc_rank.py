"""One rank of a multi-PROCESS engine run (driven by tests/test_gpu_processes.py).

Usage: python tests/ipc_rank.py SPEC.json -- SPEC names the scenario, this process's rank,
the world size, the processor grid, the IPC world name and mode, the step schedule and the
.npz to write.  The rank builds ONLY its own brick (the atoms the decomposition gives it,
global tags), attaches the node-local process world (sph_engine_comm_ipc), runs setup and
the steps, and writes its owned atoms (tags, fields, neighbour counts) after setup and after
every step of the schedule.  The parent merges the ranks' files by tag and compares them
with the oracle; nothing here computes a reference."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)

import pyoracle as po  # noqa: E402  (the System/Physics constructors only)
from c5_util import mp_engine, mp_state  # noqa: E402
from conftest import load_sph_amd  # noqa: E402
from scenarios import bubble_physics, bubble_system, c2_system, drifting, shuffled  # noqa: E402


def c2_scenario(spec):
    """tests/test_gpu_bricks.py::test_bricks_migration's system: the 12^3 lattice from rest,
    pressure-driven motion with dt 5e-3, rebuilds (and migrations) every 5 steps."""
    s = c2_system(spec.get("n", 12))
    s.v[:] = 0.0
    ph = po.c2_physics()
    ph.dt = spec.get("dt", 5e-3)
    ph.every = spec.get("every", 5)
    return s, ph


def c5_scenario(spec):
    """tests/test_c5_bricks.py's jittered slab: bubble_growth stack + fix phase_change.
    drift: the bubble instead, read in a shuffled order and moving along x at that speed, so
    atoms cross the brick faces (exchange hole fill) while Atom::sort runs every `sortfreq`."""
    nx, dim = spec["nx"], spec.get("dim", 3)
    if spec.get("drift"):
        s = drifting(shuffled(bubble_system(nx, dim=dim), 3), spec["drift"], 0.49 / nx)
        ph = bubble_physics(nx, dim=dim, prob=0.5, Tt=-1.0)
    else:
        s = bubble_system(nx, dim=dim, slab=True)
        ph = bubble_physics(nx, dim=dim, prob=0.3, Tt=-1.0)
    ph.sortfreq = spec.get("sortfreq", ph.sortfreq)
    return s, ph


def main():
    spec = json.load(open(sys.argv[1]))
    sph = load_sph_amd()
    r, P, pg = spec["rank"], spec["nranks"], tuple(spec["pg"])
    mp = spec["scenario"] == "c5"
    s, ph = (c5_scenario if mp else c2_scenario)(spec)
    owner = po.brick_owner(s, s.x, pg)
    sel = np.nonzero(owner == r)[0]
    if mp:
        eng = mp_engine(sph, s, ph, procgrid=pg, rank=r, sel=sel)
    else:
        cfg = sph.make_config(s.dim, s.ntypes, s.boxlo, s.boxhi, s.periodic, s.mass, ph.skin,
                              ph.dt, neigh_every=ph.every, kernel_path=spec.get("path", 0),
                              procgrid=pg, rank=r,
                              rhosum=dict(nstep=ph.rhosum_nstep, cut=ph.rhosum_cut),
                              tait=dict(rho0=ph.rho0, c0=ph.c0, visc=ph.visc, cut=ph.tait_cut,
                                        morris=ph.morris))
        eng = sph.Engine(cfg)
        eng.set_atoms(s.x[sel], s.v[sel], s.type[sel], s.rho[sel], s.e[sel], s.cv[sel])
        eng.set_tags(sel)
    eng.comm_ipc(spec["name"], P, r, spec["mode"])
    if spec.get("die"):  # (a rank that dies after joining: its heartbeat stops)
        os._exit(3)
    snaps = {}

    def snap(k):
        g = mp_state(eng) if mp else eng.get_atoms()
        g["counts"] = eng.neighbor_counts()
        for key, v in g.items():
            snaps[f"{k}/{key}"] = np.asarray(v)

    try:
        eng.setup()
        snap(0)
        done = 0
        for upto in spec["snap_steps"]:
            eng.run(upto - done)
            done = upto
            snap(upto)
    except sph.HipError as err:
        if not spec.get("expect_dead"):
            raise
        print("PEER_GONE", err, flush=True)
        os._exit(0)
    st = eng.stats()
    snaps["staged"] = np.asarray(st["staged"])
    snaps["nghost"] = np.asarray(st["nghost"])
    eng.close()
    np.savez(spec["out"], **snaps)


if __name__ == "__main__":
    main()
