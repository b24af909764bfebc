"""C5 on the device-resident engine: the bubble_growth stack (examples/USER/sph/bubble_growth/
bubble.lmp:57-73 -- rhosum/multiphase + colorgradient + taitwater/multiphase +
surfacetension + heatconduction/phasechange, rebuild every step) with fix phase_change
(fix_phase_change.cpp:167-352), against the oracle's Verlet driver (pyoracle.MpRefRun).

Tolerances: fields 1e-10 normwise (north_star), atom counts, insertions, types and
neighbour counts exact -- from the setup step on: the initial perfect lattice puts ~30 pairs
per atom exactly at the cutoff, which the reference's own Neighbor::full_bin keeps
(rsq <= cutneighsq, neigh_full.cpp:312; test_oracle_vs_reference_lattice_ties pins the
oracle's builder to it there).  The oracle's fix phase_change is the reference's own behaviour
(pinned by test_phasechange_golden.py), created atoms overwriting ghost slots included; the
slab cases are geometries where that matters."""
import dataclasses

import numpy as np
import pytest

import pyoracle as po
from conftest import check_fields, rel_err
from scenarios import bubble_physics, bubble_system, shuffled

TOL = 1e-10


def test_oracle_bubble_conserves_mass():
    s = bubble_system(8)
    ph = bubble_physics(8, prob=0.5, Tt=-1.0)
    ref = po.MpRefRun(s, ph)
    ref.setup()
    m0 = ref.s.rmass.sum()
    ref.run(3)
    assert ref.ninserted >= 1 and ref.s.n == s.n + ref.ninserted
    assert np.all(ref.s.type[s.n:] == 2)
    assert abs(ref.s.rmass.sum() - m0) < 1e-14 * m0
    assert np.all(np.isfinite(ref.f)) and np.all(ref.s.rmass > 0)


def test_slab_geometry_exercises_the_aliasing():
    """With the vapour in the last x layer, atoms created early in a call land on LAMMPS'
    first ghost slots -- images of the x-low layer right next to later candidates -- so the
    reference's result (MpRefRun, pc_exact) differs from evaluating every candidate on the
    atoms as found: the donations to those slots are lost and the total mass grows.  The
    engine must follow the reference (test_engine_c5_vs_oracle[slab])."""
    res = {}
    for exact in (True, False):
        s = bubble_system(8, slab=True)
        # (no sort: the global path, where pc_exact selects the port semantics)
        ph = dataclasses.replace(bubble_physics(8, prob=0.3, Tt=-1.0), sortfreq=0)
        ref = po.MpRefRun(s, ph)
        ref.pc_exact = exact
        ref.setup()
        m0 = ref.s.rmass.sum()
        ref.run(3)
        res[exact] = (ref.ninserted, ref.s.rmass.sum() - m0)
    assert res[True][0] == res[False][0] >= 2
    assert abs(res[False][1]) < 1e-14 and res[True][1] > 1e-6


def _compare(eng, ref, counts=True):
    from c5_util import mp_state
    g = mp_state(eng)
    s = ref.s
    assert g["x"].shape[0] == s.n and g["ninserted"] == ref.ninserted
    assert np.array_equal(g["type"], s.type)
    if counts:
        assert np.array_equal(eng.neighbor_counts(), ref.numneigh_full())
    check_fields(g, ref, ("x", "v", "rho", "e", "rmass", "cv", "cg", "f", "de"), TOL)
    return g


@pytest.mark.gpu
@pytest.mark.parametrize("nx,dim,slab", [(10, 3, False), (16, 2, False), (8, 3, True),
                                         (12, 2, True)])
def test_engine_c5_vs_oracle(gpu, sph_amd, nx, dim, slab):
    from c5_util import mp_engine
    s = bubble_system(nx, dim=dim, slab=slab)
    ph = bubble_physics(nx, dim=dim, prob=0.3 if slab else 0.5, Tt=-1.0)
    ref = po.MpRefRun(s, ph, spread=True)
    ref.setup()
    eng = mp_engine(sph_amd, s, ph)
    eng.setup()
    _compare(eng, ref)
    for _ in range(5):
        ref.run(1)
        eng.run(1)
        _compare(eng, ref)
    assert ref.ninserted >= 1


@pytest.mark.gpu
def test_engine_c5_no_phase_change_every2(gpu, sph_amd):
    """The stack alone with rebuilds every 2 steps: the forward-comm steps carry v, rmass, cv
    and colorgradient to the ghosts (comm_modify vel yes)."""
    from c5_util import mp_engine
    s = bubble_system(10)
    ph = bubble_physics(10, pc=False)
    ph.every = 2
    ref = po.MpRefRun(s, ph, spread=True)
    ref.setup()
    eng = mp_engine(sph_amd, s, ph)
    eng.setup()
    _compare(eng, ref)
    ref.run(5)
    eng.run(5)
    _compare(eng, ref)



@pytest.mark.gpu
@pytest.mark.parametrize("sortfreq,binsize", [(1000, 0.0), (3, 0.0), (2, 0.06), (0, 0.0)])
def test_engine_c5_local_order(gpu, sph_amd, sortfreq, binsize):
    """fix phase_change meets its candidates in LAMMPS' local order: the atoms read in a
    shuffled order, then Atom::sort at setup and every sortfreq steps (atom_modify sort;
    binsize 0 = half the neighbour cutoff), created atoms appended.  The engine tracks that
    order beside its own rows; the draws must meet the same candidates as the oracle's."""
    from c5_util import mp_engine
    s = shuffled(bubble_system(10), 7)
    ph = dataclasses.replace(bubble_physics(10, prob=0.5, Tt=-1.0), sortfreq=sortfreq,
                             sort_binsize=binsize)
    ref = po.MpRefRun(s, ph, spread=True)
    ref.setup()
    eng = mp_engine(sph_amd, s, ph)
    eng.setup()
    _compare(eng, ref)
    for _ in range(7):
        ref.run(1)
        eng.run(1)
        _compare(eng, ref)
    assert ref.ninserted >= 3


@pytest.mark.gpu
def test_engine_c5_read_order_differs_from_tags(gpu, sph_amd):
    """LAMMPS' initial local order is the read order (data-file lines), not tag order: the
    atoms handed to set_atoms in a permuted order with their tags set (sph_engine_set_tags)
    -- the engine starts its local-order index at that read order (set_atoms), the oracle
    its local lists (MpRefRun read_order).  Atom::sort at setup keeps the read order within a
    bin (stable), so the candidates meet the draws in an order that depends on it.  (Parity
    with LAMMPS itself is unpinned here: the oracle restates the order bookkeeping.)"""
    from c5_util import mp_engine, mp_state
    s = bubble_system(10)
    ph = dataclasses.replace(bubble_physics(10, prob=0.5, Tt=-1.0), sortfreq=1000)
    perm = np.random.default_rng(11).permutation(s.n).astype(np.int32)
    ref = po.MpRefRun(s, ph, spread=True, read_order=perm)
    ref.setup()
    eng = mp_engine(sph_amd, s, ph, sel=perm)
    eng.setup()

    def cmp():
        g = mp_state(eng)
        o = np.argsort(g["tag"])   # (local order -> tag order)
        g = {k: (v[o] if isinstance(v, np.ndarray) and v.shape[:1] == o.shape else v)
             for k, v in g.items()}
        assert g["x"].shape[0] == ref.s.n and g["ninserted"] == ref.ninserted
        assert np.array_equal(g["type"], ref.s.type)
        check_fields(g, ref, ("x", "v", "rho", "e", "rmass", "cv", "cg", "f", "de"), TOL)

    cmp()
    for _ in range(5):
        ref.run(1)
        eng.run(1)
        cmp()
    assert ref.ninserted >= 2
    # the same atoms read in tag order draw a different set of insertions
    ref2 = po.MpRefRun(s, ph)
    ref2.setup()
    ref2.run(5)
    assert ref2.ninserted != ref.ninserted or not np.array_equal(ref2.s.x, ref.s.x)


@pytest.mark.gpu
def test_phase_change_after_setup_rejected(gpu, sph_amd):
    """fix phase_change is armed before setup (its local-order bookkeeping starts at
    set_atoms): arming it afterwards is an error, not a silent wrong order."""
    from c5_util import mp_engine
    s = bubble_system(8)
    ph = bubble_physics(8, prob=0.5, Tt=-1.0)
    eng = mp_engine(sph_amd, s, dataclasses.replace(ph, pc=None))
    eng.setup()
    p = ph.pc
    with pytest.raises(sph_amd.HipError, match="before sph_engine_setup"):
        eng.phase_change(p["Tc"], p["Tt"], p["Hwv"], p["dr"], p["to_mass"], p["cutoff"],
                         p["from_type"], p["to_type"], seed=p["seed"], prob=p.get("prob", 0.0))
