"""The oracle's brick emulation (pyoracle.borders_bricks, MpRefRun(procgrid=...)) on the CPU:
a 1x1x1 grid reproduces the single-process CommBrick::borders and fix phase_change exactly,
and on real grids every rank's view is a consistent CommBrick picture (each ghost is the
image of its origin, created atoms lie in their rank's sub-box, mass is conserved where no
created atom lands on a donor's ghost slot)."""
import dataclasses

import numpy as np
import pytest

import pyoracle as po
from scenarios import bubble_physics, bubble_system, shuffled


def test_one_brick_grid_is_the_single_process_borders():
    s = bubble_system(10)
    g = po.borders(s, 0.3)
    bv = po.borders_bricks(s, 0.3, (1, 1, 1))[0]
    assert bv.nghost == g.nghost
    assert np.array_equal(bv.gid[bv.nlocal:], g.owner)
    assert np.array_equal(bv.x, g.x)
    assert list(bv.swap_first) == list(g.swap_first)
    assert np.array_equal(bv.src_idx, g.src)


def test_one_brick_grid_is_the_single_process_phase_change():
    s = bubble_system(10)
    ph = dataclasses.replace(bubble_physics(10, prob=0.5, Tt=-1.0), sortfreq=0)
    a = po.MpRefRun(s, ph)
    assert a.pg is None                   # (no sort: local order = tag order, global path)
    b = po.MpRefRun(s, ph)
    b.pg, b.seeds = (1, 1, 1), [b.seed]   # force the per-rank path on one rank
    for r in (a, b):
        r.setup()
        r.run(3)
    # (the per-rank path reverse-communicates along the swaps, the single path straight to
    # the owners: summation order differs, hence rounding)
    assert a.ninserted == b.ninserted >= 1
    assert np.array_equal(a.s.type, b.s.type)
    rel = lambda x, y: np.abs(x - y).max() / np.abs(y).max()
    for k in ("x", "v", "e", "rmass", "rho", "cv"):
        assert rel(getattr(b.s, k), getattr(a.s, k)) < 1e-13, k
    assert rel(b.f, a.f) < 1e-13 and rel(b.de, a.de) < 1e-13
    assert np.array_equal(a.numneigh_full(), b.numneigh_full())


def test_decomposition_changes_the_reference_result():
    """The multiphase styles' misnamed pack_comm leaves the ghosts' rho and colour gradient
    as communicated, so a pair across a brick face sees a stale neighbour where one process
    sees a fresh owned one: the reference's own results depend on the decomposition (the
    engine follows the decomposition it runs on, tests/test_c5_bricks.py)."""
    s = bubble_system(10)
    ph = bubble_physics(10, pc=False)
    a = po.MpRefRun(s, ph)
    b = po.MpRefRun(s, ph, procgrid=(2, 2, 2))
    a.setup()
    b.setup()
    rel = lambda x, y: np.abs(x - y).max() / np.abs(y).max()
    assert rel(b.s.rho, a.s.rho) < 1e-13          # rhosum/multiphase reads x and rmass only
    assert rel(b.cg, a.cg) > 1e-7 and rel(b.f, a.f) > 1e-3


@pytest.mark.parametrize("pg", [(2, 1, 1), (1, 2, 2), (2, 2, 2)])
def test_brick_views_are_consistent(pg):
    s = bubble_system(10)
    cut = 0.3
    views = po.borders_bricks(s, cut, pg)
    assert sum(v.nlocal for v in views) == s.n
    prd = s.boxhi - s.boxlo
    for v in views:
        nl = v.nlocal
        assert np.all(np.diff(v.gid[:nl]) > 0)            # owned in tag order
        want = s.x[v.gid] + v.image * prd
        assert np.allclose(v.x, want, atol=1e-14, rtol=0)
        assert np.all(v.x[nl:] >= v.lo - cut - 1e-12) and np.all(v.x[nl:] <= v.hi + cut + 1e-12)
        # the sender's copy of each ghost is the same atom
        for g in range(v.nghost):
            src = views[v.src_rank[g]]
            assert src.gid[v.src_idx[g]] == v.gid[nl + g]


@pytest.mark.parametrize("pg", [(2, 1, 1), (2, 2, 2)])
def test_bricks_phase_change_inserts_inside_subboxes(pg):
    s = bubble_system(10)
    ph = bubble_physics(10, prob=0.5, Tt=-1.0)
    ref = po.MpRefRun(s, ph, procgrid=pg)
    ref.setup()
    m0 = ref.s.rmass.sum()
    n0 = ref.s.n
    grid = po.brick_grid(s, pg)
    for _ in range(3):
        views = ref.bviews
        nb = ref.s.n
        ref.run(1)
        # the atoms created this step, rank by rank: each inside its creator's sub-box
        new = ref.s.x[nb:]
        if new.shape[0]:
            own = po.brick_owner(s, new, pg)
            assert np.all(np.diff(own) >= 0)
            for r, x in zip(own, new):
                assert np.all(x >= grid[r]["lo"]) and np.all(x[:3] < grid[r]["hi"] + 1e-12)
    assert ref.ninserted >= 2 and ref.s.n == n0 + ref.ninserted
    assert abs(ref.s.rmass.sum() - m0) < 1e-14 * m0


def test_hole_fill_is_comm_brick_exchange_scan():
    """comm_brick.cpp:620-632 by hand: slots 1 and 3 of 6 leave; slot 1 takes the last atom
    (5), slot 3 takes 4 -- which also leaves, so slot 3 then takes 3's... (n shrinks)."""
    kept, sent = po.hole_fill(np.arange(6), np.array([0, 1, 0, 1, 1, 0], bool))
    # i=1 leaves -> a[1]=5 (stays); i=3 leaves -> a[3]=a[4]=4 (leaves) -> a[3]=a[3] (n=3)
    assert kept.tolist() == [0, 5, 2]
    assert sent.tolist() == [1, 3, 4]
    kept, sent = po.hole_fill(np.arange(4), np.ones(4, bool))
    assert kept.size == 0 and sent.tolist() == [0, 3, 2, 1]
    kept, sent = po.hole_fill(np.arange(3), np.zeros(3, bool))
    assert kept.tolist() == [0, 1, 2] and sent.size == 0


def test_sort_bricks_is_atom_sort():
    """Atom::sort: bins of half the neighbour cutoff over the sub-box, x fastest, stable
    within a bin (atom.cpp:1586-1615); a single bin leaves the order alone."""
    s = bubble_system(6)
    rng = np.random.default_rng(5)
    order = rng.permutation(s.n)
    out = po.sort_bricks(s, (1, 1, 1), [order], 0.25)[0]
    lo, hi = s.boxlo, s.boxhi
    nb = [max(int((hi[k] - lo[k]) / 0.25), 1) for k in range(3)]
    ib = []
    for k in range(3):
        c = np.trunc((s.x[out, k] - lo[k]) * (nb[k] / (hi[k] - lo[k]))).astype(int)
        ib.append(np.clip(c, 0, nb[k] - 1))
    key = (ib[2] * nb[1] + ib[1]) * nb[0] + ib[0]
    assert np.all(np.diff(key) >= 0)
    pos = np.empty(s.n, int)
    pos[order] = np.arange(s.n)
    for b in np.unique(key):          # stable: the old order inside every bin
        assert np.all(np.diff(pos[out[key == b]]) > 0)
    big = po.sort_bricks(s, (1, 1, 1), [order], 10.0)[0]
    assert np.array_equal(big, order)


def test_exchange_bricks_moves_atoms_to_their_owner():
    s = bubble_system(8)
    pg = (2, 2, 1)
    own = po.brick_owner(s, s.x, pg)
    local = [np.nonzero(own == r)[0] for r in range(4)]
    rng = np.random.default_rng(1)
    x = s.x + rng.uniform(-0.08, 0.08, s.x.shape)
    x = np.clip(x, s.boxlo, np.nextafter(s.boxhi, -np.inf))
    new = po.exchange_bricks(s, pg, local, x=x)
    own2 = po.brick_owner(s, x, pg)
    assert sorted(np.concatenate(new).tolist()) == list(range(s.n))
    for r in range(4):
        assert np.all(own2[new[r]] == r)
        stay = [i for i in local[r] if own2[i] == r]
        # atoms that never left keep their relative order only where no hole took them
        assert set(stay) <= set(new[r].tolist())


def test_phase_change_meets_candidates_in_local_order():
    """With Atom::sort (default sortfreq 1000) one process meets the candidates in sorted
    order, not in read (tag) order: the same atoms read in two orders create the same atoms
    when the sort runs, other ones when it does not."""
    s = bubble_system(10)
    ph = bubble_physics(10, prob=0.5, Tt=-1.0)
    s1, s2 = shuffled(s, 1), shuffled(s, 2)
    runs = {}
    for name, sm, f in (("a1", s1, 1000), ("a2", s2, 1000), ("b1", s1, 0), ("b2", s2, 0)):
        r = po.MpRefRun(sm, dataclasses.replace(ph, sortfreq=f))
        assert (r.pg == (1, 1, 1)) == (f > 0)
        r.setup()
        r.run(2)
        assert r.ninserted >= 1
        runs[name] = r
    n0 = s.n
    new = lambda r: r.s.x[n0:][np.lexsort(r.s.x[n0:].T)]
    a1, a2, b1, b2 = (runs[k] for k in ("a1", "a2", "b1", "b2"))
    assert a1.ninserted == a2.ninserted
    assert np.abs(new(a1) - new(a2)).max() < 1e-12
    assert not (b1.ninserted == b2.ninserted and np.allclose(new(b1), new(b2)))
    # every view lists its owned atoms in the tracked local order
    bv = a1.bviews[0]
    assert np.array_equal(bv.gid[:bv.nlocal], a1.local[0])
