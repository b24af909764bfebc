"""The oracle's brick emulation (pyoracle.borders_bricks, MpRefRun(procgrid=...)) on the CPU:
a 1x1x1 grid reproduces the single-process CommBrick::borders and fix phase_change exactly,
and on real grids every rank's view is a consistent CommBrick picture (each ghost is the
image of its origin, created atoms lie in their rank's sub-box, mass is conserved where no
created atom lands on a donor's ghost slot)."""
import numpy as np
import pytest

import pyoracle as po
from scenarios import bubble_physics, bubble_system


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
    ph = bubble_physics(10, prob=0.5, Tt=-1.0)
    a = po.MpRefRun(s, ph)
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
