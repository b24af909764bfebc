"""Field parity at the BASELINE sizes: C2 and C3 at 100^3 = 1M particles,
C5 (bubble_growth stack + fix phase_change) at 60^3, engine against the oracle's
reference-faithful drivers (pyoracle.RefRun / MpRefRun) at the north-star bar -- neighbour
counts bit-exact per particle, rho / f / drho / de / x / v / e within 1e-10 normwise.

The size-dependent paths that the small tests only reach by forcing them are taken here
on their own, and asserted through sph_engine_stats: the large-union second launch of the
block force pass (blocks whose union exceeds the pass's LDS image, blk_nbig > 0), and the
inner rows walked between rebuilds (inner_rows / inner_live after the step-10 rebuild).
Reference: pair_sph_rhosum.cpp:66-204, pair_sph_taitwater.cpp:53-200,
pair_sph_taitwater_morris.cpp:52-200, pair_sph_heatconduction.cpp:47-134,
neigh_full.cpp:241-344, fix_phase_change.cpp:167-352."""
import numpy as np
import pytest

import pyoracle as po
from c5_util import mp_engine, mp_state
from conftest import check_fields
from scenarios import bubble_physics, bubble_system, c2_system, c3_system
from test_gpu_engine import compare, engine_for

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _check_block_paths(eng, large):
    st = eng.stats()
    assert st["staged"] == 1, "the block path (production) did not run"
    if large:
        assert st["blk_nbig"] > 0, "no block took the large-union launch"
    assert st["inner_rows"] == 1 and st["inner_live"] == 1, \
        "the pair passes are not walking the inner rows after the rebuild"
    return st


@pytest.mark.parametrize("system,physics,umf", [("c2", po.c2_physics, 0),
                                                ("c3", po.c3_physics, 640)])
def test_full_size_fields(gpu, sph_amd, system, physics, umf):
    """Setup plus 11 steps: the step-10 rebuild and one step on its inner rows.  At 1M the
    Hilbert-sorted blocks' unions all fit the force pass's default LDS image (no second
    launch); the C3 run caps the image at 640 records (sph_engine_tune SPH_TUNE_BLKUMF) so
    that the blocks above it take the large-union launch at full size."""
    s = (c2_system if system == "c2" else c3_system)(100)
    ph = physics()
    ph.every = 10
    eng = engine_for(sph_amd, s, ph)
    if umf:
        eng.tune(eng.TUNE_BLKUMF, umf)
    eng.setup()
    ref = po.RefRun(s, ph, spread="lean")
    ref.setup()
    assert np.array_equal(eng.neighbor_counts(), ref.numneigh_full())
    assert eng.stats()["nghost"] == ref.g.nghost
    compare(eng, ref, path=0)
    eng.run(11)
    ref.run(11)
    assert np.array_equal(eng.neighbor_counts(), ref.numneigh_full())
    compare(eng, ref, path=0)
    st = _check_block_paths(eng, large=umf > 0)
    assert st["step"] == 11 and st["nlocal"] == 100 ** 3


def test_full_size_c5_phase_change(gpu, sph_amd):
    """C5 at 60^3 (216k, rebuild every step, fix phase_change every step on the jittered
    slab: ~500 insertions per step) for 5 steps, compared at every step."""
    nx = 60
    s = bubble_system(nx, slab=True)
    ph = bubble_physics(nx, prob=0.3, Tt=-1.0)
    eng = mp_engine(sph_amd, s, ph)
    eng.setup()
    ref = po.MpRefRun(s, ph, spread=True)
    ref.setup()
    for k in range(6):
        if k:
            eng.run(1)
            ref.run(1)
        g = mp_state(eng)
        rs = ref.s
        assert int(g["ninserted"]) == ref.ninserted, k
        assert np.array_equal(g["type"], rs.type), k
        assert np.array_equal(eng.neighbor_counts(), ref.numneigh_full()), k
        check_fields(g, ref, ("x", "v", "rho", "e", "rmass", "cv", "cg", "f", "de"), TOL,
                     where=k)
    assert ref.ninserted > 1000
