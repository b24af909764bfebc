"""C1 water_collapse (examples/USER/sph/water_collapse/water_collapse.lmp, data.initial):
2-D, 15,702 atoms (9,702 water type 1 + 6,000 boundary type 2), boundary f f p,
hybrid/overlay sph/rhosum 1 (1 1 only) + sph/taitwater (* *), fix gravity -9.81 y on water,
fix meso on water, fix meso/stationary on the boundary, neigh every 5 / skin 0.3 h.
The script's fix dt/reset is not part of the pair path: the runs here use its upper limit
dt = 0.1 h / c as a fixed step.

CPU tests: the fixture, the oracle's integrators against the reference's own FixMeso /
FixMesoStationary (oracle/_ref, where built) and a short oracle run.  GPU tests: the engine
(both pair paths) against the oracle's Verlet driver over 20 steps."""
import numpy as np
import pytest

import pyoracle as po
from scenarios import water_collapse_physics, water_collapse_system

TOL = 1e-10


def test_fixture_matches_data_file_header():
    s = water_collapse_system()
    assert s.n == 15702 and s.dim == 2 and s.ntypes == 2
    assert (s.type == 1).sum() == 9702 and (s.type == 2).sum() == 6000
    assert s.mass[1] == 0.2 and s.mass[2] == 0.1
    assert np.all(s.rho[s.type == 2] == 1000.0) and np.all(s.rho > 500.0)
    assert np.all(s.v == 0.0) and np.all(s.x[:, 2] == 0.0) and np.all(s.cv == 1.0)
    assert s.periodic == (0, 0, 1)


def _ints(rng, n, nt=2):
    t = rng.integers(1, nt + 1, n).astype(np.int32)
    mass = np.array([0.0, 0.2, 0.1])
    arr = {k: rng.normal(size=(n, 3)) for k in ("x", "v", "f", "vest")}
    arr.update({k: rng.uniform(0.5, 2.0, n) for k in ("rho", "drho", "e", "de")})
    return t, mass, arr


@pytest.mark.parametrize("stationary,phase,tmask", [(0, 0, 2), (0, 1, 2), (0, 2, 2),
                                                    (1, 1, 4), (1, 2, 4), (0, 1, 0)])
def test_integrators_match_reference_fixes(stationary, phase, tmask):
    R = po.ref() if po.ref_available() else None
    if R is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    L = po.lib()
    rng = np.random.default_rng(3 + 10 * stationary + phase)
    n, dt = 500, 3e-4
    t, mass, a = _ints(rng, n)
    want = {k: v.copy() for k, v in a.items()}
    assert R.ref_fix_meso(stationary, phase, n, 2, dt, t, tmask, mass, want["x"], want["v"],
                          want["f"], want["vest"], want["rho"], want["drho"], want["e"],
                          want["de"]) == 0
    got = {k: v.copy() for k, v in a.items()}
    dtf = 0.5 * dt
    if stationary:
        L.orc_meso_stationary(n, dtf, t, tmask, got["rho"], got["drho"], got["e"], got["de"])
    elif phase == 0:
        L.orc_meso_setup_g(n, t, tmask, got["v"], got["vest"])
    elif phase == 1:
        L.orc_meso_initial_g(n, dt, dtf, t, tmask, mass, None, got["x"], got["v"], got["f"],
                             got["vest"], got["rho"], got["drho"], got["e"], got["de"])
    else:
        L.orc_meso_final_g(n, dtf, t, tmask, mass, None, got["v"], got["f"], got["rho"],
                           got["drho"], got["e"], got["de"])
    for k in ("x", "v", "vest", "rho", "e"):
        assert np.array_equal(got[k], want[k]), k
    if stationary:  # meso/stationary leaves x, v, vest alone, integrates e and rho
        inn = ((tmask >> t) & 1).astype(bool)
        for k in ("x", "v", "vest"):
            assert np.array_equal(got[k], a[k])
        assert not np.allclose(got["rho"][inn], a["rho"][inn])


def test_oracle_water_collapse_short_run():
    s = water_collapse_system()
    ph = water_collapse_physics()
    ref = po.RefRun(s, ph)
    ref.setup()
    ref.run(5)
    bc = s.type == 2
    # boundary atoms never move; water picks up the downward pull
    assert np.array_equal(ref.s.x[bc], s.x[bc]) and np.all(ref.s.v[bc] == 0.0)
    assert ref.s.v[~bc, 1].mean() < 0.0
    # rhosum recomputes only the water's rho; the boundary's rho is integrated
    assert np.all(np.isfinite(ref.s.rho)) and not np.allclose(ref.s.rho[bc], 1000.0)
    assert np.all(ref.numneigh_full() > 0)


@pytest.mark.gpu
@pytest.mark.parametrize("path", [0, 1])
def test_engine_water_collapse_20_steps(gpu, sph_amd, path):
    from test_gpu_engine import compare, engine_for
    s = water_collapse_system()
    ph = water_collapse_physics()
    ref = po.RefRun(s, ph, spread=True)
    ref.setup()
    ref.run(20)
    eng = engine_for(sph_amd, s, ph, kernel_path=path)
    eng.setup()
    eng.run(20)
    assert np.array_equal(eng.neighbor_counts(), ref.numneigh_full())
    got = compare(eng, ref, TOL, path=path)
    bc = s.type == 2
    assert np.array_equal(got["x"][bc], s.x[bc])
