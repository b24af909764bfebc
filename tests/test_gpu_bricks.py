"""GPU parity of the brick decomposition (CommBrick swaps: borders, forward comm, forward
rho, setup reverse comm, exchange/migration at rebuilds) against the single-process oracle
driver.  Several bricks run in one process, one host thread per brick, each its own engine
on the one GPU, exchanging halos through a local world (device copies) -- the same engine
code path the RCCL transport drives across GPUs; only the copy primitive differs.

Per tag: neighbor counts bit-exact, rho/f/drho/de/x/v/e within 1e-10 normwise.

The systems start at rest.  The reference's step-0 force call sees ghost `vest` as it was
at borders() time (borders run before FixMeso::setup_pre_force): with a decomposition the
ghosts of a neighbouring brick are stale, with one process only the periodic images are --
so the reference's own setup forces depend on the processor grid unless v = 0 at setup.
From rest every decomposition must agree with the single-process oracle."""
import threading

import numpy as np
import pytest

import pyoracle as po
from conftest import check_fields, rel_err
from scenarios import c2_system, c3_system

pytestmark = pytest.mark.gpu
TOL = 1e-10


def brick_index(x, lo, hi, pg):
    idx = np.zeros(x.shape[0], dtype=np.int64)
    mult = 1
    for d in range(3):
        prd = hi[d] - lo[d]
        c = np.zeros(x.shape[0], dtype=np.int64)
        for k in range(1, pg[d]):
            c += (x[:, d] >= lo[d] + prd * (k / pg[d])).astype(np.int64)
        idx += c * mult
        mult *= pg[d]
    return idx


def at_rest(s):
    s.v[:] = 0.0
    return s


LAST_STATS = []   # sph_engine_stats of every brick of the last run_bricks


def run_bricks(sph_amd, s, ph, pg, nsteps, every=None, path=0, overlap=False):
    nt = s.ntypes
    P = int(np.prod(pg))
    kw = {}
    if ph.rhosum_nstep > 0:
        kw["rhosum"] = dict(nstep=ph.rhosum_nstep, cut=ph.rhosum_cut)
    if ph.tait:
        kw["tait"] = dict(rho0=ph.rho0, c0=ph.c0, visc=ph.visc, cut=ph.tait_cut, morris=ph.morris)
    if ph.heat:
        kw["heat"] = dict(alpha=ph.alpha, cut=ph.heat_cut)
    world = sph_amd.LocalWorld(P)
    owner = brick_index(s.x, s.boxlo, s.boxhi, pg)
    engines = []
    for r in range(P):
        cfg = sph_amd.make_config(s.dim, nt, s.boxlo, s.boxhi, s.periodic, s.mass, ph.skin, ph.dt,
                                  neigh_every=every or ph.every, kernel_path=path,
                                  procgrid=pg, rank=r, **kw)
        eng = sph_amd.Engine(cfg)
        sel = np.nonzero(owner == r)[0]
        eng.set_atoms(s.x[sel], s.v[sel], s.type[sel], s.rho[sel], s.e[sel], s.cv[sel])
        eng.set_tags(sel)
        eng.comm_local(world, r)
        if overlap:
            eng.tune(eng.TUNE_OVERLAP, 1)
        engines.append(eng)
    errors = []

    def work(eng):
        try:
            eng.setup()
            eng.run(nsteps)
        except Exception as ex:  # surfaced below
            errors.append(ex)

    th = [threading.Thread(target=work, args=(e,)) for e in engines]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "brick threads hung"
    try:
        assert not errors, errors
        LAST_STATS[:] = [e.stats() for e in engines]
        for st in LAST_STATS:  # the requested pair path really ran (no silent fallback)
            assert st["staged"] == (1 if path == 0 else 0)
        return collect(engines, s)
    finally:
        for e in engines:
            e.close()
        world.close()


def collect(engines, s):
    n = s.n
    out = {k: np.zeros((n, 3)) for k in ("x", "v", "f")}
    out.update({k: np.zeros(n) for k in ("rho", "e", "drho", "de")})
    counts = np.zeros(n, dtype=np.int32)
    seen = np.zeros(n, dtype=np.int64)
    nloc = []
    for eng in engines:
        got = eng.get_atoms()
        tags = got["tag"]
        seen[tags] += 1
        for k in out:
            out[k][tags] = got[k]
        counts[tags] = eng.neighbor_counts()
        nloc.append(eng.nlocal)
    assert (seen == 1).all(), "every atom owned by exactly one brick"
    return out, counts, nloc


def compare(out, ref, tol=TOL):
    """normwise 1e-10 and the elementwise bar (conftest.check_fields, the RefRun's reordering
    spread)"""
    check_fields(out, ref, ("rho", "f", "drho", "de", "x", "v"), tol)


PATHS = [0, 1]   # 0 = block-staged LDS unions (production), 1 = row path (global gathers)


@pytest.mark.parametrize("pg,path", [((2, 1, 1), 0), ((1, 2, 2), 0), ((2, 2, 2), 0),
                                     ((2, 1, 1), 1), ((1, 2, 2), 1), ((2, 2, 2), 1)])
def test_bricks_c2_setup_and_run(gpu, sph_amd, pg, path):
    s = at_rest(c2_system(12))
    ph = po.c2_physics()
    ph.every = 4
    ref = po.RefRun(s, ph, spread=True)
    ref.setup()
    ref.run(9)                       # rebuilds (and migrations) at steps 4 and 8
    out, counts, nloc = run_bricks(sph_amd, s, ph, pg, 9, path=path)
    assert sum(nloc) == s.n
    assert np.array_equal(counts, ref.numneigh_full())
    compare(out, ref)


@pytest.mark.parametrize("pg", [(2, 2, 1), (1, 2, 2)])
def test_bricks_nonperiodic(gpu, sph_amd, pg):
    """Bricks with a non-periodic y: the bricks at the y faces send nothing across them
    (sendneed = 0, comm_brick.cpp:226-274) -- the borders' selection runs with an empty slab
    for that swap, while the inner y face between bricks still exchanges."""
    s = at_rest(c2_system(12))
    s.periodic = (1, 0, 1)
    s.boxlo[1] -= 2.0
    s.boxhi[1] += 2.0
    ph = po.c2_physics()
    ph.every = 4
    ref = po.RefRun(s, ph, spread=True)
    ref.setup()
    ref.run(9)
    out, counts, nloc = run_bricks(sph_amd, s, ph, pg, 9)
    assert sum(nloc) == s.n
    assert np.array_equal(counts, ref.numneigh_full())
    compare(out, ref)


@pytest.mark.parametrize("path", PATHS)
def test_bricks_c3_morris_heat(gpu, sph_amd, path):
    s = at_rest(c3_system(12))
    ph = po.c3_physics()
    ph.every = 3
    ref = po.RefRun(s, ph, spread=True)
    ref.setup()
    ref.run(7)
    out, counts, _ = run_bricks(sph_amd, s, ph, (2, 2, 1), 7, path=path)
    assert np.array_equal(counts, ref.numneigh_full())
    compare(out, ref)
    assert rel_err(out["e"], ref.s.e) < TOL


@pytest.mark.parametrize("path", PATHS)
def test_bricks_migration(gpu, sph_amd, path):
    """Pressure-driven motion from rest with a larger step: atoms of the lattice plane that
    sits on the brick face (x = 6) cross it between rebuilds and migrate."""
    s = at_rest(c2_system(12))
    ph = po.c2_physics()
    ph.dt = 5e-3
    ph.every = 5
    ref = po.RefRun(s, ph, spread=True)
    ref.setup()
    ref.run(40)
    side0 = s.x[:, 0] < 6.0
    moved = (ref.s.x[:, 0] < 6.0) != side0
    out, counts, nloc = run_bricks(sph_amd, s, ph, (2, 1, 1), 40, path=path)
    assert moved.any(), "no atom crossed the brick face: the test would not exercise migration"
    assert sum(nloc) == s.n
    assert np.array_equal(counts, ref.numneigh_full())
    compare(out, ref)
    if path == 0:  # the inner rows were derived again between rebuilds (ghosts' x0 too)
        assert sum(st["inner_refresh"] for st in LAST_STATS) > 0


@pytest.mark.parametrize("path", PATHS)
def test_bricks_2d(gpu, sph_amd, path):
    s = at_rest(c2_system(30, dim=2))
    ph = po.c2_physics(2.5)
    ph.every = 4
    ref = po.RefRun(s, ph, spread=True)
    ref.setup()
    ref.run(9)
    out, counts, _ = run_bricks(sph_amd, s, ph, (2, 2, 1), 9, path=path)
    assert np.array_equal(counts, ref.numneigh_full())
    compare(out, ref)


def test_rccl_communicator_single_rank(gpu, sph_amd):
    """sph_engine_comm_uid / comm_init on a one-rank communicator (the RCCL transport's
    setup and teardown; multi-GPU runs use the same calls with one rank per GPU)."""
    s = at_rest(c2_system(8))
    ph = po.c2_physics()
    cfg = sph_amd.make_config(3, 1, s.boxlo, s.boxhi, s.periodic, s.mass, ph.skin, ph.dt,
                              rhosum=dict(nstep=1, cut=ph.rhosum_cut),
                              tait=dict(rho0=ph.rho0, c0=ph.c0, visc=ph.visc, cut=ph.tait_cut),
                              kernel_path=1)
    eng = sph_amd.Engine(cfg)
    eng.set_atoms(s.x, s.v, s.type, s.rho, s.e, s.cv)
    uid = sph_amd.comm_uid()
    assert len(uid) == 128
    eng.comm_init(uid, 1, 0)
    eng.setup()
    eng.run(3)
    assert np.isfinite(eng.get_atoms()["f"]).all()
    eng.close()


@pytest.mark.parametrize("moving,path", [(False, 0), (True, 0), (True, 1)])
def test_rccl_loopback_matches_oracle(gpu, sph_amd, moving, path):
    """The RCCL data path on one GPU: a one-rank communicator in loopback mode sends every
    periodic self swap (border records at rebuilds, the per-step forward x/vest/rho/e and
    rho/EOS halos, the setup reverse comm) through ncclSend/ncclRecv to itself, packed and
    unpacked exactly as between bricks on different GPUs.  Per tag against the oracle:
    neighbor counts bit-exact, fields within 1e-10.  With one brick the ghosts are periodic
    images of the brick's own atoms, so moving particles agree with the oracle too."""
    s = c2_system(12)
    if not moving:
        s = at_rest(s)
    ph = po.c2_physics()
    ph.every = 4
    ref = po.RefRun(s, ph, spread=True)
    ref.setup()
    ref.run(9)
    cfg = sph_amd.make_config(3, 1, s.boxlo, s.boxhi, s.periodic, s.mass, ph.skin, ph.dt,
                              neigh_every=ph.every,
                              rhosum=dict(nstep=1, cut=ph.rhosum_cut),
                              tait=dict(rho0=ph.rho0, c0=ph.c0, visc=ph.visc, cut=ph.tait_cut),
                              kernel_path=path)
    eng = sph_amd.Engine(cfg)
    try:
        eng.set_atoms(s.x, s.v, s.type, s.rho, s.e, s.cv)
        eng.comm_init(sph_amd.comm_uid(), 1, 0)
        eng.comm_loopback(True)
        eng.setup()
        eng.run(9)
        out, counts, _ = collect([eng], s)
    finally:
        eng.close()
    assert np.array_equal(counts, ref.numneigh_full())
    compare(out, ref)


@pytest.mark.parametrize("pg,path", [((2, 1, 1), 1), ((2, 2, 2), 1), ((2, 1, 1), 0),
                                     ((2, 2, 2), 0)])
def test_bricks_halo_overlap(gpu, sph_amd, pg, path):
    """sph_engine_tune(SPH_TUNE_OVERLAP, 1): interior rows' (path 1) or interior blocks'
    (path 0: no ghost in the block's union) rhosum / force passes run on a second stream while
    the forward and rho halos are in flight, the boundary ones after them.  Same per-row
    arithmetic, so the same bar as the serial path: counts bit-exact, fields within 1e-10 of
    the single-process oracle over rebuilds."""
    s = at_rest(c2_system(20 if path == 0 else 14))
    ph = po.c2_physics()
    ph.every = 4
    ref = po.RefRun(s, ph, spread=True)
    ref.setup()
    ref.run(9)
    out, counts, _ = run_bricks(sph_amd, s, ph, pg, 9, path=path, overlap=True)
    assert np.array_equal(counts, ref.numneigh_full())
    compare(out, ref)
    if path == 0:
        st = LAST_STATS[0]
        assert st["staged"] == 1


@pytest.mark.parametrize("path", [1, 0])
def test_rccl_loopback_overlap(gpu, sph_amd, path):
    """The overlapped step through real RCCL send/recv (one-rank loopback), moving particles
    (the block path at 20^3: a brick with interior blocks)."""
    s = c2_system(20 if path == 0 else 12)
    ph = po.c2_physics()
    ph.every = 4
    ref = po.RefRun(s, ph, spread=True)
    ref.setup()
    ref.run(9)
    cfg = sph_amd.make_config(3, 1, s.boxlo, s.boxhi, s.periodic, s.mass, ph.skin, ph.dt,
                              neigh_every=ph.every,
                              rhosum=dict(nstep=1, cut=ph.rhosum_cut),
                              tait=dict(rho0=ph.rho0, c0=ph.c0, visc=ph.visc, cut=ph.tait_cut),
                              kernel_path=path)
    eng = sph_amd.Engine(cfg)
    try:
        eng.set_atoms(s.x, s.v, s.type, s.rho, s.e, s.cv)
        eng.comm_init(sph_amd.comm_uid(), 1, 0)
        eng.comm_loopback(True)
        eng.tune(eng.TUNE_OVERLAP, 1)
        eng.setup()
        eng.run(9)
        out, counts, _ = collect([eng], s)
    finally:
        eng.close()
    assert np.array_equal(counts, ref.numneigh_full())
    compare(out, ref)
