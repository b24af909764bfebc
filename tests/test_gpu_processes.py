"""The engine as several PROCESSES (one brick each) on the one GPU of the test box, against
the oracle.

RCCL refuses two ranks on one device, so every earlier multi-brick test ran the bricks as
threads of one process (LocalWorld).  Here each brick is its own OS process that builds only
its own atoms, exactly as one rank per GPU does; the halos move through the node-local
process world (sph_engine_comm_ipc: hipIpc-exported device outboxes, or host shared memory).
The engine issues the same Transport calls as over RCCL -- borders and migration
(comm_brick.cpp:573-864), the per-step direct forward comm and its peer grouping, the
reverse comm of the setup step and of fix phase_change (:999-1030), the MPI_Allreduce of
nins and the rank-by-rank tag_extend (fix_phase_change.cpp:338-351, atom.cpp:598-630) as
allgathers -- so only the byte mover differs from a multi-GPU run.

Bars: neighbour counts, types, atom counts, insertions exact; fields 1e-10 normwise (C5 on
the jittered slab, the strict bar of tests/test_c5_bricks.py)."""
import json
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

import pyoracle as po
from conftest import check_fields, rel_err
from ipc_rank import c2_scenario, c5_scenario

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TOL = 1e-10


def run_ranks(tmp_path, base, nranks, timeout=240):
    """Start nranks fresh processes (tests/ipc_rank.py) before any HIP call in them, wait,
    and return each rank's snapshots."""
    name = f"/sphipc_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    procs, outs = [], []
    env = dict(os.environ, SPH_IPC_TIMEOUT="90")
    for r in range(nranks):
        spec = dict(base, rank=r, nranks=nranks, name=name,
                    out=str(tmp_path / f"rank{r}.npz"))
        sp = tmp_path / f"spec{r}.json"
        sp.write_text(json.dumps(spec))
        outs.append(spec["out"])
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "ipc_rank.py"),
                                       str(sp)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            logs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r][-3000:]}"
    return [dict(np.load(o)) for o in outs]


def merge(snaps, step, n):
    """The ranks' owned atoms at `step`, by tag (every atom owned exactly once)."""
    out, seen = {}, np.zeros(n, dtype=np.int64)
    for sn in snaps:
        tags = sn[f"{step}/tag"]
        assert tags.size == 0 or (tags.min() >= 0 and tags.max() < n)
        seen[tags] += 1
        for key, v in sn.items():
            pre, _, k = key.partition("/")
            if pre != str(step) or k == "tag" or v.ndim == 0 or v.shape[:1] != tags.shape:
                continue
            if k not in out:
                out[k] = np.zeros((n,) + v.shape[1:], dtype=v.dtype)
            out[k][tags] = v
    assert (seen == 1).all(), "every atom owned by exactly one rank"
    out["nlocal"] = [int(sn[f"{step}/tag"].size) for sn in snaps]
    out["ninserted"] = sum(int(sn.get(f"{step}/ninserted", 0)) for sn in snaps)
    return out


@pytest.mark.parametrize("mode,pg", [(0, (2, 1, 1)), (1, (2, 1, 1)), (0, (1, 2, 2))])
def test_processes_c2_rebuilds_migration(gpu, tmp_path, mode, pg):
    """C2 from rest, 40 steps, rebuilds + migrations every 5 (the brick face at x = 6 is
    crossed), as separate processes; counts bit-exact and fields 1e-10 vs the one-process
    oracle at every snapshot."""
    nsteps = [5, 25, 40]
    P = int(np.prod(pg))
    snaps = run_ranks(tmp_path, dict(scenario="c2", mode=mode, pg=list(pg), snap_steps=nsteps), P)
    s, ph = c2_scenario({})
    ref = po.RefRun(s, ph, spread=True)
    ref.setup()
    side0 = s.x[:, 0] < 6.0
    done = 0
    for k in [0] + nsteps:
        ref.run(k - done)
        done = k
        got = merge(snaps, k, s.n)
        assert sum(got["nlocal"]) == s.n
        assert np.array_equal(got["counts"], ref.numneigh_full()), k
        check_fields(got, ref, ("rho", "f", "drho", "de", "x", "v"), TOL, where=k)
    assert ((ref.s.x[:, 0] < 6.0) != side0).any(), "no atom migrated: migration not exercised"
    assert all(int(sn["staged"]) == 1 for sn in snaps)   # the block path ran on every rank
    assert all(int(sn["nghost"]) > 0 for sn in snaps)


@pytest.mark.parametrize("mode,pg,dim,nx,drift", [(0, (2, 1, 1), 3, 8, 0), (1, (2, 1, 1), 3, 8, 0),
                                                  (0, (2, 2, 1), 2, 12, 0),
                                                  (0, (2, 1, 1), 3, 10, 200.0),
                                                  (1, (2, 2, 1), 2, 16, 200.0)])
def test_processes_c5_phase_change(gpu, tmp_path, mode, pg, dim, nx, drift):
    """C5 (bubble_growth stack + fix phase_change, rebuild every step) on 2 or 4 processes for
    5 steps against pyoracle.MpRefRun(procgrid): per-rank RanPark streams, dmass reverse comm,
    the nins allgather and rank-by-rank tag_extend all cross process boundaries.  drift: atoms
    migrate every step and Atom::sort runs every 2 steps, so every rank's candidates meet the
    stream in a local order that went through exchange hole fills and sorts."""
    nsteps = [1, 2, 3, 4, 5]
    P = int(np.prod(pg))
    spec = dict(scenario="c5", mode=mode, pg=list(pg), nx=nx, dim=dim, snap_steps=nsteps)
    if drift:
        spec.update(drift=drift, sortfreq=2)
    snaps = run_ranks(tmp_path, spec, P)
    s, ph = c5_scenario(spec)
    ref = po.MpRefRun(s, ph, procgrid=pg, spread=True)
    ref.setup()
    for k in [0] + nsteps:
        if k:
            ref.run(1)
        n = ref.s.n
        got = merge(snaps, k, n)
        assert got["ninserted"] == ref.ninserted, k
        assert np.array_equal(got["type"], ref.s.type), k
        assert np.array_equal(got["counts"], ref.numneigh_full()), k
        check_fields(got, ref, ("x", "v", "rho", "e", "rmass", "cv", "cg", "f", "de"), TOL,
                     where=k)
    assert ref.ninserted >= 2, "phase change did not insert across the run"
    if drift:
        moved = po.brick_owner(s, ref.s.x[:s.n], pg) != po.brick_owner(s, s.x, pg)
        assert moved.sum() >= 10, "no atom migrated: the hole fill not exercised"


@pytest.mark.parametrize("mode", [0, 1])
def test_ipc_dead_peer_fails_fast(gpu, tmp_path, mode):
    """A rank that exits after joining the world stops beating: its peer's next barrier
    fails with SPH_HIP_ECOMM after SPH_IPC_DEAD seconds, instead of waiting out a fixed
    timeout (or forever) -- and a long legitimate wait is not mistaken for a dead peer."""
    import time
    name = f"/sphipc_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    env = dict(os.environ, SPH_IPC_DEAD="3")
    procs = []
    t0 = time.time()
    for r in range(2):
        spec = dict(scenario="c2", mode=mode, pg=[2, 1, 1], snap_steps=[1], rank=r, nranks=2,
                    name=name, out=str(tmp_path / f"rank{r}.npz"), die=(r == 1),
                    expect_dead=(r == 0))
        sp = tmp_path / f"spec{r}.json"
        sp.write_text(json.dumps(spec))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "ipc_rank.py"),
                                       str(sp)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=120)
            logs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert procs[1].returncode == 3
    assert procs[0].returncode == 0, logs[0][-3000:]
    assert "PEER_GONE" in logs[0] and "has not beaten" in logs[0], logs[0][-3000:]
    assert time.time() - t0 < 100
    left = [f for f in os.listdir("/dev/shm") if f.startswith(name[1:])]
    assert left == [] or mode == 1, left
