"""Benchmark of the MI355X USER-SPH engine on BASELINE.json's headline workload.

    python bench.py [--gpus N] [--scaling strong|weak] [--steps K] [--warmup W] [--edge 100]
                    [--no-cpu] [--workload c2|c3|c5|c2pair|c5pair]

Workload (BASELINE.json configs[1]): 1M particles on a jittered 100^3 cubic lattice,
periodic, hybrid/overlay sph/rhosum (nstep 1, h 3) + sph/taitwater (rho0 1, c0 10,
visc 0.1, h 3), skin 0.3, neighbor rebuild every 10 steps, dt 1e-3, fix meso.  A "step"
is one full Verlet step of the device-resident engine (integrate, forward comm or
rebuild, rhosum, forward rho, taitwater, integrate) with everything already in HBM.

N > 1: one rank per GPU (LAMMPS' CommBrick spatial decomposition, halo exchange and
migration over RCCL/xGMI).  Without WORLD_SIZE in the environment, `--gpus N` starts the N
ranks itself (fresh child processes, before anything touches the GPU); under
torch.distributed.run WORLD_SIZE must equal --gpus.
  --scaling strong (default): the ONE 1M-particle C2 box split into N bricks (the
      north star's "1M particles at 1/2/4/8 GPUs"; 125k particles per GPU at N = 8);
  --scaling weak: every brick holds an edge^3 share of a box edge*procgrid per side
      (N = 8 is BASELINE config C4: 200^3 = 8M particles on 2x2x2 GPUs).
Rank 0 prints ONE JSON line.  `roofline` covers the dominant kernel (the taitwater force
pass), timed live with HIP events recorded on the engine's stream; `cpu_baseline` is the
reference's own compute code timed on this host on a bounded sample (rank 0, N = 1 only).
"""
import argparse
import importlib.util
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def load_pkg():
    spec = importlib.util.spec_from_file_location(
        "sph_amd", os.path.join(ROOT, "lammps-sph-multiphase_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["sph_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def make_system(n, seed):
    """Same construction as oracle/pyoracle.cubic_lattice."""
    x, v, t, rho, e, cv, _ = brick_lattice(n, (1, 1, 1), 0, seed)
    return x, v, t, rho, e, cv


def procgrid_for(nranks):
    """Brick grid for nranks: least total face area, x >= y >= z (2 -> 2x1x1, 8 -> 2x2x2)."""
    best = None
    for px in range(1, nranks + 1):
        if nranks % px:
            continue
        for py in range(1, nranks // px + 1):
            if (nranks // px) % py:
                continue
            pz = nranks // (px * py)
            if not (px >= py >= pz):
                continue
            area = px * py + py * pz + px * pz
            if best is None or area < best[0]:
                best = (area, (px, py, pz))
    return best[1]


def brick_lattice(n, pg, rank, seed=12345):
    """Rank `rank`'s n^3 share of the global (n*pg)-per-side jittered sc lattice, with the
    global tags of its sites.  pg = (1,1,1), rank 0 is exactly the single-box C2 system."""
    loc = (rank % pg[0], (rank // pg[0]) % pg[1], rank // (pg[0] * pg[1]))
    g = np.stack(np.meshgrid(np.arange(n), np.arange(n), np.arange(n), indexing="ij"), -1)
    g = g.reshape(-1, 3)
    g = g[np.lexsort((g[:, 0], g[:, 1], g[:, 2]))]   # create_atoms order: z, y, x
    g = g + np.array(loc) * n
    x = g.astype(np.float64)
    x += np.random.default_rng(seed + rank).uniform(-0.1, 0.1, size=x.shape)
    v = np.random.default_rng(4928459 + rank).normal(0.0, 0.01, size=x.shape)
    N = x.shape[0]
    NX, NY = n * pg[0], n * pg[1]
    tags = ((g[:, 2] * NY + g[:, 1]) * NX + g[:, 0]).astype(np.int32)
    return x, v, np.ones(N, np.int32), np.ones(N), np.zeros(N), np.ones(N), tags


def strong_lattice(n, pg, rank, seed=12345):
    """Rank `rank`'s brick of the single-box C2 system (n^3 sites, box [0, n)^3): the atoms
    whose position falls in the brick (uniform split, bricks numbered x fastest); the
    union over ranks is exactly make_system(n).  Tags are the global site indices."""
    x, v, t, rho, e, cv, tags = brick_lattice(n, (1, 1, 1), 0, seed)
    loc = np.array((rank % pg[0], (rank // pg[0]) % pg[1], rank // (pg[0] * pg[1])))
    w = np.array([n / p for p in pg])
    b = np.clip(np.floor(x / w).astype(int), 0, np.array(pg) - 1)
    sel = (b == loc).all(axis=1)
    return x[sel], v[sel], t[sel], rho[sel], e[sel], cv[sel], tags[sel]


def free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n):
    """Start n ranks of this script as fresh processes (one per GPU, RANK/LOCAL_RANK/
    WORLD_SIZE/MASTER_* set as torch.distributed.run would) and wait for them; if one fails
    the others are stopped.  Returns the exit code.  Nothing here touches the GPU."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:          # exact PIDs we started, never a pattern
                    q.terminate()
        time.sleep(0.05)
    return rc


def share_uid(dist, rank, make_uid):
    """RCCL unique id from rank 0 to every rank (torch.distributed object broadcast)."""
    obj = [make_uid() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def attach_comm(eng, sph, args, dist, rank, world):
    """The communicator of a multi-rank run: RCCL (default: one rank per GPU, ncclSend/Recv
    over xGMI) or the node-local process world (--transport ipc: hipIpc-exported device
    outboxes; ipc-host: host shared memory), which lets several ranks share one GPU (RCCL
    refuses that).  The name / unique id goes from rank 0 to every rank the same way."""
    if args.transport == "rccl":
        eng.comm_init(share_uid(dist, rank, sph.comm_uid), world, rank)
    else:
        name = share_uid(dist, rank, lambda: f"/sphbench_{os.getpid()}_{time.time_ns() % 10**9}")
        eng.comm_ipc(name, world, rank, 0 if args.transport == "ipc" else 1)


def transport_name(args):
    return {"rccl": "RCCL", "ipc": "hipIpc process-world",
            "ipc-host": "host-shared-memory process-world"}[args.transport]


class stdout_to_stderr:
    """RCCL prints its version banner on fd 1 at communicator init; keep stdout for the one
    JSON line of the bench contract."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def c2_config(sph, n, pg=(1, 1, 1), rank=0, strong=False):
    """C2 physics; the box is n per side split into pg bricks (strong) or n*pg per side
    (weak: an n^3 share per brick)."""
    h = 3.0
    cut = np.zeros((2, 2))
    cut[1, 1] = h
    visc = np.zeros((2, 2))
    visc[1, 1] = 0.1
    side = [float(n) for p in pg] if strong else [float(n * p) for p in pg]
    return sph.make_config(3, 1, [0.0, 0.0, 0.0], side, [1, 1, 1],
                           [0.0, 1.0], 0.3, 1e-3, neigh_every=10, rhosum=dict(nstep=1, cut=cut),
                           tait=dict(rho0=np.array([0.0, 1.0]), c0=np.array([0.0, 10.0]),
                                     visc=visc, cut=cut), procgrid=pg, rank=rank)


def cpu_baseline(n_cpu, steps=2):
    """CPU baseline on the same C2 workload at n_cpu^3 particles, one core.

    kind "reference": the reference's own USER-SPH compute code (oracle/_ref/libsph_ref.so,
    compiled from /root/reference/src by oracle/build_ref.sh -- PairSPHRhoSum::compute,
    PairSPHTaitwater::compute, Neighbor::full_bin, half_from_full_newton): rhosum on the
    full list + taitwater on the half list, `steps` times, plus one list build amortised over
    neigh_every = 10.  Falls back to the oracle's C restatement (kind "port")."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    s = po.cubic_lattice(n_cpu)
    ph = po.c2_physics()
    R = po.ref() if po.ref_available() else None
    if R is None:
        run = po.RefRun(s, ph)
        run.setup()
        t0 = time.perf_counter()
        run.run(steps)                       # steps 1..steps: forward comm, no rebuild
        t_steps = (time.perf_counter() - t0) / steps
        t0 = time.perf_counter()
        run._build()
        t_build = time.perf_counter() - t0
        per_step = t_steps + t_build / 10.0
        return {"value": s.n / per_step, "unit": "particle-steps/s", "cores": 1, "kind": "port",
                "sample": f"oracle/sph_oracle.c (scalar C restatement) on {s.n} particles "
                          f"(same C2 physics): {steps} steps timed ({t_steps:.3f} s/step) + one "
                          f"neighbor rebuild ({t_build:.2f} s) amortised over neigh_every=10"}
    cns, cmax = po.cutneighsq(1, ph.cutmax(1), ph.skin)
    g = po.borders(s, cmax)
    args = (3, 1, g.nlocal, g.nghost, np.ascontiguousarray(g.x), g.type, s.boxlo, s.boxhi,
            s.boxlo, s.boxhi, cmax, np.ascontiguousarray(cns))
    t0 = time.perf_counter()
    foff = np.zeros(g.nlocal + 1, dtype=np.int64)
    tot = R.ref_neigh_full(*args, foff, None, 0)
    fnb = np.zeros(tot, dtype=np.int32)
    R.ref_neigh_full(*args, foff, fnb.ctypes.data, tot)
    hoff = np.zeros(g.nlocal + 1, dtype=np.int64)
    htot = R.ref_neigh_half_from_full(g.nlocal, g.nghost, g.x, foff, fnb, hoff, None)
    hnb = np.zeros(htot, dtype=np.int32)
    R.ref_neigh_half_from_full(g.nlocal, g.nghost, g.x, foff, fnb, hoff, hnb.ctypes.data)
    t_build = (time.perf_counter() - t0) / 2.0   # two passes of full_bin (count + fill)
    rho = g.gather(s.rho)
    vest = g.gather(s.v)
    f = np.zeros((g.nall, 3))
    drho = np.zeros(g.nall)
    de = np.zeros(g.nall)
    cut = np.ascontiguousarray(ph.tait_cut)
    visc = np.ascontiguousarray(ph.visc)
    t_rho = t_tait = 0.0
    for _ in range(steps):
        t0 = time.perf_counter()
        R.ref_rhosum(3, 1, g.nlocal, g.nghost, g.x, g.type, s.mass, cut, foff, fnb, rho)
        t1 = time.perf_counter()
        R.ref_taitwater(3, 1, g.nlocal, g.nghost, 1, g.x, vest, rho, g.type, s.mass, ph.rho0,
                        ph.c0, visc, cut, hoff, hnb, f, drho, de)
        t2 = time.perf_counter()
        t_rho += (t1 - t0) / steps
        t_tait += (t2 - t1) / steps
    per_step = t_rho + t_tait + t_build / 10.0
    return {"value": s.n / per_step, "unit": "particle-steps/s", "cores": 1,
            "kind": "reference",
            "sample": f"reference USER-SPH compute code (oracle/_ref, built from the reference "
                      f"sources, g++ -O3) on {s.n} particles, same C2 inputs: "
                      f"PairSPHRhoSum::compute {t_rho:.3f} s + PairSPHTaitwater::compute "
                      f"{t_tait:.3f} s per step (mean of {steps}) + Neighbor::full_bin + "
                      f"half_from_full_newton {t_build:.2f} s amortised over neigh_every=10; "
                      f"comm/integrate (<1%) not included",
            "pair_only_particle_steps_per_s": s.n / (t_rho + t_tait)}


def _brick_cpu_worker(a):
    """One brick of cpu_baseline_cores, in its own process: the reference's list build and
    rhosum + taitwater on the brick's owned + ghost atoms (borders_bricks), per step."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    R = po.ref()
    x, typ, nlocal, nghost, lo, hi, cmax, cns, rho, vest, mass, cut, visc, rho0, c0, steps = a
    args = (3, 1, nlocal, nghost, x, typ, lo, hi, lo, hi, cmax, cns)
    t0 = time.perf_counter()
    foff = np.zeros(nlocal + 1, dtype=np.int64)
    tot = R.ref_neigh_full(*args, foff, None, 0)
    fnb = np.zeros(max(tot, 1), dtype=np.int32)
    R.ref_neigh_full(*args, foff, fnb.ctypes.data, tot)
    hoff = np.zeros(nlocal + 1, dtype=np.int64)
    htot = R.ref_neigh_half_from_full(nlocal, nghost, x, foff, fnb, hoff, None)
    hnb = np.zeros(max(htot, 1), dtype=np.int32)
    R.ref_neigh_half_from_full(nlocal, nghost, x, foff, fnb, hoff, hnb.ctypes.data)
    t_build = (time.perf_counter() - t0) / 2.0
    nall = nlocal + nghost
    f, drho, de = np.zeros((nall, 3)), np.zeros(nall), np.zeros(nall)
    t0 = time.perf_counter()
    for _ in range(steps):
        R.ref_rhosum(3, 1, nlocal, nghost, x, typ, mass, cut, foff, fnb, rho)
        R.ref_taitwater(3, 1, nlocal, nghost, 1, x, vest, rho, typ, mass, rho0, c0, visc, cut,
                        hoff, hnb, f, drho, de)
    return (time.perf_counter() - t0) / steps + t_build / 10.0


def host_cores():
    """The cores this process may run on: its CPU affinity set, capped by OMP_NUM_THREADS
    where that is set (the GPU pool's boxes give a GPU's job 16 cores of a larger machine,
    whose os.cpu_count() shows them all)"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS", "")
    if cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_baseline_cores(n_cpu, nproc=8, steps=2):
    """The C2 CPU baseline on nproc cores as LAMMPS runs it with MPI: the n_cpu^3 box split
    into nproc bricks (2x2x2 at 8, CommBrick::borders ghosts, pyoracle.borders_bricks), each
    brick's reference list build + rhosum + taitwater in its own process at the same time;
    per step = the slowest brick (halo exchange and reverse comm, ~1 % on one core, not
    timed).  Processes are spawned (not forked: the parent holds a HIP context)."""
    import multiprocessing as mpc
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    if not po.ref_available():
        return None
    s = po.cubic_lattice(n_cpu)
    ph = po.c2_physics()
    cns, cmax = po.cutneighsq(1, ph.cutmax(1), ph.skin)
    pg = procgrid_for(nproc)
    work = []
    for v in po.borders_bricks(s, cmax, pg):
        work.append((np.ascontiguousarray(v.x), np.ascontiguousarray(v.type), v.nlocal, v.nghost,
                     np.asarray(v.lo, float), np.asarray(v.hi, float), cmax,
                     np.ascontiguousarray(cns), np.ascontiguousarray(s.rho[v.gid]),
                     np.ascontiguousarray(s.v[v.gid]), s.mass, np.ascontiguousarray(ph.tait_cut),
                     np.ascontiguousarray(ph.visc), ph.rho0, ph.c0, steps))
    with mpc.get_context("spawn").Pool(nproc) as pool:
        per = pool.map(_brick_cpu_worker, work)
    t = max(per)
    return {"value": s.n / t, "unit": "particle-steps/s", "cores": nproc, "kind": "reference",
            "host_cpus_visible": os.cpu_count(),
            "sample": f"reference USER-SPH compute code (oracle/_ref) on {s.n} particles split "
                      f"into {pg[0]}x{pg[1]}x{pg[2]} bricks, one process per brick running at "
                      f"the same time (LAMMPS' MPI decomposition): list build / 10 + rhosum + "
                      f"taitwater per step, slowest brick {t:.3f} s (bricks "
                      f"{min(per):.3f}-{t:.3f} s); halo exchange not timed"}


# ---- C3: two-phase Morris + heat conduction on the engine ----------
C3_MASS, C3_RHO0, C3_E = (1.0, 0.5), (1.0, 0.5), (1.0, 2.0)


def c3_system(n, seed=12345, tseed=87287):
    """C2's lattice with type 2 by Bernoulli(0.5) (seed 87287), m = (1, 0.5), rho = rho0 =
    (1, 0.5), e = (1, 2) by type, cv = 1 -- as oracle/pyoracle.cubic_lattice(ntypes=2)."""
    x, v, t, rho, e, cv, _ = brick_lattice(n, (1, 1, 1), 0, seed)
    t[np.random.default_rng(tseed).random(t.shape[0]) < 0.5] = 2
    rho = np.where(t == 1, C3_RHO0[0], C3_RHO0[1])
    e = np.where(t == 1, C3_E[0], C3_E[1])
    return x, v, t, rho, e, cv


def c3_tables(h=3.0):
    cut = np.zeros((3, 3))
    cut[1:, 1:] = h
    visc = np.zeros((3, 3))
    visc[1:, 1:] = 0.01
    alpha = np.zeros((3, 3))
    alpha[1:, 1:] = 0.1
    return cut, visc, alpha


def c3_config(sph, n):
    cut, visc, alpha = c3_tables()
    return sph.make_config(3, 2, [0.0, 0.0, 0.0], [float(n)] * 3, [1, 1, 1],
                           [0.0, C3_MASS[0], C3_MASS[1]], 0.3, 1e-3, neigh_every=10,
                           tait=dict(rho0=np.array([0.0, *C3_RHO0]),
                                     c0=np.array([0.0, 10.0, 10.0]), visc=visc, cut=cut,
                                     morris=True),
                           heat=dict(alpha=alpha, cut=cut))


def c3_cpu_baseline(n_cpu, steps=2):
    """The reference's own PairSPHTaitwaterMorris::compute + PairSPHHeatConduction::compute
    (oracle/_ref, 1 core) on the C3 input at n_cpu^3 particles, half list, plus one
    Neighbor::full_bin + half_from_full_newton amortised over neigh_every = 10."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    if not po.ref_available():
        return None
    R = po.ref()
    x, v, t, rho, e, cv = c3_system(n_cpu)
    s = po.cubic_lattice(n_cpu, ntypes=2, type2_frac=0.5, mass=C3_MASS, rho=C3_RHO0, e=C3_E)
    assert np.array_equal(s.type, t) and np.array_equal(s.x, x)
    cut, visc, alpha = c3_tables()
    cns, cmax = po.cutneighsq(2, cut, 0.3)
    g = po.borders(s, cmax)
    args = (3, 2, g.nlocal, g.nghost, np.ascontiguousarray(g.x), g.type, s.boxlo, s.boxhi,
            s.boxlo, s.boxhi, cmax, np.ascontiguousarray(cns))
    t0 = time.perf_counter()
    foff = np.zeros(g.nlocal + 1, dtype=np.int64)
    tot = R.ref_neigh_full(*args, foff, None, 0)
    fnb = np.zeros(tot, dtype=np.int32)
    R.ref_neigh_full(*args, foff, fnb.ctypes.data, tot)
    hoff = np.zeros(g.nlocal + 1, dtype=np.int64)
    htot = R.ref_neigh_half_from_full(g.nlocal, g.nghost, g.x, foff, fnb, hoff, None)
    hnb = np.zeros(htot, dtype=np.int32)
    R.ref_neigh_half_from_full(g.nlocal, g.nghost, g.x, foff, fnb, hoff, hnb.ctypes.data)
    t_build = (time.perf_counter() - t0) / 2.0
    rho_all, e_all, vest = g.gather(s.rho), g.gather(s.e), g.gather(s.v)
    f = np.zeros((g.nall, 3))
    drho = np.zeros(g.nall)
    de = np.zeros(g.nall)
    rho0 = np.array([0.0, *C3_RHO0])
    c0 = np.array([0.0, 10.0, 10.0])
    t_m = t_h = 0.0
    for _ in range(steps):
        t0 = time.perf_counter()
        R.ref_taitwater_morris(3, 2, g.nlocal, g.nghost, 1, g.x, vest, rho_all, g.type, s.mass,
                               rho0, c0, visc, cut, hoff, hnb, f, drho, de)
        t1 = time.perf_counter()
        R.ref_heatconduction(3, 2, g.nlocal, g.nghost, 1, g.x, e_all, rho_all, g.type, s.mass,
                             alpha, cut, hoff, hnb, de)
        t2 = time.perf_counter()
        t_m += (t1 - t0) / steps
        t_h += (t2 - t1) / steps
    per_step = t_m + t_h + t_build / 10.0
    return {"value": s.n / per_step, "unit": "particle-steps/s", "cores": 1,
            "kind": "reference",
            "sample": f"reference USER-SPH compute code (oracle/_ref, g++ -O3) on {s.n} "
                      f"particles, same C3 inputs: PairSPHTaitwaterMorris::compute {t_m:.3f} s "
                      f"+ PairSPHHeatConduction::compute {t_h:.3f} s per step (mean of {steps}) "
                      f"+ Neighbor::full_bin + half_from_full_newton {t_build:.2f} s amortised "
                      f"over neigh_every=10; comm/integrate not included"}


def c3_main(args, sph):
    """Config 3 (BASELINE.json configs[2]): 1M particles, two types, sph/taitwater/morris +
    sph/heatconduction, the device-resident engine step on one GPU."""
    n = args.edge
    x, v, t, rho, e, cv = c3_system(n)
    eng = sph.Engine(c3_config(sph, n))
    eng.set_atoms(x, v, t, rho, e, cv)
    eng.setup()
    eng.run(args.warmup)
    eng.sync()
    eng.set_timing(True, classes=(eng.T_RHO, eng.T_TAIT))  # (the fused pass, as C2)
    t0 = time.perf_counter()
    eng.run(args.steps)
    eng.sync()
    elapsed = time.perf_counter() - t0
    st = eng.stats()
    eng.set_timing(True)  # the other classes over 10 more steps, outside the timed region
    eng.run(10)
    eng.sync()
    st_x = eng.stats()
    nloc = st["nlocal"]
    n_half = st["nbr_full"] / max(nloc, 1) / 2.0
    # morris 104 + 4 N_h, heat 56 + 4 N_h (fused here into one pass)
    bytes_pass = 160.0 + 8.0 * n_half
    ms_pass = st["ms_tait"] / max(st["n_tait"], 1)
    ach = bytes_pass * nloc / (ms_pass * 1e-3) / 1e9
    out = {
        "metric": "particle-steps/s + achieved HBM GB/s, 1M-particle taitwater+rhosum, 1/2/4/8 GPUs",
        "value": n ** 3 * args.steps / elapsed,
        "unit": "particle-steps/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (jittered sc lattice, Bernoulli(0.5) types, gaussian velocities, seeded)",
        "config": {"workload": f"C3: {n ** 3} particles cubic lattice, two types, "
                               "sph/taitwater/morris + sph/heatconduction, periodic, skin 0.3, "
                               "rebuild every 10",
                   "particles_per_gpu": nloc, "ghosts_per_gpu": st["nghost"],
                   "n_half_per_particle": n_half, "parallelism": "single GPU"},
        "roofline": {"bound": "hbm",
                     "kernel": ("k_blk_force" if st["staged"] == 1 else "k_row2_force")
                               + "<MORRIS, TAIT|HEAT> (taitwater/morris + heatconduction, "
                               "one fused pass)",
                     "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": ach / PEAK_HBM_GBS, "traffic": None,
                     "bytes_per_particle": bytes_pass, "ms_per_launch": ms_pass},
        "kernels": {"neighbor_build_ms": st_x["ms_neigh"] / max(st_x["n_neigh"], 1),
                    "integrate_ms_per_step": st_x["ms_integrate"] / 10,
                    "comm_ms_per_step": st_x["ms_comm"] / 10,
                    "timing_note": "fused pass: HIP events in the timed region; the rest: 10 "
                                   "further steps with every class timed"},
    }
    if not args.no_cpu:
        cb = c3_cpu_baseline(args.cpu_n)
        if cb is not None:
            out["cpu_baseline"] = cb
    print(json.dumps(out), flush=True)
    eng.close()


# ---- C5 multiphase pair passes (SURVEY.md 8(d) C5 physics, 8(a) rows a6-a8 + 8(f) rank 2) --
def kd_lists(x, rc):
    """Full and half (i < j) CSR lists of all pairs within rc (k-d tree; open boundaries)."""
    from scipy.spatial import cKDTree
    N = x.shape[0]
    pairs = cKDTree(x).query_pairs(rc, output_type="ndarray")
    pairs = pairs[np.lexsort((pairs[:, 1], pairs[:, 0]))]
    hoff = np.zeros(N + 1, dtype=np.int64)
    np.add.at(hoff, pairs[:, 0] + 1, 1)
    half = (np.cumsum(hoff), pairs[:, 1].astype(np.int32))
    both = np.concatenate([pairs, pairs[:, ::-1]])
    del pairs
    both = both[np.lexsort((both[:, 1], both[:, 0]))]
    foff = np.zeros(N + 1, dtype=np.int64)
    np.add.at(foff, both[:, 0] + 1, 1)
    return (np.cumsum(foff), both[:, 1].astype(np.int32)), half


def c2_pair_main(args, sph):
    """The headline styles through the drop-in pair-style layer, as LAMMPS calls them:
    sph/rhosum on its FULL list (pair_sph_rhosum.cpp:57-62), sph/taitwater on the default
    HALF list with newton on (Newton-3 j share gathered through the reverse half list),
    C2 physics, lists within h + skin.  Device time of the kernels (HIP events); the per-call
    PCIe staging of a LAMMPS-driven call is reported separately."""
    n = args.edge
    x, v, t, rho, e, cv = make_system(n, 12345)
    N = x.shape[0]
    (foff, fnb), (hoff, hnb) = kd_lists(x, 3.3)
    h = 3.0
    cut = np.zeros((2, 2))
    cut[1, 1] = h
    visc = np.zeros((2, 2))
    visc[1, 1] = 0.1
    mass = np.array([0.0, 1.0])
    rho0, c0 = np.array([0.0, 1.0]), np.array([0.0, 10.0])
    ctx = sph.PairContext(3, 1, 1)
    ctx.atoms(N, 0, x, t, vest=v, rho=rho, e=e)
    ctx.rhosum_coeff(cut, mass)
    ctx.taitwater_coeff(rho0, c0, c0 ** 2 * rho0 / 7.0, visc, cut, mass)
    r = np.zeros(N)
    f, drho, de = np.zeros((N, 3)), np.zeros(N), np.zeros(N)

    def step(first_half_call_after_upload=True):
        ms = {}
        t0 = time.perf_counter()
        ctx.list_csr(sph.SPH_LIST_FULL, foff, fnb)
        ctx.rhosum(r)
        ms["rhosum"] = ctx.last_kernel_ms()
        ctx.list_csr(sph.SPH_LIST_HALF, hoff, hnb)
        ctx.taitwater(f, drho, de)
        ms["taitwater"] = ctx.last_kernel_ms()   # includes the reverse-list build
        ctx.taitwater(f, drho, de)
        ms["taitwater_list_reused"] = ctx.last_kernel_ms()
        return ms, time.perf_counter() - t0

    # the calling pattern of a LAMMPS run with the sph/<style>/hip shim: every compute()
    # restages the atoms (sph_hip_atoms) and stages its NeighList keyed by the build
    # (sph_hip_list_keyed, key = neighbor->ncalls); a rebuild every `every` steps
    nl_full, nl_half = sph.NeighList(foff, fnb), sph.NeighList(hoff, hnb)
    every = 10
    cns = np.zeros((2, 2))
    cns[1, 1] = 3.3 * 3.3   # Neighbor::cutneighsq = (h + skin)^2

    xs, vs, rs, es = (np.ascontiguousarray(a, dtype=np.float64).copy() for a in (x, v, rho, e))
    dl_parts = {}

    def lammps_step(k, device_lists):
        t0 = time.perf_counter()
        key = k // every
        if not device_lists:
            ctx.atoms(N, 0, x, t, vest=v, rho=rho, e=e)
            ctx.list_neighlist(sph.SPH_LIST_FULL, nl_full, key)
            ctx.rhosum(r)
            kms = ctx.last_kernel_ms()
            ctx.atoms_rho(rho)     # (same step: the shim restages rho only)
            ctx.list_neighlist(sph.SPH_LIST_HALF, nl_half, key)
            ctx.taitwater(f, drho, de)
            return time.perf_counter() - t0, kms + ctx.last_kernel_ms()
        # the shim's device-list path: LAMMPS' arrays registered as mapped host memory (once,
        # sph_hip_host_arrays), the whole atom set restaged at a rebuild, positions / vest /
        # rho / e between rebuilds (sph_hip_atoms_update), the lists built on the device at a
        # new key (sph_hip_build_list), rho written and f / drho / de added in place
        rb = k % every == 0
        tt = [t0]

        def lap():
            tt.append(time.perf_counter())
        if rb:
            ctx.atoms(N, 0, xs, t, vest=vs, rho=rs, e=es)
        else:
            ctx.atoms_update(xs, vest=vs, rho=rs, e=es)
        lap()
        ctx.build_list(sph.SPH_LIST_FULL, cns, key)
        lap()
        ctx.rhosum(rs)
        kms = ctx.last_kernel_ms()
        lap()
        ctx.atoms_rho(rs)
        lap()
        ctx.build_list(sph.SPH_LIST_HALF, cns, key)
        lap()
        ctx.taitwater(f, drho, de)
        lap()
        part = dl_parts.setdefault("rebuild" if rb else "reuse", [0, [0.0] * 6])
        part[0] += 1
        for i in range(6):
            part[1][i] += (tt[i + 1] - tt[i]) * 1e3
        return tt[-1] - t0, kms + ctx.last_kernel_ms()

    for _ in range(args.warmup):
        step()
    ctx.set_timing(True)
    acc, wall = {}, 0.0
    for _ in range(args.steps):
        ms, w = step()
        wall += w
        for k, val in ms.items():
            acc[k] = acc.get(k, 0.0) + val / args.steps
    nls = max(args.steps, every) // every * every   # whole rebuild periods
    pattern = {}
    for dl in (False, True):
        if dl:
            ctx.host_arrays(N, x=xs, vest=vs, rho=rs, e=es, f=f, drho=drho, de=de)
            for k in range(2):   # (untimed: first-use allocations of the device-list buffers)
                lammps_step(2000 + k, dl)
            dl_parts.clear()
        lw, lk = 0.0, 0.0
        for k in range(nls):
            w, km = lammps_step(k + (1000 if dl else 0), dl)
            lw += w
            lk += km
        pattern[dl] = (lw, lk)
    lw, lk = pattern[False]
    n_full, n_half = foff[-1] / N, hoff[-1] / N
    by = {"rhosum": 40 + 4 * n_half, "taitwater": 104 + 4 * n_half}
    by["taitwater_list_reused"] = by["taitwater"]
    kern = {k: {"ms_per_call": acc[k], "bytes_per_particle": by[k],
                "achieved_GBs": by[k] * N / (acc[k] * 1e-3) / 1e9} for k in acc}
    t_dev = (acc["rhosum"] + acc["taitwater"]) * 1e-3
    out = {
        "metric": "kernel particle-steps/s, C2 rhosum + taitwater via the pair-style layer",
        "value": N / t_dev, "unit": "particle-steps/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": t_dev * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (jittered sc lattice, gaussian velocities, seeded)",
        "config": {"workload": f"C2 physics on {N} particles, open box, rhosum on the full list "
                               "+ taitwater on the half list (newton on), lists within h + skin "
                               "= 3.3; the taitwater call after a list upload includes the "
                               "reverse half-list build",
                   "n_full_per_particle": n_full, "n_half_per_particle": n_half,
                   "wall_ms_per_step_incl_pcie": wall / args.steps * 1e3,
                   "lammps_pattern": {
                       "what": "per step: sph_hip_atoms + sph_hip_list_keyed(FULL) + rhosum, "
                               "sph_hip_atoms_rho + sph_hip_list_keyed(HALF) + taitwater; lists "
                               f"rebuilt every {every} steps (key = build)",
                       "steps": nls,
                       "wall_ms_per_step_incl_pcie": lw / nls * 1e3,
                       "kernel_ms_per_step": lk / nls,
                       "wall_over_kernel": lw * 1e3 / max(lk, 1e-12)},
                   "lammps_pattern_device_lists": {
                       "what": "the shim's device-list path: LAMMPS' arrays registered as "
                               "mapped host memory (sph_hip_host_arrays), sph_hip_atoms at a "
                               "rebuild else sph_hip_atoms_update, sph_hip_build_list FULL / "
                               "HALF at each new key (no host list copy or upload), rho "
                               "written and f / drho / de added in place by the device",
                       "wall_ms_by_call": {
                           kind: dict(zip(("atoms", "build_full", "rhosum", "atoms_rho",
                                           "build_half", "taitwater"),
                                          [round(v / c, 4) for v in tot]), steps=c)
                           for kind, (c, tot) in dl_parts.items()},
                       "steps": nls,
                       "wall_ms_per_step_incl_pcie": pattern[True][0] / nls * 1e3,
                       "kernel_ms_per_step": pattern[True][1] / nls,
                       "wall_over_kernel": pattern[True][0] * 1e3 / max(pattern[True][1], 1e-12)}},
        "roofline": {"bound": "hbm", "kernel": "taitwater (half list: forward + reverse "
                                               "gather)",
                     "achieved": kern["taitwater"]["achieved_GBs"], "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": kern["taitwater"]["achieved_GBs"] / PEAK_HBM_GBS,
                     "traffic": None},
        "kernels": kern,
    }
    print(json.dumps(out), flush=True)
    ctx.close()


def c5_pair_system(n, seed=2024):
    """Two-phase n^3 block (bubble_growth physics in dx = 1 units: h = 3, rho_l = 1,
    rho_v = 0.1, c = 200/sqrt(rho), eta 1 / 0.69, gamma 1, rbackground 0, cv 0.04 / 0.06):
    a vapour sphere (type 2, radius n/4) in liquid (type 1), jittered sc lattice, open
    boundaries (no ghosts).  Full and half (i < j) lists within h from a k-d tree."""
    rng = np.random.default_rng(seed)
    g = np.stack(np.meshgrid(np.arange(n), np.arange(n), np.arange(n), indexing="ij"), -1)
    x = g.reshape(-1, 3).astype(np.float64) + rng.uniform(-0.1, 0.1, size=(n ** 3, 3))
    c = (n - 1) / 2.0
    vap = np.linalg.norm(x - c, axis=1) < n / 4.0
    ty = np.where(vap, 2, 1).astype(np.int32)
    rho0 = np.where(vap, 0.1, 1.0)
    d = dict(x=x, type=ty, rmass=rho0.copy(), rho=rho0 * (1 + 0.01 * rng.uniform(-1, 1, n ** 3)),
             cv=np.where(vap, 0.06, 0.04), vest=rng.normal(0.0, 0.01, size=x.shape))
    d["e"] = d["cv"] * np.where(vap, 0.1, 0.02) * (1 + 0.1 * rng.uniform(-1, 1, n ** 3))
    h = 3.0
    (d["full_off"], d["full_nbr"]), (d["half_off"], d["half_nbr"]) = kd_lists(x, h)
    t2 = lambda a11, a12, a22: np.array([[0, 0, 0], [0, a11, a12], [0, a12, a22]], float)
    cl, cvap = 200.0, 200.0 / np.sqrt(0.1)
    d.update(h=h, cut=t2(h, h, h), rho0=np.array([0.0, 1.0, 0.1]),
             c0=np.array([0.0, cl, cvap]), gamma=np.array([0.0, 1.0, 1.0]),
             rbg=np.zeros(3), visc=t2(1.0, 2 * 0.69 / 1.69, 0.69),
             cg_alpha=t2(0.0, 1.0, 0.0), alpha=t2(0.1, 2 * 0.1 * 0.05 / 0.15, 0.05),
             fixflag=np.array([[0, 0, 0], [0, 0, 2], [0, 2, 0]], np.int32), tc=t2(0, 0.0, 0))
    return d


def c5_pair_bytes(n_half, n_full):
    """Compulsory bytes per particle of each pass (SURVEY.md 8(d) convention: each array read
    or written once, int32 CSR, fp64; x 24, v 24, rho 8, rmass 8, type 4, e 8, cv 8, cg 24)."""
    return {"rhosum/multiphase": 24 + 4 + 8 + 4 + 4 * n_full + 8,
            "colorgradient": 24 + 4 + 8 + 8 + 4 + 4 * n_full + 24,
            "taitwater/multiphase": 24 + 24 + 8 + 8 + 4 + 4 + 4 * n_half + 24,
            "surfacetension": 24 + 24 + 8 + 8 + 4 + 4 + 4 * n_half + 24,
            "heatconduction/phasechange": 24 + 8 + 8 + 8 + 8 + 4 + 4 + 4 * n_half + 8}


def c5_pair_main(args, sph):
    """The C5 pair passes through the pair-style layer (sph_hip_* entry points), the calls a
    LAMMPS run of bubble_growth's hybrid/overlay makes per step: rhosum/multiphase and
    colorgradient on the full list, taitwater/multiphase, surfacetension and
    heatconduction/phasechange on the half list.  `value` is particle-steps/s of the five
    passes' DEVICE time (HIP events around the kernels; inputs staged once, so the per-call
    PCIe staging a LAMMPS run adds is excluded and reported separately)."""
    n = args.edge
    d = c5_pair_system(n)
    N = d["x"].shape[0]
    ctx = sph.PairContext(3, 2, 1)
    ctx.atoms(N, 0, d["x"], d["type"], vest=d["vest"], rho=d["rho"], e=d["e"])
    ctx.atoms_multiphase(d["rmass"], d["cv"])
    ctx.rhosum_multiphase_coeff(d["cut"])
    ctx.colorgradient_coeff(d["cg_alpha"], d["cut"])
    ctx.taitwater_multiphase_coeff(d["rho0"], d["c0"], d["gamma"], d["rbg"], d["visc"], d["cut"])
    ctx.surfacetension_coeff(d["cut"])
    ctx.heatconduction_phasechange_coeff(d["alpha"], d["cut"], fixflag=d["fixflag"], tc=d["tc"])
    rho, cg = np.zeros(N), np.zeros((N, 3))
    f, de = np.zeros((N, 3)), np.zeros(N)

    def step():
        ms = {}
        t0 = time.perf_counter()
        ctx.list_csr(sph.SPH_LIST_FULL, d["full_off"], d["full_nbr"])
        ctx.rhosum_multiphase(rho)
        ms["rhosum/multiphase"] = ctx.last_kernel_ms()
        ctx.colorgradient(cg)
        ms["colorgradient"] = ctx.last_kernel_ms()
        ctx.list_csr(sph.SPH_LIST_HALF, d["half_off"], d["half_nbr"])
        ctx.taitwater_multiphase(f)
        ms["taitwater/multiphase"] = ctx.last_kernel_ms()
        ctx.surfacetension(cg, f)
        ms["surfacetension"] = ctx.last_kernel_ms()
        ctx.heatconduction_phasechange(de)
        ms["heatconduction/phasechange"] = ctx.last_kernel_ms()
        return ms, time.perf_counter() - t0

    for _ in range(args.warmup):
        step()
    ctx.set_timing(True)
    acc = {}
    wall = 0.0
    for _ in range(args.steps):
        ms, w = step()
        wall += w
        for k, v in ms.items():
            acc[k] = acc.get(k, 0.0) + v / args.steps
    t_dev = sum(acc.values()) * 1e-3
    n_full = d["full_off"][-1] / N
    n_half = d["half_off"][-1] / N
    by = c5_pair_bytes(n_half, n_full)
    kern = {k: {"ms_per_call": acc[k], "bytes_per_particle": by[k],
                "achieved_GBs": by[k] * N / (acc[k] * 1e-3) / 1e9} for k in acc}
    dom = max(acc, key=acc.get)
    out = {
        "metric": "kernel particle-steps/s, C5 multiphase pair passes (pair-style layer)",
        "value": N / t_dev, "unit": "particle-steps/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": t_dev * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic two-phase block (vapour sphere in liquid), seeded",
        "config": {"workload": f"C5 pair passes: {N} particles, bubble_growth physics (h = 3 dx), "
                               "open box, rhosum/multiphase + colorgradient (full list), "
                               "taitwater/multiphase + surfacetension + "
                               "heatconduction/phasechange (half list, newton on)",
                   "n_full_per_particle": n_full, "n_half_per_particle": n_half,
                   "wall_ms_per_step_incl_pcie": wall / args.steps * 1e3},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": kern[dom]["achieved_GBs"],
                     "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": kern[dom]["achieved_GBs"] / PEAK_HBM_GBS, "traffic": None},
        "kernels": kern,
    }
    if not args.no_cpu:
        out["cpu_baseline"] = c5_pair_cpu(d)
    print(json.dumps(out), flush=True)
    ctx.close()


def c5_pair_cpu(d):
    """The reference's own compute() of the five styles (oracle/_ref) on the same input, one
    core, one call each."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    if not po.ref_available():
        return None
    R = po.ref()
    N = d["x"].shape[0]
    x, ty, rm = np.ascontiguousarray(d["x"]), d["type"], d["rmass"]
    nz = lambda a: a if a.size else np.zeros(1, np.int32)
    cut = d["cut"]
    B = d["c0"] ** 2 * d["rho0"] / np.where(d["gamma"] > 0, d["gamma"], 1.0)
    t = {}
    t0 = time.perf_counter()
    rho = d["rho"].copy()
    R.ref_rhosum_multiphase(3, 2, N, 0, x, ty, rm, cut, d["full_off"], nz(d["full_nbr"]), rho)
    t["rhosum/multiphase"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    cg = np.zeros((N, 3))
    R.ref_colorgradient(3, 2, N, 0, x, d["rho"], rm, ty, d["cg_alpha"], cut, d["full_off"],
                        nz(d["full_nbr"]), cg)
    t["colorgradient"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    f = np.zeros((N, 3))
    R.ref_taitwater_multiphase(3, 2, N, 0, 1, x, d["vest"], d["rho"], ty, rm, d["rho0"],
                               d["c0"], d["gamma"], d["rbg"], d["visc"], cut, d["half_off"],
                               nz(d["half_nbr"]), f)
    t["taitwater/multiphase"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    R.ref_surfacetension(3, 2, N, 0, 1, x, d["rho"], rm, ty, cg, cut, d["half_off"],
                         nz(d["half_nbr"]), f)
    t["surfacetension"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    de = np.zeros(N)
    R.ref_heatconduction_phasechange(3, 2, N, 0, 1, x, d["e"], d["cv"], d["rho"], rm, ty,
                                     d["alpha"], d["fixflag"].ctypes.data, d["tc"].ctypes.data,
                                     cut, d["half_off"], nz(d["half_nbr"]), de)
    t["heatconduction/phasechange"] = time.perf_counter() - t0
    tot = sum(t.values())
    return {"value": N / tot, "unit": "particle-steps/s", "cores": 1, "kind": "reference",
            "sample": f"reference compute() of the five styles (oracle/_ref) on the same "
                      f"{N} particles, one call each: " +
                      ", ".join(f"{k} {v:.3f} s" for k, v in t.items())}


def c5_system(n, dim=3, rv=0.05):
    """BASELINE C5 geometry (examples/USER/sph/bubble_growth/bubble.lmp, vars.lmp, in.phases):
    unit box, lattice sc dx = 1/n with origin 0.5, liquid (type 1), vapour (type 2) inside the
    script's 'region rsq sphere ... 0.05' at the centre; rho_l 1, rho_v 0.1, cv 0.04 / 0.06,
    e = cv T (T_l = Tinf = 1, T_v = Tc = 0), rmass = dx^dim rho (in.phases 'set type mass')."""
    dx = 1.0 / n
    nz = n if dim == 3 else 1
    g = np.stack(np.meshgrid(np.arange(n), np.arange(n), np.arange(nz), indexing="ij"),
                 -1).reshape(-1, 3)
    g = g[np.lexsort((g[:, 0], g[:, 1], g[:, 2]))]
    x = (g + 0.5) * dx
    if dim == 2:
        x[:, 2] = 0.0
    c = np.array([0.5, 0.5, 0.5 if dim == 3 else 0.0])
    vap = ((x - c) ** 2).sum(1) < rv * rv
    t = np.where(vap, 2, 1).astype(np.int32)
    rho = np.where(vap, 0.1, 1.0)
    cv = np.where(vap, 0.06, 0.04)
    e = np.where(vap, 0.0, 0.04)
    return x, np.zeros_like(x), t, rho, e, cv, rho * dx ** dim


def c5_physics(n, dim=3):
    """bubble.lmp:57-73 pair stack with vars.lmp values (h = 3 dx, neighbor 0 bin, every 1),
    dt = the min of settimestep.lmp's limits, fix phase_change Tc 0 Tt 0.1 Hwv 8 dr dx/2
    mass_v h 1 2 1 123456 0.01."""
    dx = 1.0 / n
    h = 3.0 * dx
    rho_l, rho_v, cv_l, cv_v = 1.0, 0.1, 0.04, 0.06
    c_l, c_v = 200.0 / np.sqrt(rho_l), 200.0 / np.sqrt(rho_v)
    eta_l, eta_v, D_l, D_v, alpha = 1.0, 0.69, 0.2, 0.6, 500.0
    t2 = lambda a11, a12, a22: np.array([[0, 0, 0], [0, a11, a12], [0, a12, a22]], float)
    hh = t2(h, h, h)
    mp = dict(rhosum_nstep=1, rhosum_cut=hh, cg_nstep=1, cg_alpha=t2(0.0, alpha, 0.0),
              cg_cut=hh, rho0=[0.0, rho_l, rho_v], c0=[0.0, c_l, c_v], gamma=[0.0, 1.0, 1.0],
              rbg=[0.0, 0.0, 0.0], visc=t2(eta_l, 2 * eta_l * eta_v / (eta_l + eta_v), eta_v),
              tait_cut=hh, st_cut=hh,
              heat_alpha=t2(D_l, 2 * D_l * D_v / (D_l + D_v), D_v), heat_cut=hh,
              heat_fixflag=np.array([[0, 0, 0], [0, 0, 2], [0, 2, 0]]), heat_tc=t2(0, 0, 0))
    beta = 0.1
    dt = min(beta * 1.44 * rho_v * cv_v * dx ** 2 / D_v, beta * 1.44 * rho_l * cv_l * dx ** 2 / D_l,
             dx * dx / (8.0 * eta_v) * rho_v, dx * dx / (8.0 * eta_l) * rho_l,
             0.25 * np.sqrt(rho_v * dx ** 3 / (6 * alpha)), 0.25 * np.sqrt(rho_l * dx ** 3 / (6 * alpha)),
             0.25 * dx / c_v, 0.25 * dx / c_l)
    pc = dict(Tc=0.0, Tt=0.1, Hwv=8.0, dr=0.5 * dx, to_mass=dx ** dim * rho_v, cutoff=h,
              from_type=1, to_type=2, nevery=1, seed=123456, prob=0.01)
    return mp, dt, pc


def brick_of(x, boxlo, boxhi, pg):
    """The rank owning each position on a uniform brick grid, ranks x fastest: sublo <= x <
    subhi with the engine's split points (sph_engine_create, CommBrick::exchange)."""
    r = np.zeros(x.shape[0], dtype=np.int64)
    mult = 1
    for d in range(3):
        prd = boxhi[d] - boxlo[d]
        c = np.zeros(x.shape[0], dtype=np.int64)
        for k in range(1, pg[d]):
            c += (x[:, d] >= boxlo[d] + prd * (k / pg[d])).astype(np.int64)
        r += c * mult
        mult *= pg[d]
    return r


def c5_main(args, sph, dist=None, rank=0, world=1, dev=0):
    """C5 on the device-resident engine: the bubble_growth stack + fix phase_change,
    rebuilding every step as the script does.  One GPU: the largest single-GPU C5, 159^3 =
    4.02M.  N GPUs: the same 4.02M box split into bricks (strong scaling; BASELINE C5 is this
    box over 8 GPUs), every rank running fix phase_change on its own atoms with its own
    random stream, dmass reverse comm and tag_extend over RCCL.  `value` = particle-steps/s
    of the whole step (integration, phase change, exchange, borders, list build, the five
    pair passes), all ranks, max-over-ranks time."""
    n = args.edge
    x, v, t, rho, e, cv, rmass = c5_system(n)
    mp, dt, pc = c5_physics(n)
    N = x.shape[0]
    pg = procgrid_for(world)
    cfg = sph.make_config(3, 2, [0.0] * 3, [1.0] * 3, [1, 1, 1], [0.0, 1.0, 1.0], 0.0, dt,
                          neigh_every=1, mp=mp, procgrid=pg, rank=rank)
    eng = sph.Engine(cfg, device=dev)
    if world > 1:
        sel = np.nonzero(brick_of(x, [0.0] * 3, [1.0] * 3, pg) == rank)[0]
        eng.set_atoms(x[sel], v[sel], t[sel], rho[sel], e[sel], cv[sel])
        eng.set_atoms_multiphase(rmass[sel], cv[sel])
        eng.set_tags(sel.astype(np.int32))
    else:
        eng.set_atoms(x, v, t, rho, e, cv)
        eng.set_atoms_multiphase(rmass, cv)
    eng.phase_change(pc["Tc"], pc["Tt"], pc["Hwv"], pc["dr"], pc["to_mass"], pc["cutoff"],
                     pc["from_type"], pc["to_type"], nevery=pc["nevery"], seed=pc["seed"],
                     prob=pc["prob"])
    def barrier():
        if dist is not None:
            dist.barrier()

    with stdout_to_stderr():
        if world > 1:
            attach_comm(eng, sph, args, dist, rank, world)
        eng.setup()
        eng.run(args.warmup)
    eng.sync()
    barrier()
    eng.sync()
    eng.set_timing(True, classes=(eng.T_RHO, eng.T_TAIT))  # (the pair passes only, as C2)
    t0 = time.perf_counter()
    eng.run(args.steps)
    eng.sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    st = eng.stats()
    eng.set_timing(True)  # the other classes over 3 more steps, outside the timed region
    eng.run(3)
    eng.sync()
    st_x = eng.stats()
    nloc = st["nlocal"]
    n_full = st["nbr_full"] / max(nloc, 1)
    n_half = n_full / 2.0
    by = c5_pair_bytes(n_half, n_full)
    # rhosum/multiphase summed inside the list fill (stats flags bit 0, the production
    # default): its time is in the neighbour build, so the T_RHO class -- colorgradient and
    # the rho store -- carries the colorgradient bytes only
    rho_fused = bool(st["flags"] & 1)
    b_full = by["colorgradient"] + (0.0 if rho_fused else by["rhosum/multiphase"])
    b_half = by["taitwater/multiphase"] + by["surfacetension"] + by["heatconduction/phasechange"]
    ms_full = st["ms_rhosum"] / max(st["n_rhosum"], 1)
    ms_half = st["ms_tait"] / max(st["n_tait"], 1)
    ach_half = b_half * nloc / (ms_half * 1e-3) / 1e9
    ach_full = b_full * nloc / (ms_full * 1e-3) / 1e9
    ins = int(eng.get_atoms_multiphase()["ninserted"])
    if dist is not None:
        import torch
        tt = torch.tensor([ins], dtype=torch.int64)
        dist.all_reduce(tt)
        ins = int(tt.item())
    par = (f"spatial decomposition {pg[0]}x{pg[1]}x{pg[2]}, {transport_name(args)} halo exchange "
           "+ migration + fix phase_change dmass reverse comm and tag_extend, one rank per GPU"
           if world > 1 else "single GPU")
    out = {
        "metric": "particle-steps/s, C5 bubble_growth multiphase stack + fix phase_change",
        "value": N * args.steps / elapsed, "unit": "particle-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (bubble_growth geometry: sc lattice, vapour sphere r 0.05)",
        "config": {"workload": f"C5: {N} particles ({n}^3), bubble_growth/bubble.lmp stack "
                               "(rhosum/multiphase, colorgradient, taitwater/multiphase, "
                               "surfacetension, heatconduction/phasechange) + fix phase_change "
                               "every step, rebuild every step, skin 0",
                   "particles_per_gpu": nloc, "ghosts_per_gpu": st["nghost"],
                   "n_full_per_particle": n_full, "n_half_per_particle": n_half,
                   "atoms_inserted": ins, "dt": dt, "parallelism": par},
        "roofline": {"bound": "hbm",
                     "kernel": "k_mp2_gather (taitwater/multiphase + surfacetension + "
                               "heatconduction/phasechange fused: full-list gather, each pair "
                               "in its half-list orientation; the symmetric-style gather of "
                               "sph_mp2_kernels.h, every gamma equal as bubble.lmp)",
                     "achieved": ach_half, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": ach_half / PEAK_HBM_GBS, "traffic": None,
                     "bytes_per_particle": b_half, "ms_per_launch": ms_half},
        "kernels": {("full-list pass (colorgradient; rhosum/multiphase fused into the list "
                     "fill, timed with the neighbour build)" if rho_fused else
                     "full-list passes (rhosum/multiphase + colorgradient)"):
                        {"ms_per_step": ms_full, "achieved_GBs": ach_full,
                         "bytes_per_particle": b_full},
                    "neighbor_build_and_phase_change_ms": st_x["ms_neigh"] / max(st_x["n_neigh"], 1),
                    "integrate_ms_per_step": st_x["ms_integrate"] / 3,
                    "comm_ms_per_step": st_x["ms_comm"] / 3,
                    "timing_note": "pair passes: HIP events in the timed region; neighbor "
                                   "build / phase change, integrate, comm: 3 further steps "
                                   "with every class timed"},
    }
    attach_pmc_traffic(out, "k_mp2_gather", b_half * nloc, world, args,
                       fname="pmc_traffic_c5.json")
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = c5_cpu_baseline(args.c5_cpu_n, steps=1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    with stdout_to_stderr():
        eng.close()
    if dist is not None:
        dist.destroy_process_group()


def c5_cpu_baseline(n_cpu, steps=2):
    """The same C5 step in the reference's own code (oracle/_ref, one core) on the same
    bubble geometry at n_cpu^3 particles: Neighbor::full_bin + half_from_full_newton (the
    script rebuilds every step), the five pair styles' compute(), and FixPhaseChange::
    pre_exchange, `steps` times; borders/comm and FixMeso (<1 %) are not timed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes as C
    import pyoracle as po
    if not po.ref_available():
        return None
    R = po.ref()
    x, v, ty, rho, e, cv, rmass = c5_system(n_cpu)
    mp, dt, pc = c5_physics(n_cpu)
    N = x.shape[0]
    s = po.System(3, np.zeros(3), np.ones(3), (1, 1, 1), x, v, ty, rho, e, cv, 2, np.zeros(3),
                  rmass=rmass)
    h = float(mp["rhosum_cut"][1, 1])
    cut = np.ascontiguousarray(mp["rhosum_cut"])
    cns, cmax = po.cutneighsq(2, cut, 0.0)
    g = po.borders(s, cmax)
    gx = np.ascontiguousarray(g.x)
    nz = lambda a: a if a.size else np.zeros(1, np.int32)
    d = {k: np.ascontiguousarray(g.gather(a)) for k, a in
         dict(v=v, rho=rho, e=e, cv=cv, rmass=rmass).items()}
    rho0, c0 = np.array(mp["rho0"], float), np.array(mp["c0"], float)
    gam, rbg = np.array(mp["gamma"], float), np.array(mp["rbg"], float)
    visc = np.ascontiguousarray(mp["visc"], dtype=float)
    alpha = np.ascontiguousarray(mp["cg_alpha"], dtype=float)
    halpha = np.ascontiguousarray(mp["heat_alpha"], dtype=float)
    ff = np.ascontiguousarray(mp["heat_fixflag"], dtype=np.int32)
    tc = np.ascontiguousarray(mp["heat_tc"], dtype=float)
    args = ["pc", "all", "phase_change", repr(pc["Tc"]), repr(pc["Tt"]), repr(pc["Hwv"]),
            repr(pc["dr"]), repr(pc["to_mass"]), repr(pc["cutoff"]), "1", "2", "1",
            str(pc["seed"]), repr(pc["prob"]), "region", "box", "units", "box"]
    av = (C.c_char_p * len(args))(*[a.encode() for a in args])
    hnd = R.ref_pc_new(3, 2, s.boxlo, s.boxhi, 0, dt, len(args), av)
    t = dict(list=0.0, pair=0.0, pc=0.0)
    for step in range(steps):
        t0 = time.perf_counter()
        args_n = (3, 2, g.nlocal, g.nghost, gx, g.type, s.boxlo, s.boxhi, s.boxlo, s.boxhi,
                  cmax, np.ascontiguousarray(cns))
        foff = np.zeros(g.nlocal + 1, dtype=np.int64)
        tot = R.ref_neigh_full(*args_n, foff, None, 0)
        fnb = np.zeros(max(tot, 1), dtype=np.int32)
        R.ref_neigh_full(*args_n, foff, fnb.ctypes.data, tot)
        hoff = np.zeros(g.nlocal + 1, dtype=np.int64)
        htot = R.ref_neigh_half_from_full(g.nlocal, g.nghost, gx, foff, fnb, hoff, None)
        hnb = np.zeros(max(htot, 1), dtype=np.int32)
        R.ref_neigh_half_from_full(g.nlocal, g.nghost, gx, foff, fnb, hoff, hnb.ctypes.data)
        t1 = time.perf_counter()
        t["list"] += (t1 - t0) / 2.0   # (two full_bin passes: count + fill)
        rr = d["rho"].copy()
        cg = np.zeros((g.nall, 3))
        f = np.zeros((g.nall, 3))
        de = np.zeros(g.nall)
        t0 = time.perf_counter()
        R.ref_rhosum_multiphase(3, 2, g.nlocal, g.nghost, gx, g.type, d["rmass"], cut, foff,
                                nz(fnb), rr)
        R.ref_colorgradient(3, 2, g.nlocal, g.nghost, gx, d["rho"], d["rmass"], g.type, alpha,
                            cut, foff, nz(fnb), cg)
        R.ref_taitwater_multiphase(3, 2, g.nlocal, g.nghost, 1, gx, d["v"], d["rho"], g.type,
                                   d["rmass"], rho0, c0, gam, rbg, visc, cut, hoff, nz(hnb), f)
        R.ref_surfacetension(3, 2, g.nlocal, g.nghost, 1, gx, d["rho"], d["rmass"], g.type, cg,
                             cut, hoff, nz(hnb), f)
        R.ref_heatconduction_phasechange(3, 2, g.nlocal, g.nghost, 1, gx, d["e"], d["cv"],
                                         d["rho"], d["rmass"], g.type, halpha, ff.ctypes.data,
                                         tc.ctypes.data, cut, hoff, nz(hnb), de)
        t["pair"] += time.perf_counter() - t0
        nmax = g.nall + 4096
        A = {}
        for k, src in (("x", gx), ("v", d["v"]), ("vest", d["v"]), ("cg", cg)):
            A[k] = np.zeros((nmax, 3))
            A[k][:g.nall] = src
        for k in ("e", "rmass", "rho", "cv"):
            A[k] = np.zeros(nmax)
            A[k][:g.nall] = d[k]
        A["type"] = np.zeros(nmax, np.int32)
        A["type"][:g.nall] = g.type
        nr = C.c_long(0)
        t0 = time.perf_counter()
        R.ref_pc_pre_exchange(hnd, step + 1, g.nlocal, g.nghost, nmax, A["x"], A["v"], A["vest"],
                              A["cg"], A["e"], A["rmass"], A["rho"], A["cv"], A["type"], foff,
                              nz(fnb), len(g.swap_first) - 1, g.swap_first, nz(g.src),
                              C.byref(nr))
        t["pc"] += time.perf_counter() - t0
    per = {k: v / steps for k, v in t.items()}
    tot = sum(per.values())
    return {"value": N / tot, "unit": "particle-steps/s", "cores": 1, "kind": "reference",
            "sample": f"reference code (oracle/_ref, g++ -O3, one core) on the same C5 bubble "
                      f"geometry at {n_cpu}^3 = {N} particles, per step (mean of {steps}): "
                      f"Neighbor::full_bin + half_from_full_newton {per['list']:.3f} s, the five "
                      f"pair styles' compute() {per['pair']:.3f} s, FixPhaseChange::pre_exchange "
                      f"{per['pc']:.4f} s; borders/comm and FixMeso not timed"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="N > 1: strong = the one edge^3 box split into N bricks (default); "
                         "weak = an edge^3 share per GPU (C4 at N = 8)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--edge", type=int, default=None,
                    help="lattice edge (default 100; c5pair 80: C5's ~0.5M particles per GPU)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-n", type=int, default=100)
    ap.add_argument("--c5-cpu-n", type=int, default=100,
                    help="c5: edge of the two-phase block the reference's five styles are "
                         "timed on for cpu_baseline (100^3 = 1M: ~35 s for the one timed "
                         "step on one core, the largest size that fits a minute)")
    ap.add_argument("--workload", choices=["c2", "c3", "c5", "c2pair", "c5pair"], default="c2",
                    help="c2: the headline engine step (default); c3: two-phase Morris + "
                         "heat conduction engine step (config 3); c5: the bubble_growth "
                         "multiphase stack + fix phase_change on the engine (--edge 159 = "
                         "4.02M, the largest single-GPU C5); c2pair: rhosum + taitwater "
                         "through the pair-style layer; c5pair: the multiphase pair passes "
                         "through the pair-style layer (--edge sets n^3)")
    ap.add_argument("--path", type=int, default=int(os.environ.get("SPH_PATH", "0")),
                    help="pair-kernel path (sph_engine_config.kernel_path): 0 = block-staged "
                         "(production), 1 = row path")
    ap.add_argument("--comm-loopback", action="store_true",
                    help="one GPU: route the periodic self swaps through a one-rank RCCL "
                         "communicator (send/recv to itself) -- the multi-GPU halo path's cost "
                         "without the xGMI transfer")
    ap.add_argument("--overlap", action="store_true",
                    help="bricks / loopback: interior blocks' (rows') pair passes on a second "
                         "stream while the halos move (sph_engine_tune SPH_TUNE_OVERLAP)")
    ap.add_argument("--transport", choices=["rccl", "ipc", "ipc-host"], default="rccl",
                    help="N > 1: rccl = one rank per GPU over RCCL/xGMI (default); ipc / "
                         "ipc-host = the node-local process world (hipIpc device outboxes / "
                         "host shared memory), ranks may share a GPU")
    ap.add_argument("--dry-run", action="store_true",
                    help="host path only (rank launch, decomposition, timing reduction), no "
                         "HIP device: prints the JSON line with value null")
    args = ap.parse_args()
    assert args.gpus >= 1

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    assert world == args.gpus, f"WORLD_SIZE={world} but --gpus {args.gpus}"
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    sph = None if args.dry_run else load_pkg()
    ndev = 0 if args.dry_run else sph.device_count()
    assert args.dry_run or ndev > 0, "bench.py needs a HIP device"
    if args.workload in ("c2pair", "c5pair"):
        assert world == 1, "the pair-layer workloads run on one GPU"
        args.edge = args.edge or 80
        return (c2_pair_main if args.workload == "c2pair" else c5_pair_main)(args, sph)
    if args.workload == "c5":
        args.edge = args.edge or 159
        return c5_main(args, sph, dist, rank, world, local % max(ndev, 1))
    args.edge = args.edge or 100
    if args.workload == "c3":
        assert world == 1, "the C3 workload runs on one GPU"
        return c3_main(args, sph)
    dev = local % max(ndev, 1)

    strong = args.scaling == "strong" and world > 1
    pg = procgrid_for(world)
    if strong:
        x, v, t, rho, e, cv, tags = strong_lattice(args.edge, pg, rank)
        n_total = args.edge ** 3
    else:
        x, v, t, rho, e, cv, tags = brick_lattice(args.edge, pg, rank)
        n_total = args.edge ** 3 * world

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(val):
        if dist is None:
            return val
        import torch
        tt = torch.tensor([val], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    if strong:
        workload = (f"C2 strong scaling: one {args.edge}^3 = {n_total} particle cubic lattice "
                    f"split into {pg[0]}x{pg[1]}x{pg[2]} bricks (~{n_total // world} per GPU), "
                    "sph/rhosum + sph/taitwater, periodic, skin 0.3, rebuild every 10")
    elif world > 1:
        workload = (f"C2 weak scaling: {args.edge ** 3} particles/GPU, one "
                    f"{args.edge * pg[0]}x{args.edge * pg[1]}x{args.edge * pg[2]} box in "
                    f"{pg[0]}x{pg[1]}x{pg[2]} bricks (BASELINE C4 at 8 GPUs), sph/rhosum + "
                    "sph/taitwater, periodic, skin 0.3, rebuild every 10")
    else:
        workload = (f"C2: {args.edge ** 3} particles cubic lattice, sph/rhosum + "
                    "sph/taitwater, periodic, skin 0.3, rebuild every 10")
    parallelism = (("single GPU, halos through RCCL loopback" if args.comm_loopback
                    else "single GPU") if world == 1 else
                   f"spatial decomposition {pg[0]}x{pg[1]}x{pg[2]}, {transport_name(args)} halo exchange + "
                   "migration, one rank per GPU")
    if args.overlap:
        parallelism += ", interior blocks' pair passes overlapped with the halo exchanges"
    base = {
        "metric": "particle-steps/s + achieved HBM GB/s, 1M-particle taitwater+rhosum, 1/2/4/8 GPUs",
        "unit": "particle-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (jittered sc lattice, gaussian velocities, seeded)",
    }

    if args.dry_run:
        counts = [None] * world
        if dist is not None:
            dist.all_gather_object(counts, int(x.shape[0]))
        else:
            counts = [int(x.shape[0])]
        barrier()
        elapsed = max_over_ranks(0.0)
        if rank == 0:
            out = dict(base, value=None, ms_per_step=elapsed, dry_run=True,
                       config={"workload": workload, "parallelism": parallelism,
                               "particles_per_rank": counts, "particles_total": sum(counts)})
            print(json.dumps(out), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    cfg = c2_config(sph, args.edge, pg, rank, strong=strong)
    cfg.kernel_path = args.path
    eng = sph.Engine(cfg, device=dev)
    if args.overlap:
        eng.tune(eng.TUNE_OVERLAP, 1)
    eng.set_atoms(x, v, t, rho, e, cv)
    if world > 1:
        eng.set_tags(tags)
    with stdout_to_stderr():  # communicator init, first exchanges and warmup
        if world > 1:
            attach_comm(eng, sph, args, dist, rank, world)
        elif args.comm_loopback:
            eng.comm_init(sph.comm_uid(), 1, 0)
            eng.comm_loopback(True)
        eng.setup()
        eng.run(args.warmup)
    eng.sync()

    barrier()
    eng.sync()
    # HIP events in the timed region only around the two pair passes (the roofline kernels):
    # an event pair per scope is ~4 % of a 1M step and ~20 % of a 125k one
    eng.set_timing(True, classes=(eng.T_RHO, eng.T_TAIT))
    t0 = time.perf_counter()
    eng.run(args.steps)
    eng.sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = max_over_ranks(t1 - t0)
    st = eng.stats()
    # the other classes (rebuild, integrate, comm) over 10 more steps, outside the timed region
    eng.set_timing(True)
    eng.run(10)
    eng.sync()
    st_x = eng.stats()

    nloc = st["nlocal"]
    total_ps = n_total * args.steps / elapsed
    n_full = st["nbr_full"] / max(nloc, 1)
    n_half = n_full / 2.0
    # algorithmic bytes per particle per pass (half-list CSR, int32, fp64)
    bytes_tait = 104.0 + 4.0 * n_half
    bytes_rho = 40.0 + 4.0 * n_half
    ms_tait = st["ms_tait"] / max(st["n_tait"], 1)
    ms_rho = st["ms_rhosum"] / max(st["n_rhosum"], 1)
    ach_tait = bytes_tait * nloc / (ms_tait * 1e-3) / 1e9
    ach_rho = bytes_rho * nloc / (ms_rho * 1e-3) / 1e9
    ach_pair = (bytes_tait + bytes_rho) * nloc / ((ms_tait + ms_rho) * 1e-3) / 1e9
    kname = "k_blk_force" if st["staged"] == 1 else "k_row2_force"
    out = dict(base, value=total_ps, ms_per_step=elapsed / args.steps * 1e3)
    out["config"] = {"workload": workload,
                     "particles_per_gpu": nloc, "ghosts_per_gpu": st["nghost"],
                     "n_full_per_particle": n_full, "n_half_per_particle": n_half,
                     "parallelism": parallelism,
                     "kernel_path": ("block-staged LDS unions + 16-bit slot rows"
                                     if st["staged"] == 1 else "row path (global gathers)")}
    out["roofline"] = {"bound": "hbm", "kernel": kname + "<TAIT> (sph/taitwater pass)",
                       "achieved": ach_tait, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                       "frac": ach_tait / PEAK_HBM_GBS, "traffic": None,
                       "bytes_per_particle": bytes_tait, "ms_per_launch": ms_tait}
    out["kernels"] = {"rhosum": {"ms_per_launch": ms_rho, "achieved_GBs": ach_rho,
                                 "bytes_per_particle": bytes_rho},
                      "rhosum+taitwater": {"achieved_GBs": ach_pair,
                                           "frac": ach_pair / PEAK_HBM_GBS,
                                           "kernel_particle_steps_per_s":
                                               nloc / ((ms_tait + ms_rho) * 1e-3)},
                      "neighbor_build_ms": st_x["ms_neigh"] / max(st_x["n_neigh"], 1),
                      "integrate_ms_per_step": st_x["ms_integrate"] / 10,
                      "comm_ms_per_step": st_x["ms_comm"] / 10,
                      "timing_note": "rhosum/taitwater: HIP events in the timed region; "
                                     "neighbor build, integrate, comm: 10 further steps "
                                     "with every class timed"}
    attach_pmc_traffic(out, kname, bytes_tait * nloc, world, args)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args.cpu_n)
        # beside it, the same reference code on all the cores this process may use (one
        # brick per process)
        out["cpu_baseline_cores"] = cpu_baseline_cores(args.cpu_n, nproc=host_cores())
    if rank == 0:
        print(json.dumps(out), flush=True)
    with stdout_to_stderr():  # communicator teardown
        eng.close()
    if dist is not None:
        dist.destroy_process_group()


def attach_pmc_traffic(out, kname, alg_bytes, world, args, fname="pmc_traffic.json"):
    """HBM traffic per step of the roofline kernel from PMC counters, measured on THIS
    workload by tools/pmc_traffic.sh and committed as profiles/<round>/pmc_traffic.json with
    the kernel, config and commit it was taken on.  Attached as `traffic` only when that
    record matches this run (same kernel family, single GPU, same lattice edge and steps);
    otherwise it is omitted (traffic null) rather than reported from another configuration."""
    for rnd in ("r06", "r05", "r04", "r03", "r02"):
        tj = os.path.join(ROOT, "profiles", rnd, fname)
        if not os.path.exists(tj):
            continue
        rec = json.load(open(tj))
        meta = rec.get("_meta", {})
        if (meta.get("world") != world or meta.get("edge") != args.edge
                or meta.get("path") != args.path):
            continue
        v = rec.get(kname, {})
        if v.get("traffic_bytes"):
            out["roofline"]["traffic"] = v["traffic_bytes"] / 1e9
            out["roofline"]["traffic_unit"] = (
                f"GB per step of {kname} (its launches summed; PMC 2*FETCH_SIZE + WRITE_SIZE, "
                f"tools/pmc_traffic.sh, profiles/{rnd}/{fname}, commit "
                f"{meta.get('commit', '?')})")
            out["roofline"]["algorithmic_GB_per_step"] = alg_bytes / 1e9
            va = v.get("valu")
            if va:  # what binds the pass: its fp64 VALU issue (PMC SQ_INSTS_VALU / duration)
                out["roofline"]["valu_issue_frac"] = va["issue_frac_fp64"]
                out["roofline"]["valu_issue_unit"] = (
                    "VALU wave-instructions of the main launch / its duration / the fp64 issue "
                    "peak (256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles), same PMC record")
            return


if __name__ == "__main__":
    main()
