"""The N > 1 host path of bench.py on CPU (torch.distributed gloo, world size 2): brick grid,
each rank's share of the global lattice, the RCCL unique-id broadcast from rank 0, and the
max-over-ranks timing reduction.  The device side of the decomposition is covered by
tests/test_gpu_bricks.py (several bricks in one process on the GPU)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, q):
    import torch

    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pg = bench.procgrid_for(world)
        n = 4
        x, v, t, rho, e, cv, tags = bench.brick_lattice(n, pg, rank)
        uid = bench.share_uid(dist, rank, lambda: bytes(range(128)))
        gathered = [None] * world
        dist.all_gather_object(gathered, (tags.tolist(), x.tolist()))
        tt = torch.tensor([0.1 * (rank + 1)], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        q.put((rank, pg, uid, gathered, float(tt.item())))
    finally:
        dist.destroy_process_group()


def test_two_rank_bricks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    for rank, pg, uid, gathered, tmax in res:
        assert pg == (2, 1, 1)
        assert uid == bytes(range(128))              # rank 0's id reached every rank
        assert tmax == pytest.approx(0.2)            # max over ranks
    gathered = res[0][3]
    tags = np.concatenate([np.array(g[0]) for g in gathered])
    xs = np.concatenate([np.array(g[1]) for g in gathered])
    n, NX = 4, 8
    assert np.array_equal(np.sort(tags), np.arange(n * n * NX))  # a partition of the box
    # every site lies in its rank's brick (up to the +-0.1 jitter the first exchange fixes)
    for r, g in enumerate(gathered):
        xr = np.array(g[1])
        assert (xr[:, 0] >= r * n - 0.1).all() and (xr[:, 0] < (r + 1) * n + 0.1).all()
    # the sites are exactly those of the global lattice, tag = (z*NY + y)*NX + x
    site = np.rint(xs).astype(int)
    assert np.array_equal((site[:, 2] * n + site[:, 1]) * NX + site[:, 0], tags)


def _bench_json(args):
    import json
    import subprocess
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # ONE JSON line, from rank 0 only
    return json.loads(lines[0])


def test_bench_launches_ranks_strong():
    """`bench.py --gpus 2` without WORLD_SIZE starts its own two ranks (fresh processes);
    the rank-0 line says n_gpus 2 and the strong split partitions the one 1M box."""
    out = _bench_json(["--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0"])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert "strong" in out["config"]["workload"] and "2x1x1" in out["config"]["workload"]
    assert out["config"]["particles_total"] == 100 ** 3
    assert len(out["config"]["particles_per_rank"]) == 2


def test_bench_launches_ranks_weak():
    out = _bench_json(["--gpus", "4", "--dry-run", "--scaling", "weak", "--edge", "10"])
    assert out["n_gpus"] == 4 and out["scaling"] == "weak"
    assert "weak" in out["config"]["workload"]
    assert out["config"]["particles_per_rank"] == [1000] * 4


def test_strong_lattice_partition():
    """The strong split's bricks partition make_system(n) exactly (same sites, jitter,
    velocities), so N = 1 and N > 1 run the same physical system."""
    import bench
    n = 12
    x0, v0, *_ = bench.make_system(n, 12345)
    pg = bench.procgrid_for(8)
    parts = [bench.strong_lattice(n, pg, r) for r in range(8)]
    tags = np.concatenate([p[6] for p in parts])
    assert np.array_equal(np.sort(tags), np.arange(n ** 3))
    order = np.argsort(tags)
    xs = np.concatenate([p[0] for p in parts])[order]
    vs = np.concatenate([p[1] for p in parts])[order]
    assert np.array_equal(xs, x0) and np.array_equal(vs, v0)


def test_bench_rejects_world_mismatch():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def _visible_devices():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "sph_amd_probe", os.path.join(ROOT, "lammps-sph-multiphase_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.device_count()


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["c2", "c5"])
def test_bench_two_gpus(workload):
    """`bench.py --gpus 2` over RCCL when the box shows two devices (the driver's multi-GPU
    node); skipped on a one-GPU box, where two RCCL ranks cannot share the card."""
    import subprocess
    probe = subprocess.run([sys.executable, "-c",
                            "import test_multi_rank as t; print(t._visible_devices())"],
                           cwd=os.path.dirname(__file__), capture_output=True, text=True,
                           timeout=240)
    ndev = int(probe.stdout.strip().splitlines()[-1]) if probe.returncode == 0 else 0
    if ndev < 2:
        pytest.skip(f"{ndev} HIP device(s) visible")
    args = ["--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu", "--workload", workload]
    if workload == "c5":
        args += ["--edge", "60"]
    out = _bench_json(args)
    assert out["n_gpus"] == 2 and out["value"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("workload,edge", [("c2", "24"), ("c5", "30")])
def test_bench_two_processes_ipc(workload, edge):
    """`bench.py --gpus 2 --transport ipc` on the one GPU of the test box: bench's own rank
    launch (fresh processes before any HIP call), the world name broadcast from rank 0,
    hipIpc halos between the two processes, barrier + max-over-ranks timing, ONE JSON line
    from rank 0 -- the multi-GPU bench path with only the byte mover swapped."""
    out = _bench_json(["--gpus", "2", "--transport", "ipc", "--steps", "3", "--warmup", "1",
                       "--no-cpu", "--workload", workload, "--edge", edge])
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert "hipIpc" in out["config"]["parallelism"]
