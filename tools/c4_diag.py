"""C4 (200^3 = 8M, C2 physics) as one brick against 2x2x2 LocalWorld bricks, step by step:
per field the largest difference and where the worst atoms sit (distance to the nearest brick
face / box face).  A diagnostic for tests/test_gpu_configs.py::test_c4_8m_bricks_match_one_brick.
usage: python tools/c4_diag.py [n=100] [steps=11] [rest]  (rest: velocities zeroed)"""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
from c5_util import bricks_step  # noqa: E402
from conftest import load_sph_amd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 11
PG = (2, 2, 2)
sph = load_sph_amd()
parts = [bench.brick_lattice(n, PG, r) for r in range(8)]
if len(sys.argv) > 3 and sys.argv[3] == "rest":
    for p in parts:
        p[1][:] = 0.0
N = sum(p[0].shape[0] for p in parts)
tags = np.concatenate([p[6] for p in parts])
order = np.argsort(tags)
glob = [np.concatenate([p[k] for p in parts])[order] for k in range(6)]
e1 = sph.Engine(bench.c2_config(sph, 2 * n))
e1.set_atoms(*glob)
world = sph.LocalWorld(8)
engines = []
for r, p in enumerate(parts):
    eng = sph.Engine(bench.c2_config(sph, n, PG, r))
    eng.set_atoms(*p[:6])
    eng.set_tags(p[6])
    eng.comm_local(world, r)
    engines.append(eng)


def collect():
    out = {}
    for eng in engines:
        g = eng.get_atoms()
        t = g["tag"]
        for k, v in g.items():
            if k == "tag" or not isinstance(v, np.ndarray) or v.shape[:1] != t.shape:
                continue
            out.setdefault(k, np.zeros((N,) + v.shape[1:], v.dtype))[t] = v
        out.setdefault("counts", np.zeros(N, np.int32))[t] = eng.neighbor_counts()
    return out


def report(step):
    one = e1.get_atoms()
    one["counts"] = e1.neighbor_counts()
    b = collect()
    print(f"== step {step}: counts equal {np.array_equal(b['counts'], one['counts'])}", flush=True)
    for k in ("x", "v", "rho", "f", "drho", "de", "e"):
        a, w = b[k].reshape(N, -1), one[k].reshape(N, -1)
        d = np.abs(a - w).max(axis=1)
        i = np.argsort(d)[::-1][:4]
        xs = one["x"][i]
        face = np.minimum(np.abs(xs - n), np.minimum(np.abs(xs), np.abs(xs - 2 * n))).min(axis=1)
        print(f"  {k:5s} max|diff| {d.max():.3e} (rel {d.max() / np.abs(w).max():.2e}); worst tags "
              f"{i.tolist()} x {np.round(xs, 3).tolist()} dist to a face {np.round(face, 3).tolist()} "
              f"n(diff>1e-12*max) {(d > 1e-12 * np.abs(w).max()).sum()}", flush=True)


e1.setup()
bricks_step(engines, lambda e: e.setup())
report(0)
for s in range(1, steps + 1):
    e1.run(1)
    bricks_step(engines, lambda e: e.run(1))
    if s in (1, 2, 3, 5, 9, 10, 11) or s == steps:
        report(s)
print("one-brick stats", e1.stats())
print("brick 0 stats", engines[0].stats())
