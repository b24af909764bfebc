"""C5 bubble on 2x2x2 LocalWorld bricks against pyoracle.MpRefRun(procgrid=(2, 2, 2)), step
by step: neighbour-count mismatches (tag, position, engine / oracle counts, brick of the atom,
distance to the nearest brick face) and insertion counts.  A diagnostic for
tests/test_gpu_configs.py::test_c5_bricks_vs_oracle_32.  usage: python tools/c5_bricks_diag.py [nx=32] [steps=4] [pg=2,2,2] [nopc]"""
import dataclasses
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import pyoracle as po  # noqa: E402
from c5_util import bricks_step, mp_bricks, mp_collect  # noqa: E402
from conftest import load_sph_amd  # noqa: E402
from scenarios import bubble_physics, bubble_system  # noqa: E402

nx = int(sys.argv[1]) if len(sys.argv) > 1 else 32
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
PG = tuple(int(v) for v in sys.argv[3].split(",")) if len(sys.argv) > 3 else (2, 2, 2)
sph = load_sph_amd()
s = bubble_system(nx)
ph = bubble_physics(nx, prob=0.5, Tt=-1.0)
if len(sys.argv) > 4 and sys.argv[4] == "nopc":
    ph = dataclasses.replace(ph, pc=None)
ref = po.MpRefRun(s, ph, procgrid=PG)
ref.setup()
owner = po.brick_owner(s, s.x, PG)
world, engines = mp_bricks(sph, s, ph, PG, owner)
bricks_step(engines, lambda e: e.setup())
for step in range(steps + 1):
    if step:
        ref.run(1)
        bricks_step(engines, lambda e: e.run(1))
    out = mp_collect(engines, ref.s.n)
    rc = ref.numneigh_full()
    bad = np.nonzero(out["counts"] != rc)[0]
    print(f"== step {step}: n {ref.s.n} inserted engine {out['ninserted']} oracle {ref.ninserted}; "
          f"count mismatches {bad.size}", flush=True)
    for t in bad[:12]:
        x = ref.s.x[t]
        m = np.mod(x, 0.5)
        face = float(np.minimum(m, 0.5 - m).min())
        print(f"  tag {t} type {ref.s.type[t]} x {np.round(x, 6).tolist()} engine {out['counts'][t]} "
              f"oracle {rc[t]} brick {int(po.brick_owner(ref.s, x[None, :], PG)[0])} "
              f"min dist to a brick plane {face:.4g} created {t >= s.n}", flush=True)
    if bad.size:
        d = np.abs(out["x"] - ref.s.x).max()
        print(f"  max |x diff| {d:.3e}", flush=True)
