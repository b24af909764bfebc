"""Per-step field errors of the C5 brick engine vs the per-rank oracle (GPU diagnostic)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pyoracle as po  # noqa: E402
from c5_util import bricks_step, mp_bricks, mp_collect  # noqa: E402
from scenarios import bubble_physics, bubble_system  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

sph = ge._import_pkg()
nx, pg = int(sys.argv[1]), tuple(int(v) for v in sys.argv[2].split(","))
s = bubble_system(nx)
ph = bubble_physics(nx, prob=0.5, Tt=-1.0)
if len(sys.argv) > 3:   # styles kept: t(ait) s(urface tension) h(eat)
    ph.tait, ph.st, ph.heat = ("t" in sys.argv[3]), ("s" in sys.argv[3]), ("h" in sys.argv[3])
ref = po.MpRefRun(s, ph, procgrid=pg)
ref.setup()
world, engines = mp_bricks(sph, s, ph, pg, po.brick_owner(s, s.x, pg))
bricks_step(engines, lambda e: e.setup())
for step in range(5):
    if step:
        ref.run(1)
        bricks_step(engines, lambda e: e.run(1))
    out = mp_collect(engines, ref.s.n)
    r = ref.s
    msg = [f"step {step} n {r.n} ins {out['ninserted']}/{ref.ninserted}"]
    for k, want in (("x", r.x), ("v", r.v), ("rho", r.rho), ("e", r.e), ("rmass", r.rmass),
                    ("cg", ref.cg), ("f", ref.f), ("de", ref.de)):
        d = np.abs(out[k] - want)
        d = d.max(axis=1) if d.ndim > 1 else d
        i = int(np.argmax(d))
        msg.append(f"{k} {d[i] / np.abs(want).max():.2e}@{i}(t{r.type[i]})")
    print(" ".join(msg), flush=True)
for e in engines:
    e.close()
world.close()
