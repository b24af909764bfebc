"""Diagnostic: C5 bricks with a drifting system (atoms migrate) -- per-step field errors,
engine vs oracle, with and without fix phase_change."""
import dataclasses
import sys

import numpy as np

sys.path[:0] = ["tests", "oracle"]
import pyoracle as po  # noqa: E402
from c5_util import bricks_step, mp_bricks, mp_collect  # noqa: E402
from scenarios import bubble_physics, bubble_system, drifting, shuffled  # noqa: E402
from conftest import load_sph_amd  # noqa: E402

sph = load_sph_amd()


def run(pc, vx, pg=(2, 1, 1), nx=10, steps=6, sortfreq=4):
    s = drifting(shuffled(bubble_system(nx), 3), vx, 0.49 / nx)
    ph = dataclasses.replace(bubble_physics(nx, prob=0.5, Tt=-1.0, pc=pc), sortfreq=sortfreq)
    ref = po.MpRefRun(s, ph, procgrid=pg)
    ref.setup()
    own0 = po.brick_owner(s, s.x, pg)
    world, engines = mp_bricks(sph, s, ph, pg, own0)
    bricks_step(engines, lambda e: e.setup())
    for step in range(steps + 1):
        if step:
            ref.run(1)
            bricks_step(engines, lambda e: e.run(1))
        out = mp_collect(engines, ref.s.n)
        fl = {"x": ref.s.x, "v": ref.s.v, "rho": ref.s.rho, "e": ref.s.e, "rmass": ref.s.rmass,
              "cg": ref.cg, "f": ref.f, "de": ref.de}
        errs = {}
        worst = {}
        for k, b in fl.items():
            a = out[k]
            d = np.abs(a - b).reshape(len(b), -1).max(axis=1)
            errs[k] = d.max() / max(np.abs(b).max(), 1e-300)
            worst[k] = int(d.argmax())
        moved = int((po.brick_owner(s, ref.s.x[:s.n], pg) != own0).sum())
        print(f"pc={pc} vx={vx} step {step} nins {ref.ninserted}/{out['ninserted']} moved {moved} "
              + " ".join(f"{k}:{v:.1e}@{worst[k]}" for k, v in errs.items()), flush=True)
    for e in engines:
        e.close()
    world.close()


for pc, vx in ((False, 200.0), (True, 0.0), (True, 200.0)):
    run(pc, vx)
