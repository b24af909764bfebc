"""Debug helper: brick-decomposed engine vs oracle after n steps; prints error location."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import conftest  # noqa: E402
import pyoracle as po  # noqa: E402
from scenarios import c2_system  # noqa: E402
from test_gpu_bricks import run_bricks  # noqa: E402

sph = conftest.load_sph_amd()
pg = tuple(int(v) for v in sys.argv[1].split(","))
for nsteps in [int(v) for v in sys.argv[2].split(",")]:
    s = c2_system(12)
    ph = po.c2_physics()
    ph.every = 4
    ref = po.RefRun(s, ph)
    ref.setup()
    ref.run(nsteps)
    out, counts, nloc = run_bricks(sph, s, ph, pg, nsteps)
    for k, want in (("rho", ref.s.rho), ("f", ref.f), ("x", ref.s.x), ("v", ref.s.v),
                    ("drho", ref.drho), ("de", ref.de)):
        err = np.abs(out[k] - want)
        if err.ndim > 1:
            err = err.max(1)
        i = int(err.argmax())
        print(f"pg={pg} steps={nsteps} {k}: max rel {err.max() / np.abs(want).max():.3e} at atom {i}"
              f" x={ref.s.x[i]} nbad={(err > 1e-10 * np.abs(want).max()).sum()}", flush=True)
