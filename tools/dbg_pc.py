"""Debug helper: C5 slab geometry, engine vs oracle insertions per step (exact and port)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "oracle")); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np
import pyoracle as po
from conftest import load_sph_amd
from scenarios import bubble_system, bubble_physics
from c5_util import mp_engine, mp_state
sph = load_sph_amd()
nx, dim = int(sys.argv[1]), int(sys.argv[2])
s = bubble_system(nx, dim=dim, slab=True); ph = bubble_physics(nx, dim=dim, prob=0.3, Tt=-1.0)
refs = []
for exact in (True, False):
    r = po.MpRefRun(s, ph); r.pc_exact = exact; r.setup(); refs.append(r)
eng = mp_engine(sph, s, ph); eng.setup()
for step in range(5):
    for r in refs: r.run(1)
    eng.run(1)
    g = mp_state(eng)
    print(step + 1, "eng", g["ninserted"], "exact", refs[0].ninserted, "port", refs[1].ninserted,
          "rmass err exact %.2e port %.2e" % (
              np.abs(g["rmass"][:refs[0].s.n] - refs[0].s.rmass).max() if g["x"].shape[0] == refs[0].s.n else -1,
              np.abs(g["rmass"][:refs[1].s.n] - refs[1].s.rmass).max() if g["x"].shape[0] == refs[1].s.n else -1))
