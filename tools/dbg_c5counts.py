"""Debug helper: C5 neighbour counts at setup, engine vs oracle."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "oracle")); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np
import pyoracle as po
from conftest import load_sph_amd
from scenarios import bubble_system, bubble_physics
from c5_util import mp_engine, mp_state
sph = load_sph_amd()
for nx, dim, pc in ((10, 3, True), (10, 3, False), (16, 2, True)):
    s = bubble_system(nx, dim=dim); ph = bubble_physics(nx, dim=dim, prob=0.5, Tt=-1.0, pc=pc)
    r = po.MpRefRun(s, ph); r.setup()
    eng = mp_engine(sph, s, ph); eng.setup()
    ce, co = eng.neighbor_counts(), r.numneigh_full()
    g = mp_state(eng)
    d = np.nonzero(ce != co)[0]
    print(nx, dim, pc, "rows differing", d.size, "of", ce.size, "sum eng", ce.sum(), "oracle", co.sum())
    if d.size:
        # engine atom order may differ from the oracle's; compare by position
        print("  first rows", d[:8], ce[d[:8]], co[d[:8]])
        print("  eng x", g["x"][d[:3]], "oracle x", r.s.x[d[:3]])
        print("  same order?", np.abs(g["x"] - r.s.x).max())
