"""debug: C5 engine vs oracle step by step"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pyoracle as po
from scenarios import bubble_system, bubble_physics
from c5_util import mp_engine, mp_state
import bench
sph = bench.load_pkg()
nx = int(sys.argv[1]) if len(sys.argv) > 1 else 10
s = bubble_system(nx); ph = bubble_physics(nx, prob=0.5, Tt=-1.0)
ref = po.MpRefRun(s, ph); ref.setup()
eng = mp_engine(sph, s, ph); eng.setup()
def rel(a, b):
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)
def rep(k):
    g = mp_state(eng)
    if g["x"].shape[0] != ref.s.n:
        print(k, "nlocal", g["x"].shape[0], ref.s.n, "ins", g["ninserted"], ref.ninserted); return
    c = eng.neighbor_counts(); rc = ref.numneigh_full()
    print(k, "n", ref.s.n, "ins", g["ninserted"], "x %.1e v %.1e rho %.1e e %.1e f %.1e de %.1e rm %.1e cg %.1e cnt %d type %d" % (
        rel(g["x"], ref.s.x), rel(g["v"], ref.s.v), rel(g["rho"], ref.s.rho), rel(g["e"], ref.s.e),
        rel(g["f"], ref.f), rel(g["de"], ref.de), rel(g["rmass"], ref.s.rmass), rel(g["cg"], ref.cg),
        int((c != rc).sum()), int((g["type"] != ref.s.type).sum())), flush=True)
rep(0)
for k in range(1, 7):
    ref.run(1); eng.run(1); rep(k)
