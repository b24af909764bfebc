"""Per step of C2 (bench.py's 1M lattice): the force pass's time and whether its rows were
the inner ones (sph_engine_stats inner_live / inner_refresh) -- why the pass slows down
inside a rebuild interval."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
from conftest import load_sph_amd  # noqa: E402

sph = load_sph_amd()
x, v, t, rho, e, cv, tags = bench.strong_lattice(100, (1, 1, 1), 0)
eng = sph.Engine(bench.c2_config(sph, 100))
eng.set_atoms(x, v, t, rho, e, cv)
eng.setup()
eng.set_timing(True, classes=(eng.T_RHO, eng.T_TAIT))
prev = eng.stats()
for k in range(25):
    eng.run(1)
    eng.sync()
    st = eng.stats()
    ms = (st["ms_tait"] - prev["ms_tait"]) / max(st["n_tait"] - prev["n_tait"], 1)
    mr = (st["ms_rhosum"] - prev["ms_rhosum"]) / max(st["n_rhosum"] - prev["n_rhosum"], 1)
    print(f"step {st['step']:3d} force {ms * 1e3:7.1f} us rhosum {mr * 1e3:6.1f} us "
          f"inner_rows {st['inner_rows']} "
          f"live {st['inner_live']} refreshes {st['inner_refresh']} builds {st['nbr_builds']}",
          flush=True)
    prev = st
eng.close()
