"""Per step of C2 (bench.py's 1M lattice): the force pass's time and whether its rows were
the inner ones (sph_engine_stats inner_live / inner_refresh) -- why the pass slows down
inside a rebuild interval.  --jitter A: a further uniform +-A displacement (spacing 1; bench.py's
lattice already carries +-0.1); --resetup: a second setup() after the 25 steps and 25 more (disordered start);
--pairs: also the pairs per atom inside the cutoff (scipy, periodic box) and the largest speed;
--clocks: the gfx clock and socket power amd-smi reports after each step;
--sampler: the shader clock DURING each step, from tools/libclock_sampler.so (a one-wave
kernel on its own stream sampling the clock counter against the 100 MHz real-time counter
beside the engine's kernels: no serialisation), as the mean clock over the step's first
0.5 ms and per 100 us window."""
import argparse
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

ap = argparse.ArgumentParser()
ap.add_argument("--jitter", type=float, default=0.0)
ap.add_argument("--resetup", action="store_true")
ap.add_argument("--pairs", action="store_true")
ap.add_argument("--clocks", action="store_true")
ap.add_argument("--sampler", action="store_true")
args = ap.parse_args()
import numpy as np  # noqa: E402

sph = load_sph_amd()
x, v, t, rho, e, cv, tags = bench.strong_lattice(100, (1, 1, 1), 0)
if args.jitter > 0:
    x = x + args.jitter * np.random.default_rng(1).uniform(-1, 1, x.shape)  # (spacing 1)
    print(f"jitter {args.jitter}", flush=True)
eng = sph.Engine(bench.c2_config(sph, 100))


_smi = []


def clock_line():
    try:
        import amdsmi
        if not _smi:
            amdsmi.amdsmi_init()
            _smi.append(amdsmi.amdsmi_get_processor_handles()[0])
        m = amdsmi.amdsmi_get_gpu_metrics_info(_smi[0])
        keys = ("average_gfxclk_frequency", "current_gfxclk", "current_socket_power",
                "average_socket_power", "temperature_hotspot", "throttle_status")
        return " " + " ".join(f"{k} {m[k]}" for k in keys if k in m)
    except Exception as ex:  # (reported, not fatal: a probe)
        return f" smi {type(ex).__name__}: {ex}"


def pairs_line():
    from scipy.spatial import cKDTree
    a = eng.get_atoms()
    xa = np.mod(a["x"], 100.0)
    q = xa[::20]  # (every 20th atom's pairs)
    c = cKDTree(q, boxsize=100.0).count_neighbors(cKDTree(xa, boxsize=100.0), 3.0)
    n = q.shape[0]
    return f" pairs/atom {(c - n) / n:.3f} vmax {np.abs(a['v']).max():.4f}"


_clk = []


def sampler_start():
    import ctypes
    if not _clk:
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libclock_sampler.so"))
        lib.clk_start.argtypes = [ctypes.c_int, ctypes.c_double]
        lib.clk_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _clk.append(lib)
    assert _clk[0].clk_start(100, 1000.0) == 0


def sampler_line():
    buf = np.zeros(200, dtype=np.uint64)
    assert _clk[0].clk_read(buf.ctypes.data, 100) == 0
    t = buf[0::2].astype(np.float64) * 10.0  # ns
    c = buf[1::2].astype(np.float64)
    ghz = np.diff(np.concatenate([[0.0], c])) / np.diff(np.concatenate([[0.0], t]))
    w = [float(ghz[k * 10:(k + 1) * 10].mean()) for k in range(10)]
    m = t <= 500e3
    return (f" clk0.5ms {c[m][-1] / t[m][-1]:.3f} GHz windows " +
            " ".join(f"{g:.2f}" for g in w))


eng.set_atoms(x, v, t, rho, e, cv)
eng.setup()
eng.set_timing(True, classes=(eng.T_RHO, eng.T_TAIT))
prev = eng.stats()
for k in range(50 if args.resetup else 25):
    if k == 25:
        eng.setup()
        print("setup again", flush=True)
        prev = eng.stats()
    if args.sampler:
        sampler_start()
    eng.run(1)
    eng.sync()
    st = eng.stats()
    ms = (st["ms_tait"] - prev["ms_tait"]) / max(st["n_tait"] - prev["n_tait"], 1)
    mr = (st["ms_rhosum"] - prev["ms_rhosum"]) / max(st["n_rhosum"] - prev["n_rhosum"], 1)
    print(f"step {st['step']:3d} force {ms * 1e3:7.1f} us rhosum {mr * 1e3:6.1f} us "
          f"inner_rows {st['inner_rows']} "
          f"live {st['inner_live']} refreshes {st['inner_refresh']} builds {st['nbr_builds']}"
          + (pairs_line() if args.pairs else "") + (clock_line() if args.clocks else "") + (sampler_line() if args.sampler else ""),
          flush=True)
    prev = st
eng.close()
