"""Wall time of each engine step of the C2 bench workload (setup, then one step at a time
with a device sync), with the inner-row state after each: which steps of a short run are
slow, and why.  usage: python tools/step_times.py [edge] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    sph = bench.load_pkg()
    x, v, t, rho, e, cv = bench.make_system(n, 12345)
    eng = sph.Engine(bench.c2_config(sph, n))
    eng.set_atoms(x, v, t, rho, e, cv)
    t0 = time.perf_counter()
    eng.setup()
    eng.sync()
    print(f"setup {1e3 * (time.perf_counter() - t0):8.3f} ms", flush=True)
    for k in range(steps):
        t0 = time.perf_counter()
        eng.run(1)
        eng.sync()
        st = eng.stats()
        print(f"step {st['step']:3d} {1e3 * (time.perf_counter() - t0):8.3f} ms  inner_live "
              f"{st['inner_live']} refreshes {st['inner_refresh']}", flush=True)


if __name__ == "__main__":
    main()
