"""Time the neighbour rebuild (sph_engine_rebuild_passes) on the C2 1M workload for one
engine config; SPH_BEXP (build study variants) applies to the timed rebuilds only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    sph = bench.load_pkg()
    x, v, t, rho, e, cv = bench.make_system(n, 12345)
    cfg = bench.c2_config(sph, n)
    cfg.kernel_path = int(os.environ.get("SPH_PATH", "0"))
    bexp = os.environ.pop("SPH_BEXP", None)
    eng = sph.Engine(cfg)
    eng.set_atoms(x, v, t, rho, e, cv)
    eng.setup()
    eng.run(2)
    if bexp is not None:
        os.environ["SPH_BEXP"] = bexp
    eng.rebuild_passes(1)
    eng.sync()
    eng.set_timing(True)
    eng.rebuild_passes(reps)
    st = eng.stats()
    print(json.dumps({"path": cfg.kernel_path, "bexp": bexp, "staged": st["staged"],
                      "rebuild_ms": st["ms_neigh"] / max(st["n_neigh"], 1)}))


if __name__ == "__main__":
    main()
