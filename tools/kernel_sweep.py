"""Time the pair kernels (rhosum, taitwater) on the C2 1M workload for one engine config.
Run once per SPH_GROUP value (the group width is read once per process)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    sph = bench.load_pkg()
    x, v, t, rho, e, cv = bench.make_system(n, 12345)
    cfg = bench.c2_config(sph, n)
    cfg.kernel_path = int(os.environ.get("SPH_PATH", "0"))
    exp = os.environ.pop("SPH_EXP", None)   # study variants: the timed passes only
    eng = sph.Engine(cfg)
    eng.set_atoms(x, v, t, rho, e, cv)
    eng.setup()
    eng.run(12)                 # past the first rebuild: the steady-state (strided) list
    if exp is not None:
        os.environ["SPH_EXP"] = exp
    eng.pair_passes(3)
    eng.sync()
    eng.set_timing(True)
    eng.pair_passes(reps)
    st = eng.stats()
    print(json.dumps({"group": os.environ.get("SPH_GROUP", "8"), "path": cfg.kernel_path,
                      "staged": st["staged"], "stage_max": st["stage_max"],
                      "rows_max": st["nbr_maxrow"],
                      "rhosum_ms": st["ms_rhosum"] / st["n_rhosum"],
                      "tait_ms": st["ms_tait"] / st["n_tait"],
                      "comm_ms": st["ms_comm"] / max(st["n_rhosum"], 1)}))


if __name__ == "__main__":
    main()
