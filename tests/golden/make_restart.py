"""Golden per-atom restart records from the REFERENCE's own AtomVecMeso::pack_restart
(atom_vec_meso.cpp:729-757) and AtomVecMesoMultiPhase::pack_restart
(atom_vec_meso_multiphase.cpp:887-916), compiled into oracle/_ref and called per atom by
ref_pack_restart (oracle/ref_harness.cpp).  Inputs are random fields with packed image
flags of both signs.  Run here:  python tests/golden/make_restart.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
import pyoracle as po  # noqa: E402


def main():
    R = po.ref()
    rng = np.random.default_rng(31)
    n = 9
    d = dict(x=rng.normal(size=(n, 3)) * 5, tag=np.arange(3, 3 + n, dtype=np.int32),
             type=rng.integers(1, 3, n).astype(np.int32),
             mask=np.array([1, 3, 1, 5, 1, 1, 3, 1, 1], np.int32),
             image=po.img_pack(rng.integers(-3, 4, size=(n, 3))).astype(np.int32),
             v=rng.normal(size=(n, 3)), rho=rng.uniform(0.5, 2, n), cg=rng.normal(size=(n, 3)),
             rmass=rng.uniform(0.5, 2, n), e=rng.uniform(0, 3, n), cv=rng.uniform(0.5, 2, n),
             vest=rng.normal(size=(n, 3)))
    out = dict(d)
    for mp, width, key in ((0, 17, "rec_meso"), (1, 21, "rec_multiphase")):
        rec = np.zeros((n, 32))
        ln = R.ref_pack_restart(mp, n, d["x"], d["tag"], d["type"], d["mask"], d["image"], d["v"],
                                d["rho"], d["cg"], d["rmass"], d["e"], d["cv"], d["vest"], 32,
                                rec)
        assert ln == width, (ln, width)
        out[key] = rec[:, :width].copy()
    np.savez_compressed(os.path.join(HERE, "restart_records.npz"), **out)
    print("restart_records.npz:", {k: v.shape for k, v in out.items() if k.startswith("rec")})


if __name__ == "__main__":
    main()
