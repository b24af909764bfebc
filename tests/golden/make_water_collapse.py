"""Convert the reference's C1 input (examples/USER/sph/water_collapse/data.initial, a LAMMPS
data file for atom_style meso) into the fixture tests/golden/water_collapse.npz.

The fixture is DATA: the file's own numbers (box, masses, per-atom id/type/rho/e/cv/x/image
and velocities), stored as plain arrays (np.savez_compressed, no pickles), so the tests and
the GPU box never need /root/reference.  atom_style meso data line (atom_vec_meso.cpp:
data_atom): atom-ID atom-type rho e cv x y z [ix iy iz].

Run here (where /root/reference exists):  python tests/golden/make_water_collapse.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/examples/USER/sph/water_collapse/data.initial"


def parse(path):
    lines = open(path).read().splitlines()
    natoms = ntypes = 0
    box = np.zeros((3, 2))
    k = 0
    while k < len(lines):
        t = lines[k].split("#")[0].strip()
        if t.endswith("atoms"):
            natoms = int(t.split()[0])
        elif t.endswith("atom types"):
            ntypes = int(t.split()[0])
        for d, ax in enumerate("xyz"):
            if t.endswith(f"{ax}lo {ax}hi"):
                box[d] = [float(v) for v in t.split()[:2]]
        if t in ("Masses", "Atoms", "Velocities") or t.startswith("Atoms"):
            break
        k += 1
    sections = {}
    while k < len(lines):
        head = lines[k].split("#")[0].strip()
        if not head:
            k += 1
            continue
        name = head.split()[0]
        n = ntypes if name == "Masses" else natoms
        k += 1
        while not lines[k].strip():
            k += 1
        sections[name] = [lines[k + i].split() for i in range(n)]
        k += n
    return natoms, ntypes, box, sections


def main():
    natoms, ntypes, box, sec = parse(SRC)
    mass = np.zeros(ntypes + 1)
    for row in sec["Masses"]:
        mass[int(row[0])] = float(row[1])
    a = sec["Atoms"]
    ids = np.array([int(r[0]) for r in a], dtype=np.int32)
    typ = np.array([int(r[1]) for r in a], dtype=np.int32)
    vals = np.array([[float(v) for v in r[2:8]] for r in a])
    img = np.array([[int(v) for v in r[8:11]] if len(r) >= 11 else [0, 0, 0] for r in a],
                   dtype=np.int32)
    vel = np.zeros((natoms, 3))
    if "Velocities" in sec:
        pos = {i: k for k, i in enumerate(ids)}
        for r in sec["Velocities"]:
            vel[pos[int(r[0])]] = [float(v) for v in r[1:4]]
    out = os.path.join(HERE, "water_collapse.npz")
    np.savez_compressed(out, id=ids, type=typ, rho=vals[:, 0], e=vals[:, 1], cv=vals[:, 2],
                        x=vals[:, 3:6], image=img, v=vel, mass=mass, boxlo=box[:, 0],
                        boxhi=box[:, 1])
    print(f"{out}: {natoms} atoms, {ntypes} types, masses {mass[1:]}, box {box.tolist()}")


if __name__ == "__main__":
    sys.exit(main())
