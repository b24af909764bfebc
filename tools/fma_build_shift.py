"""How far the reference's OWN results move between legitimate builds of its sources:
oracle/_ref/libsph_ref.so (g++ -O3 for baseline x86-64: no FMA, nothing contracted -- the
build the oracle is pinned to) against oracle/_ref_fma/libsph_ref.so (the same sources with
-mfma -ffp-contract=fast, as GCC builds them for any FMA machine, e.g. -march=native) and
oracle/_ref_fastmath/libsph_ref.so (the reference's own fast-math recipe,
src/MAKE/Makefile.mingw64-cross:10-11: -O3 -march=core2 -ffast-math).  All take identical inputs (the oracle's C5 / C2 states after setup + a few steps) and compute one
pass of each USER-SPH style; per field: the normwise error and the elementwise relative error
over |b| > 1e-6 ||b||inf (SURVEY 8(d)'s elementwise floor).  A measurement helper (CPU, this
container only: it needs /root/reference for the two builds, oracle/build_ref.sh and
VARIANT=fma / VARIANT=fastmath oracle/build_ref.sh).  Output: profiles/r06/fma_build_shift.json."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import pyoracle as po  # noqa: E402
from scenarios import bubble_physics, bubble_system, c2_system, c3_system  # noqa: E402

A = po.ref()
VARIANTS = {v: po._bind_harness(os.path.join(ROOT, "oracle", "_ref_" + v, "libsph_ref.so"), "ref_")
            for v in ("fma", "fastmath")}
assert A is not None, "oracle/_ref not built"
B = None


def shift(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    m = np.abs(a) > 1e-6 * np.abs(a).max()
    return dict(normwise=float(np.abs(a - b).max() / np.abs(a).max()),
                elementwise=float((np.abs(a - b)[m] / np.abs(a[m])).max()),
                elements_over_1e10=int(((np.abs(a - b)[m] / np.abs(a[m])) > 1e-10).sum()),
                elements_checked=int(m.sum()))


def nz(a):
    return a if a.size else np.zeros(1, np.int32)


def c5_case(nx, slab, steps):
    s = bubble_system(nx, slab=slab)
    ph = bubble_physics(nx, prob=0.3 if slab else 0.5, Tt=-1.0)
    r = po.MpRefRun(s, ph)
    r.setup()
    r.run(steps)
    r._build()   # (lists and ghosts of the current positions)
    g, t, nt = r.g, r.tabs, s.ntypes
    out = {}
    res = {}
    for L, tag in ((A, "base"), (B, "variant")):
        cg = np.zeros((g.nall, 3))
        L.ref_colorgradient(s.dim, nt, g.nlocal, g.nghost, g.x, r.rho_all, r.rm_all, g.type,
                            np.ascontiguousarray(t["cg_alpha"]), np.ascontiguousarray(t["cg_cut"]),
                            r.foff, nz(r.fnb), cg)
        f = np.zeros((g.nall, 3))
        L.ref_taitwater_multiphase(s.dim, nt, g.nlocal, g.nghost, 1, g.x, r.v_all, r.rho_all,
                                   g.type, r.rm_all, ph.rho0, ph.c0, ph.gamma, ph.rbg,
                                   np.ascontiguousarray(t["visc"]),
                                   np.ascontiguousarray(t["tait_cut"]), r.hoff, nz(r.hnb), f)
        fs = np.zeros((g.nall, 3))
        L.ref_surfacetension(s.dim, nt, g.nlocal, g.nghost, 1, g.x, r.rho_all, r.rm_all, g.type,
                             r.cg_all, np.ascontiguousarray(t["st_cut"]), r.hoff, nz(r.hnb), fs)
        de = np.zeros(g.nall)
        ff = np.ascontiguousarray(t["heat_fixflag"], dtype=np.int32)
        tc = np.ascontiguousarray(t["heat_tc"])
        L.ref_heatconduction_phasechange(s.dim, nt, g.nlocal, g.nghost, 1, g.x, r.e_all,
                                         r.cv_all, r.rho_all, r.rm_all, g.type,
                                         np.ascontiguousarray(t["heat_alpha"]), ff.ctypes.data,
                                         tc.ctypes.data, np.ascontiguousarray(t["heat_cut"]),
                                         r.hoff, nz(r.hnb), de)
        res[tag] = dict(colorgradient=cg[:g.nlocal], taitwater_multiphase=f[:g.nlocal],
                        surfacetension=fs[:g.nlocal], heatconduction_phasechange=de[:g.nlocal])
    for k in res["base"]:
        out[k] = shift(res["base"][k], res["variant"][k])
    return out


def c2_case(c3=False):
    s = c3_system(10) if c3 else c2_system(12)
    ph = po.c3_physics() if c3 else po.c2_physics()
    r = po.RefRun(s, ph)
    r.setup()
    r.run(3)
    r._build()
    g, nt = r.g, s.ntypes
    res = {}
    for L, tag in ((A, "base"), (B, "variant")):
        f = np.zeros((g.nall, 3))
        drho = np.zeros(g.nall)
        de = np.zeros(g.nall)
        fn = L.ref_taitwater_morris if ph.morris else L.ref_taitwater
        rho_all = g.gather(r.s.rho)
        vest_all = g.gather(r.vest)
        fn(s.dim, nt, g.nlocal, g.nghost, 1, g.x, vest_all, rho_all, g.type, s.mass, ph.rho0,
           ph.c0, np.ascontiguousarray(ph.visc), np.ascontiguousarray(ph.tait_cut), r.hoff,
           nz(r.hnb), f, drho, de)
        res[tag] = dict(f=f[:g.nlocal], drho=drho[:g.nlocal], de=de[:g.nlocal])
    return {k: shift(res["base"][k], res["variant"][k]) for k in res["base"]}


out = {"note": __doc__}
for v, L in VARIANTS.items():
    B = L
    out[v] = {"C5 bubble 10^3, after setup + 3 steps": c5_case(10, False, 3),
              "C5 slab 8^3, after setup + 3 steps": c5_case(8, True, 3),
              "C2 12^3 jittered, after setup + 3 steps": c2_case(),
              "C3 10^3 two types, after setup + 3 steps": c2_case(c3=True)}
path = os.path.join(ROOT, "profiles", "r06", "fma_build_shift.json")
os.makedirs(os.path.dirname(path), exist_ok=True)
with open(path, "w") as fh:
    json.dump(out, fh, indent=1)
for v in VARIANTS:
    for k, d0 in out[v].items():
        print(v, k)
        for f, d in d0.items():
            print(f"  {f:28s} normwise {d['normwise']:.2e} elementwise {d['elementwise']:.2e} "
                  f"({d['elements_over_1e10']} of {d['elements_checked']} elements over 1e-10)")
