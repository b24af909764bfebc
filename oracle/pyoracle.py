"""ctypes bindings for the parity oracle (TEST INFRASTRUCTURE ONLY).

Two CPU libraries sit behind this module:

* ``oracle/liboracle_sph.so`` -- the plain-C restatement (``sph_oracle.c``); always
  buildable (``make -C oracle``); travels to the GPU box.
* ``oracle/_ref/libsph_ref.so`` -- the reference's own USER-SPH compute code compiled from
  /root/reference/src (``oracle/build_ref.sh``); exists only where it was built.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg import this.
Nothing in the product package (``lammps-sph-multiphase_amd/``) may import it.

Arrays follow LAMMPS conventions (see sph_oracle.h): x/v/vest/f are (n, 3) float64,
per-type tables are length ntypes+1 and per-pair tables (ntypes+1, ntypes+1), 1-based.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle_sph.so")
REF_SO = os.path.join(HERE, "_ref", "libsph_ref.so")

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_lp = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_i, _l, _d = C.c_int, C.c_long, C.c_double


class OrcDomain(C.Structure):
    _fields_ = [("dim", C.c_int), ("boxlo", C.c_double * 3), ("boxhi", C.c_double * 3),
                ("periodic", C.c_int * 3)]


class PcParams(C.Structure):
    """orc_pc_params (sph_oracle.h): fix phase_change arguments."""
    _fields_ = [("dim", C.c_int), ("Tc", C.c_double), ("Tt", C.c_double), ("Hwv", C.c_double),
                ("dr", C.c_double), ("to_mass", C.c_double), ("cutoff", C.c_double),
                ("from_type", C.c_int), ("to_type", C.c_int), ("energy_chance", C.c_int),
                ("change_chance", C.c_double), ("rate", C.c_double), ("dt", C.c_double),
                ("maxattempt", C.c_int), ("sublo", C.c_double * 3),
                ("subhi", C.c_double * 3), ("boxhi", C.c_double * 3), ("top", C.c_int * 3)]


def phasechange(p: "PcParams", seed, nlocal, x, v, vest, cg, e, rmass, rho, cv, type_, off,
                neigh, cap=None):
    """FixPhaseChange::pre_exchange (oracle).  e is updated in place.  Returns
    (seed, nins, new_atoms (nins, 13), parent, dmass)."""
    nall = x.shape[0]
    cap = nall if cap is None else cap
    sd = C.c_int(int(seed))
    dmass = np.zeros(nall)
    rec = np.zeros((max(cap, 1), 13))
    par = np.zeros(max(cap, 1), dtype=np.int32)
    n = lib().orc_phasechange(C.byref(p), C.byref(sd), nlocal, nall, x, v, vest, cg, e, rmass,
                              rho, cv, type_, off, _nz(neigh), dmass, cap, rec.ctypes.data,
                              par.ctypes.data)
    return sd.value, n, rec[:min(n, cap)].copy(), par[:min(n, cap)].copy(), dmass


def pc_params_from_args(args, dim, boxlo, boxhi, dt) -> "PcParams":
    """FixPhaseChange's argument list (fix_phase_change.cpp:46-87, options :358-390) ->
    PcParams for one process owning the whole box."""
    a = [str(v) for v in args]
    p = PcParams()
    p.dim = int(dim)
    p.Tc, p.Tt, p.Hwv, p.dr, p.to_mass, p.cutoff = (float(v) for v in a[3:9])
    p.from_type, p.to_type = int(a[9]), int(a[10])
    m = 13
    if a[m] == "ENERGY":
        p.energy_chance, p.rate, m = 1, float(a[m + 1]), m + 2
    else:
        p.energy_chance, p.change_chance, m = 0, float(a[m]), m + 1
    p.maxattempt = 10
    while m < len(a):
        if a[m] == "attempt":
            p.maxattempt = int(a[m + 1])
        m += 2
    p.dt = float(dt)
    for k in range(3):
        p.sublo[k], p.subhi[k], p.boxhi[k] = float(boxlo[k]), float(boxhi[k]), float(boxhi[k])
        p.top[k] = 1
    return p


def pre_exchange_ref(p: "PcParams", seed, g: "Ghosted", arrays: dict, off, neigh, extra=64):
    """FixPhaseChange::pre_exchange with the reference's memory behaviour (oracle
    orc_pre_exchange_ref).  arrays: x, v, vest, cg, e, rmass, rho, cv, type over the g.nall
    atoms (LAMMPS order).  Returns (seed, new nlocal, arrays after the call, cut to the new
    nlocal)."""
    nmax = g.nall + extra
    a = {}
    for k in ("x", "v", "vest", "cg"):
        b = np.zeros((nmax, 3))
        b[:g.nall] = arrays[k]
        a[k] = b
    for k in ("e", "rmass", "rho", "cv"):
        b = np.zeros(nmax)
        b[:g.nall] = arrays[k]
        a[k] = b
    t = np.zeros(nmax, dtype=np.int32)
    t[:g.nall] = arrays["type"]
    a["type"] = t
    sd = C.c_int(int(seed))
    dm = np.zeros(nmax)
    n = lib().orc_pre_exchange_ref(C.byref(p), C.byref(sd), g.nlocal, g.nghost, nmax, a["x"],
                                   a["v"], a["vest"], a["cg"], a["e"], a["rmass"], a["rho"],
                                   a["cv"], a["type"], off, _nz(neigh), len(g.swap_first) - 1,
                                   g.swap_first, _nz(g.src), dm)
    if n < 0:
        return pre_exchange_ref(p, seed, g, arrays, off, neigh, extra * 4)
    return sd.value, n, {k: v[:n].copy() for k, v in a.items()}


def build_oracle() -> str:
    src = os.path.join(HERE, "sph_oracle.c")
    if (not os.path.exists(ORACLE_SO)) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", HERE, "liboracle_sph.so"], check=True)
    return ORACLE_SO


_lib = None
_ref = None


# the same restatement in other legitimate builds (oracle/Makefile): "fma" = -mfma
# -ffp-contract=fast (any FMA machine), "fastmath" = the reference's own Makefile.mingw64-cross
# flags (-O3 -march=core2 -ffast-math); used only by the build-variation shadows of _Spread
BUILD_SO = {"fma": os.path.join(HERE, "liboracle_sph_fma.so"),
            "fastmath": os.path.join(HERE, "liboracle_sph_fastmath.so")}
_lib_build = {}
_use_build = [None]  # (set while a build-variation shadow steps, _Spread._qf)


def lib():
    """the C restatement (liboracle_sph.so), or -- only while a build-variation shadow of
    _Spread steps -- the same source in another build (BUILD_SO)"""
    b = _use_build[0]
    if b is not None:
        if b not in _lib_build:
            if not os.path.exists(BUILD_SO[b]):
                subprocess.run(["make", "-s", "-C", HERE, os.path.basename(BUILD_SO[b])],
                               check=True)
            _lib_build[b] = _bind_oracle(C.CDLL(BUILD_SO[b]))
        return _lib_build[b]
    return _lib_plain()


def _lib_plain():
    global _lib
    if _lib is None:
        _lib = _bind_oracle(C.CDLL(build_oracle()))
    return _lib


def _bind_oracle(L):
    if True:
        P = C.POINTER(OrcDomain)
        L.orc_pbc.argtypes = [P, _i, _dp]
        L.orc_borders.argtypes = [P, _d, _i, _dp, _ip, _i, _ip, _ip]
        L.orc_borders.restype = _i
        L.orc_borders_ex.argtypes = [P, _d, _i, _dp, _ip, _i, _ip, _ip, _ip, _ip,
                                     C.POINTER(_i)]
        L.orc_borders_ex.restype = _i
        L.orc_reverse_swaps.argtypes = [_i, _i, _ip, _ip, _dp]
        L.orc_pre_exchange_ref.argtypes = [C.POINTER(PcParams), C.POINTER(_i), _i, _i, _i,
                                           _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _ip, _lp,
                                           _ip, _i, _ip, _ip, _dp]
        L.orc_pre_exchange_ref.restype = _i
        L.orc_forward_comm.argtypes = [P, _i, _i, _ip, _ip, _dp, C.c_void_p, C.c_void_p,
                                       C.c_void_p]
        L.orc_reverse_comm.argtypes = [_i, _i, _ip, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_cutneighsq.argtypes = [_i, _dp, _d, _dp, C.POINTER(C.c_double)]
        L.orc_neigh_full.argtypes = [_i, _i, _i, _dp, _ip, _i, _dp, _lp, C.c_void_p, _l]
        L.orc_neigh_full.restype = _l
        L.orc_neigh_half_from_full.argtypes = [_i, _dp, _lp, _ip, _lp, C.c_void_p]
        L.orc_neigh_half_from_full.restype = _l
        L.orc_rhosum.argtypes = [_i, _i, _dp, _ip, _i, _dp, _dp, _dp, _lp, _ip, _dp]
        L.orc_taitwater.argtypes = [_i, _i, _i, _dp, _dp, _dp, _ip, _i, _dp, _dp, _dp, _dp,
                                    _dp, _dp, _dp, _lp, _ip, _dp, _dp, _dp, C.c_void_p]
        L.orc_taitwater_morris.argtypes = L.orc_taitwater.argtypes
        L.orc_heatconduction.argtypes = [_i, _i, _i, _dp, _dp, _dp, _ip, _i, _dp, _dp, _dp,
                                         _dp, _lp, _ip, _dp]
        for n in ("orc_kernel_quintic2d", "orc_kernel_quintic3d", "orc_dw_quintic2d",
                  "orc_dw_quintic3d"):
            getattr(L, n).argtypes = [_d]
            getattr(L, n).restype = _d
        L.orc_set_quintic_factored.argtypes = [_i]
        L.orc_set_quintic_factored.restype = None
        L.orc_set_pow_mode.argtypes = [_i]
        L.orc_set_pow_mode.restype = None
        L.orc_rhosum_multiphase.argtypes = [_i, _i, _dp, _ip, _i, _dp, _dp, _dp, _lp, _ip,
                                            _dp]
        L.orc_taitwater_multiphase.argtypes = [_i, _i, _i, _dp, _dp, _dp, _ip, _i, _dp, _dp,
                                               _dp, _dp, _dp, _dp, _dp, _dp, _dp, _lp, _ip,
                                               _dp]
        L.orc_heatconduction_phasechange.argtypes = [_i, _i, _i, _dp, _dp, _dp, _dp, _dp,
                                                     _ip, _i, _dp, C.c_void_p, C.c_void_p,
                                                     _dp, _dp, _lp, _ip, _dp]
        L.orc_colorgradient.argtypes = [_i, _i, _dp, _dp, _dp, _ip, _i, _dp, _dp, _dp, _lp,
                                        _ip, _dp]
        L.orc_surfacetension.argtypes = [_i, _i, _i, _dp, _dp, _dp, _ip, _i, _dp, _dp, _dp,
                                         _lp, _ip, _dp]
        L.orc_park_uniform.argtypes = [C.POINTER(_i)]
        L.orc_park_uniform.restype = _d
        L.orc_phasechange.argtypes = [C.POINTER(PcParams), C.POINTER(_i), _i, _i, _dp, _dp,
                                      _dp, _dp, _dp, _dp, _dp, _dp, _ip, _lp, _ip, _dp, _i,
                                      C.c_void_p, C.c_void_p]
        L.orc_phasechange.restype = _i
        L.orc_phasechange_finish.argtypes = [_i, _dp, _dp, _dp]
        L.orc_meso_setup.argtypes = [_i, _dp, _dp]
        L.orc_meso_initial.argtypes = [_i, _d, _d, _ip, _dp, C.c_void_p, _dp, _dp, _dp, _dp,
                                       _dp, _dp, _dp, _dp]
        L.orc_meso_final.argtypes = [_i, _d, _ip, _dp, C.c_void_p, _dp, _dp, _dp, _dp, _dp,
                                     _dp]
        L.orc_meso_setup_g.argtypes = [_i, _ip, _i, _dp, _dp]
        L.orc_meso_initial_g.argtypes = [_i, _d, _d, _ip, _i, _dp, C.c_void_p, _dp, _dp, _dp,
                                         _dp, _dp, _dp, _dp, _dp]
        L.orc_meso_final_g.argtypes = [_i, _d, _ip, _i, _dp, C.c_void_p, _dp, _dp, _dp, _dp,
                                       _dp, _dp]
        L.orc_meso_stationary.argtypes = [_i, _d, _ip, _i, _dp, _dp, _dp, _dp]
        L.orc_gravity.argtypes = [_i, _ip, _i, _dp, C.c_void_p, _dp, _dp]
    return L


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def _bind_harness(path, pre):
    """ctypes signatures of oracle/ref_harness.cpp's entry points (prefix ref_ or shim_)"""
    R = C.CDLL(path)
    g = lambda n: getattr(R, pre + n)  # noqa: E731
    g("neigh_full").argtypes = [_i, _i, _i, _i, _dp, _ip, _dp, _dp, _dp, _dp, _d, _dp, _lp,
                                C.c_void_p, _l]
    g("neigh_full").restype = _l
    g("neigh_half_from_full").argtypes = [_i, _i, _dp, _lp, _ip, _lp, C.c_void_p]
    g("neigh_half_from_full").restype = _l
    g("fix_meso").argtypes = [_i, _i, _i, _i, _d, _ip, _i, _dp, _dp, _dp, _dp, _dp, _dp, _dp,
                              _dp, _dp]
    g("rhosum").argtypes = [_i, _i, _i, _i, _dp, _ip, _dp, _dp, _lp, _ip, _dp]
    g("taitwater").argtypes = [_i, _i, _i, _i, _i, _dp, _dp, _dp, _ip, _dp, _dp, _dp, _dp, _dp,
                               _lp, _ip, _dp, _dp, _dp]
    g("taitwater_morris").argtypes = g("taitwater").argtypes
    g("heatconduction").argtypes = [_i, _i, _i, _i, _i, _dp, _dp, _dp, _ip, _dp, _dp, _dp, _lp,
                                    _ip, _dp]
    g("rhosum_multiphase").argtypes = [_i, _i, _i, _i, _dp, _ip, _dp, _dp, _lp, _ip, _dp]
    g("taitwater_multiphase").argtypes = [_i, _i, _i, _i, _i, _dp, _dp, _dp, _ip, _dp, _dp,
                                          _dp, _dp, _dp, _dp, _dp, _lp, _ip, _dp]
    g("heatconduction_phasechange").argtypes = [_i, _i, _i, _i, _i, _dp, _dp, _dp, _dp, _dp,
                                                _ip, _dp, C.c_void_p, C.c_void_p, _dp, _lp,
                                                _ip, _dp]
    g("colorgradient").argtypes = [_i, _i, _i, _i, _dp, _dp, _dp, _ip, _dp, _dp, _lp, _ip, _dp]
    g("surfacetension").argtypes = [_i, _i, _i, _i, _i, _dp, _dp, _dp, _ip, _dp, _dp, _lp, _ip,
                                    _dp]
    g("pc_new").argtypes = [_i, _i, _dp, _dp, _l, _d, _i, C.POINTER(C.c_char_p)]
    g("pc_new").restype = C.c_void_p
    g("pc_pre_exchange").argtypes = [C.c_void_p, _l, _i, _i, _i, _dp, _dp, _dp, _dp, _dp, _dp,
                                     _dp, _dp, _ip, _lp, _ip, _i, _ip, _ip, C.POINTER(_l)]
    g("pc_pre_exchange").restype = _i
    g("pack_restart").argtypes = [_i, _i, _dp, _ip, _ip, _ip, _ip, _dp, _dp, _dp, _dp, _dp, _dp,
                                  _dp, _i, _dp]
    g("pack_restart").restype = _i
    g("set_device_lists").argtypes = [_i, _d]
    g("set_device_lists").restype = None
    g("rhosum_skip").argtypes = [_i, _i, _i, _i, _dp, _ip, _dp, _dp, _i, _ip, _lp, _ip, _ip,
                                 _ip, _dp]
    for n in ("kernel_quintic2d", "kernel_quintic3d", "dw_quintic2d", "dw_quintic3d"):
        g(n).argtypes = [_d]
        g(n).restype = _d
    # the ref_* names on either library, so callers can swap one for the other
    class _Named:
        pass
    out = _Named()
    out.lib = R
    for n in ("neigh_full", "neigh_half_from_full", "fix_meso", "rhosum", "taitwater",
              "taitwater_morris", "heatconduction", "rhosum_multiphase", "taitwater_multiphase",
              "heatconduction_phasechange", "colorgradient", "surfacetension", "pc_new",
              "pc_pre_exchange", "pack_restart", "kernel_quintic2d", "kernel_quintic3d",
              "dw_quintic2d", "dw_quintic3d", "set_device_lists", "rhosum_skip"):
        setattr(out, "ref_" + n, g(n))
    return out


def ref():
    """The reference's own compute code (oracle/_ref/libsph_ref.so), or None if it was not
    built."""
    global _ref
    if _ref is None and ref_available():
        _ref = _bind_harness(REF_SO, "ref_")
    return _ref


SHIM_SO = os.path.join(HERE, "_ref", "libsph_shim.so")
_shim = None


def shim_available() -> bool:
    return os.path.exists(SHIM_SO)


def shim():
    """The same harness driving this repo's drop-in LAMMPS classes (sph/<style>/hip, fix
    phase_change/hip -> libsph_hip.so): oracle/_ref/libsph_shim.so, entry points under their
    ref_* names.  None if it was not built."""
    global _shim
    if _shim is None and shim_available():
        _shim = _bind_harness(SHIM_SO, "shim_")
        f = _shim.lib.shim_style_lookup
        f.argtypes = [_i, C.c_char_p, C.c_char_p, C.c_char_p, _i]
        f.restype = _i
    return _shim


# ---------------------------------------------------------------------------------------
# System description
# ---------------------------------------------------------------------------------------
@dataclass
class System:
    """Owned particles of one periodic (or not) orthogonal box, LAMMPS atom_style meso."""

    dim: int
    boxlo: np.ndarray
    boxhi: np.ndarray
    periodic: tuple
    x: np.ndarray            # (n,3)
    v: np.ndarray            # (n,3)
    type: np.ndarray         # (n,) int32, 1-based
    rho: np.ndarray
    e: np.ndarray
    cv: np.ndarray
    ntypes: int
    mass: np.ndarray         # (ntypes+1,)
    rmass: np.ndarray | None = None
    extra: dict = field(default_factory=dict)

    @property
    def n(self) -> int:
        return int(self.x.shape[0])

    def domain(self) -> OrcDomain:
        d = OrcDomain()
        d.dim = self.dim
        for k in range(3):
            d.boxlo[k] = float(self.boxlo[k])
            d.boxhi[k] = float(self.boxhi[k])
            d.periodic[k] = int(self.periodic[k])
        return d

    def copy(self) -> "System":
        s = System(self.dim, self.boxlo.copy(), self.boxhi.copy(), tuple(self.periodic),
                   self.x.copy(), self.v.copy(), self.type.copy(), self.rho.copy(),
                   self.e.copy(), self.cv.copy(), self.ntypes, self.mass.copy(),
                   None if self.rmass is None else self.rmass.copy(), dict(self.extra))
        return s


def cubic_lattice(n: int, dx: float = 1.0, jitter: float = 0.1, seed: int = 12345,
                  vel_sigma: float = 0.01, vseed: int = 4928459, ntypes: int = 1,
                  type2_frac: float = 0.0, tseed: int = 87287, dim: int = 3,
                  mass=(1.0,), rho=(1.0,), e=(0.0,), cv=(1.0,)) -> System:
    """SURVEY.md section 8(d) synthetic boxes: sc lattice n^dim, spacing dx, periodic, every
    coordinate jittered by U(-jitter, jitter)*dx, gaussian velocities; optional type 2 by
    Bernoulli(type2_frac).  (numpy RNG -- not LAMMPS' RanPark -- the same arrays are fed
    to every implementation under test.)"""
    nz = n if dim == 3 else 1
    g = np.stack(np.meshgrid(np.arange(n), np.arange(n), np.arange(nz), indexing="ij"),
                 -1).reshape(-1, 3)
    # LAMMPS create_atoms loops z outermost then y then x; order atoms the same way
    g = g[np.lexsort((g[:, 0], g[:, 1], g[:, 2]))]
    x = g.astype(np.float64) * dx
    rng = np.random.default_rng(seed)
    x += rng.uniform(-jitter, jitter, size=x.shape) * dx
    if dim == 2:
        x[:, 2] = 0.0
    N = x.shape[0]
    vr = np.random.default_rng(vseed)
    v = vr.normal(0.0, vel_sigma, size=(N, 3))
    if dim == 2:
        v[:, 2] = 0.0
    t = np.ones(N, dtype=np.int32)
    if ntypes >= 2 and type2_frac > 0:
        tr = np.random.default_rng(tseed)
        t[tr.random(N) < type2_frac] = 2
    mass_t = np.zeros(ntypes + 1)
    rho_t = np.zeros(ntypes + 1)
    e_t = np.zeros(ntypes + 1)
    cv_t = np.zeros(ntypes + 1)
    for k in range(1, ntypes + 1):
        mass_t[k] = mass[min(k - 1, len(mass) - 1)]
        rho_t[k] = rho[min(k - 1, len(rho) - 1)]
        e_t[k] = e[min(k - 1, len(e) - 1)]
        cv_t[k] = cv[min(k - 1, len(cv) - 1)]
    boxlo = np.zeros(3)
    boxhi = np.array([n * dx, n * dx, (n * dx) if dim == 3 else 0.5 * dx])
    if dim == 2:
        boxlo[2] = -0.5 * dx
    return System(dim, boxlo, boxhi, (1, 1, 1 if dim == 3 else 0), x, v, t, rho_t[t].copy(),
                  e_t[t].copy(), cv_t[t].copy(), ntypes, mass_t)


# ---------------------------------------------------------------------------------------
# Wrappers around the C restatement
# ---------------------------------------------------------------------------------------
@dataclass
class Ghosted:
    """Owned + ghost atoms after CommBrick::borders (one process)."""

    nlocal: int
    nghost: int
    x: np.ndarray            # (nall,3)
    type: np.ndarray
    owner: np.ndarray        # (nghost,)
    image: np.ndarray        # (nghost,3)
    src: np.ndarray | None = None         # (nghost,) sendlist entry each ghost came from
    swap_first: np.ndarray | None = None  # (nswap+1,) first ghost of each CommBrick swap

    @property
    def nall(self) -> int:
        return self.nlocal + self.nghost

    def gather(self, a: np.ndarray) -> np.ndarray:
        """Extend a per-owned array to owned+ghost by copying from owners."""
        return np.concatenate([a, a[self.owner]], axis=0)


def borders(sysm: System, cutghost: float, x: np.ndarray | None = None) -> Ghosted:
    L = lib()
    xo = sysm.x if x is None else x
    n = xo.shape[0]
    nmax = int(n * 3 + 1000)
    while True:
        xa = np.zeros((nmax, 3))
        xa[:n] = xo
        ta = np.zeros(nmax, dtype=np.int32)
        ta[:n] = sysm.type
        own = np.zeros(nmax, dtype=np.int32)
        img = np.zeros(3 * nmax, dtype=np.int32)
        d = sysm.domain()
        src = np.zeros(nmax, dtype=np.int32)
        sf = np.zeros(8, dtype=np.int32)
        ns = C.c_int(0)
        ng = L.orc_borders_ex(C.byref(d), cutghost, n, xa, ta, nmax, own, img, src, sf,
                              C.byref(ns))
        if ng >= 0:
            break
        nmax *= 2
    return Ghosted(n, ng, xa[:n + ng].copy(), ta[:n + ng].copy(), own[:ng].copy(),
                   img[:3 * ng].reshape(-1, 3).copy(), src[:ng].copy(),
                   sf[:ns.value + 1].copy())


def cutneighsq(ntypes: int, cutmax: np.ndarray, skin: float):
    out = np.zeros((ntypes + 1, ntypes + 1))
    cm = C.c_double()
    lib().orc_cutneighsq(ntypes, np.ascontiguousarray(cutmax, dtype=np.float64), skin, out,
                         C.byref(cm))
    return out, cm.value


def neigh_full(dim: int, g: Ghosted, ntypes: int, cns: np.ndarray):
    L = lib()
    off = np.zeros(g.nlocal + 1, dtype=np.int64)
    tot = L.orc_neigh_full(dim, g.nlocal, g.nall, g.x, g.type, ntypes, cns, off, None, 0)
    neigh = np.zeros(max(tot, 1), dtype=np.int32)
    tot2 = L.orc_neigh_full(dim, g.nlocal, g.nall, g.x, g.type, ntypes, cns, off,
                            neigh.ctypes.data, tot)
    assert tot2 == tot
    return off, neigh[:tot]


def half_from_full(g: Ghosted, foff: np.ndarray, fneigh: np.ndarray):
    L = lib()
    hoff = np.zeros(g.nlocal + 1, dtype=np.int64)
    fn = np.ascontiguousarray(fneigh if fneigh.size else np.zeros(1, np.int32))
    tot = L.orc_neigh_half_from_full(g.nlocal, g.x, foff, fn, hoff, None)
    h = np.zeros(max(tot, 1), dtype=np.int32)
    L.orc_neigh_half_from_full(g.nlocal, g.x, foff, fn, hoff, h.ctypes.data)
    return hoff, h[:tot]


def _reverse_rows(off, nb):
    """every CSR row reversed"""
    off = np.asarray(off, dtype=np.int64)
    if nb.size == 0:
        return nb.copy()
    row = np.repeat(np.arange(len(off) - 1), np.diff(off))
    k = np.arange(nb.size, dtype=np.int64)
    return nb[off[row] + off[row + 1] - 1 - k]


def _rotate_rows(off, nb):
    """every CSR row rotated by half its length"""
    off = np.asarray(off, dtype=np.int64)
    if nb.size == 0:
        return nb.copy()
    ln = np.diff(off)
    row = np.repeat(np.arange(len(off) - 1), ln)
    k = np.arange(nb.size, dtype=np.int64) - off[row]
    L = ln[row]
    return nb[off[row] + (k + L // 2) % np.maximum(L, 1)]


def _reorder_rows(off, nb, how):
    """how: True / "reverse" = each row reversed; "rotate" = each row rotated by half"""
    if how is True or how == "reverse":
        return _reverse_rows(off, nb)
    return _rotate_rows(off, nb)


def _nz(a):
    return a if a.size else np.zeros(1, dtype=a.dtype)


def rhosum(dim, g: Ghosted, ntypes, mass, cut, off, neigh):
    cut = np.ascontiguousarray(cut, dtype=np.float64)
    cutsq = cut * cut
    rho = np.zeros(g.nall)
    lib().orc_rhosum(dim, g.nlocal, g.x, g.type, ntypes, mass, cut, cutsq, off, _nz(neigh),
                     rho)
    return rho[:g.nlocal]


def taitwater(dim, g: Ghosted, ntypes, newton, vest_all, rho_all, mass, rho0, c0, visc,
              cut, off, neigh, morris=False, B=None, virial=False):
    cut = np.ascontiguousarray(cut, dtype=np.float64)
    cutsq = cut * cut
    if B is None:
        B = c0 * c0 * rho0 / 7.0
    f = np.zeros((g.nall, 3))
    drho = np.zeros(g.nall)
    de = np.zeros(g.nall)
    vir = np.zeros(6)
    fn = lib().orc_taitwater_morris if morris else lib().orc_taitwater
    fn(dim, g.nlocal, newton, g.x, np.ascontiguousarray(vest_all), np.ascontiguousarray(rho_all),
       g.type, ntypes, mass, rho0, c0, np.ascontiguousarray(B, dtype=np.float64),
       np.ascontiguousarray(visc, dtype=np.float64), cut, cutsq, off, _nz(neigh), f, drho, de,
       vir.ctypes.data if virial else None)
    if virial:
        return f, drho, de, vir
    return f, drho, de


def heatconduction(dim, g: Ghosted, ntypes, newton, e_all, rho_all, mass, alpha, cut, off,
                   neigh):
    cut = np.ascontiguousarray(cut, dtype=np.float64)
    de = np.zeros(g.nall)
    lib().orc_heatconduction(dim, g.nlocal, newton, g.x, np.ascontiguousarray(e_all),
                             np.ascontiguousarray(rho_all), g.type, ntypes, mass,
                             np.ascontiguousarray(alpha, dtype=np.float64), cut, cut * cut,
                             off, _nz(neigh), de)
    return de


def reverse_comm(g: Ghosted, f=None, drho=None, de=None):
    lib().orc_reverse_comm(g.nlocal, g.nghost, g.owner if g.nghost else np.zeros(1, np.int32),
                           None if f is None else f.ctypes.data,
                           None if drho is None else drho.ctypes.data,
                           None if de is None else de.ctypes.data)


# ---------------------------------------------------------------------------------------
# Reference-faithful Verlet driver over the C restatement (one process, newton on, half
# lists derived from full ones, reverse comm of ghost forces) -- the CPU twin of the
# device engine's step, used as the multi-step parity oracle.
#   Verlet::setup  src/verlet.cpp:88-139      Verlet::run  src/verlet.cpp:222-308
# ---------------------------------------------------------------------------------------
@dataclass
class Physics:
    """Hybrid/overlay pair stack of the BASELINE configs (per-type (nt+1), per-pair
    (nt+1,nt+1) tables, 1-based)."""

    skin: float = 0.3
    dt: float = 1e-3
    every: int = 10
    rhosum_nstep: int = 1
    rhosum_cut: np.ndarray | None = None
    tait: bool = True
    morris: bool = False
    rho0: np.ndarray | None = None
    c0: np.ndarray | None = None
    visc: np.ndarray | None = None
    tait_cut: np.ndarray | None = None
    heat: bool = False
    alpha: np.ndarray | None = None
    heat_cut: np.ndarray | None = None
    # fix meso/stationary on the types of this mask, fix meso on the others
    stationary_mask: int = 0
    # fix gravity (style vector, acceleration per unit mass) on the types of gravity_mask
    # (0 = all)
    gravity: tuple = (0.0, 0.0, 0.0)
    gravity_mask: int = 0

    def rho_keep(self, nt):
        """Types sph/rhosum has no coefficient pair for: under hybrid/overlay their rows are
        on its skip list (pair_hybrid.cpp:439-471) and keep their rho."""
        keep = np.zeros(nt + 1, dtype=bool)
        if self.rhosum_cut is None:
            return keep
        c = np.asarray(self.rhosum_cut)
        for t in range(1, nt + 1):
            keep[t] = not any(c[min(t, j), max(t, j)] > 0 for j in range(1, nt + 1))
        return keep

    def cutmax(self, nt):
        cm = np.zeros((nt + 1, nt + 1))
        for on, c in ((self.rhosum_nstep > 0, self.rhosum_cut), (self.tait, self.tait_cut),
                      (self.heat, self.heat_cut)):
            if on and c is not None:
                cm = np.maximum(cm, np.asarray(c))
        # init_one mirrors the upper triangle
        for i in range(nt + 1):
            for j in range(i):
                cm[i, j] = cm[j, i]
        return cm


def c2_physics(h=3.0) -> Physics:
    """rhosum(nstep 1, h) + taitwater(rho0 1, c0 10, visc 0.1, h), m=1."""
    t = np.zeros((2, 2))
    t[1, 1] = h
    v = np.zeros((2, 2))
    v[1, 1] = 0.1
    return Physics(rhosum_cut=t.copy(), rho0=np.array([0.0, 1.0]), c0=np.array([0.0, 10.0]),
                   visc=v, tait_cut=t.copy())


def c3_physics(h=3.0) -> Physics:
    """two types, taitwater/morris (rho0 1|0.5, c0 10, visc 0.01, h) +
    heatconduction (D 0.1, h); no rhosum."""
    t = np.zeros((3, 3))
    t[1:, 1:] = h
    v = np.zeros((3, 3))
    v[1:, 1:] = 0.01
    a = np.zeros((3, 3))
    a[1:, 1:] = 0.1
    return Physics(rhosum_nstep=0, rhosum_cut=None, morris=True, rho0=np.array([0.0, 1.0, 0.5]),
                   c0=np.array([0.0, 10.0, 10.0]), visc=v, tait_cut=t.copy(), heat=True,
                   alpha=a, heat_cut=t.copy())


SPREAD_ORDERS = (True, "rotate")  # rows reversed; rows rotated by half their length
SPREAD_ULP_SEED = 4242


def ulp_perturbed(sysm: "System", seed=SPREAD_ULP_SEED) -> "System":
    """a copy of the system with x, v, rho, e each moved by one ulp, random sign"""
    s = sysm.copy()
    rng = np.random.default_rng(seed)
    x0 = s.x.copy()
    for name in ("x", "v", "rho", "e"):
        a = getattr(s, name)
        a += np.spacing(a) * rng.choice((-1.0, 1.0), size=a.shape)
    for d in range(s.dim):  # (an atom moved out of the box keeps its coordinate)
        out = (s.x[:, d] < s.boxlo[d]) | (s.x[:, d] >= s.boxhi[d])
        s.x[out, d] = x0[out, d]
    return s


class _Spread:
    """spread=True: the run keeps three shadow runs of the same physics, stepped with it --
    every list row reversed, every row rotated (SPREAD_ORDERS), and the inputs moved by one
    ulp (ulp_perturbed); spread(k) is, per element of field k, the largest distance of their
    results from this run's: how far the reference's own result moves under a reordered
    summation or last-bit changes of its inputs (the tests' elementwise bar).
    Every shadow runs the reference's own arithmetic (no shadow evaluates anything in the
    engine's form: round 5's factored-quintic shadow is gone, the engine evaluates the
    reference's expanded quintic instead).  Reordering alone misses elements whose reference
    sum happens to be order-insensitive while its terms cancel (a C3 atom between two phases:
    spread < 1e-18 absolute): the ulp shadow covers those.  For the C5 stack (MpRefRun) two
    more shadows run the same source in two other legitimate builds: for an FMA machine
    (liboracle_sph_fma.so: GCC contracting a*b + c, as a -march=native build of LAMMPS does)
    and with the reference's own fast-math recipe (liboracle_sph_fastmath.so: -O3
    -march=core2 -ffast-math, src/MAKE/Makefile.mingw64-cross:10-11).  On the bubble lattice
    the reference's sums cancel pairwise, so neither reordering nor a one-ulp input moves
    them, while any change in a term's last bits does: the reference's OWN sources built
    those ways move C5 colour-gradient / multiphase-force elements by up to ~1e-9 / ~1e-7
    relative (tools/fma_build_shift.py, profiles/r06/fma_build_shift.json), so the C5 bar is
    16 x how far the reference moves between legitimate builds of itself."""

    def _init_spread(self, spread, make, make_ulp, build=False):
        self.alts = []
        self.qfact = False
        self.build = None
        if spread:
            # spread="lean" (the 1M tests): one reordering + the ulp shadow
            for how in (SPREAD_ORDERS[:1] if spread == "lean" else SPREAD_ORDERS):
                a = make()
                a.rev = how
                self.alts.append(a)
            self.alts.append(make_ulp())
            if build:  # (C5: the same source in two other builds, see the class doc)
                for b in ("fma", "fastmath"):
                    a = make()
                    a.build = b
                    self.alts.append(a)

    def _qf(self, on):
        if self.build:
            _use_build[0] = self.build if on else None
        if self.qfact:  # (tools/cg_probe.py: a run evaluating the quintic dW factored)
            lib().orc_set_quintic_factored(1 if on else 0)
        if getattr(self, "powm", 0):  # (orc_set_pow_mode: 1 correctly rounded, 2 one ulp up)
            lib().orc_set_pow_mode(self.powm if on else 0)

    def field(self, k):
        s = self.s
        if k in ("rho", "x", "v", "e", "rmass", "cv"):
            return getattr(s, k)
        return getattr(self, k)

    def build_rel(self, k):
        """the largest elementwise relative distance (over |b| > 1e-6 ||b||inf) of field k
        between this run and its build-variation shadows (the same source in the other
        legitimate builds, BUILD_SO): the reference's own field-level reproducibility across
        its builds; None without such shadows"""
        want = np.asarray(self.field(k), dtype=np.float64).ravel()
        if not want.size or not np.abs(want).max():
            return None
        m = np.abs(want) > 1e-6 * np.abs(want).max()
        out = None
        for a in self.alts:
            if not a.build or a.s.n != self.s.n or not np.array_equal(a.s.type, self.s.type):
                continue
            b = np.asarray(a.field(k), dtype=np.float64).ravel()
            r = float((np.abs(b[m] - want[m]) / np.abs(want[m])).max())
            out = r if out is None else max(out, r)
        return out

    def spread(self, k):
        """per-element spread of field k (None without shadow runs)"""
        if not self.alts:
            return None
        want = np.asarray(self.field(k), dtype=np.float64)
        out = np.zeros_like(want)
        used = 0
        for a in self.alts:
            # (a shadow whose fix phase_change took another decision -- a candidate's
            # temperature within its last bits of the threshold -- is left out)
            if a.s.n != self.s.n or not np.array_equal(a.s.type, self.s.type):
                continue
            out = np.maximum(out, np.abs(np.asarray(a.field(k), dtype=np.float64) - want))
            used += 1
        return out if used else None


class RefRun(_Spread):
    """Owned state + the reference's per-step sequence, computed by the C restatement."""

    def __init__(self, sysm: System, ph: Physics, spread=False):
        self.s = sysm.copy()
        self.ph = ph
        nt = sysm.ntypes
        self.cns, self.cutneighmax = cutneighsq(nt, ph.cutmax(nt), ph.skin)
        n = sysm.n
        self.vest = np.zeros((n, 3))          # AtomVecMeso::create_atom: vest = 0
        self.f = np.zeros((n, 3))
        self.drho = np.zeros(n)
        self.de = np.zeros(n)
        self.step = 0
        self.last_build = 0
        self.dtf = 0.5 * ph.dt
        self.B = None if ph.rho0 is None else ph.c0 * ph.c0 * ph.rho0 / 7.0
        # rev: the same run with every full-list row (and so every half row) reversed (True)
        # or shuffled (an int seed) -- the reference's own result under a reordered summation
        # (the tests' elementwise bar)
        self.rev = False
        self.rev_builds = 0
        self._init_spread(spread, lambda: RefRun(sysm, ph),
                          lambda: RefRun(ulp_perturbed(sysm), ph))

    # -- helpers -------------------------------------------------------------------------
    def _build(self):
        s = self.s
        x0 = s.x.copy()
        lib().orc_pbc(C.byref(s.domain()), s.n, s.x)
        self.image = getattr(self, "image", np.zeros((s.n, 3), np.int64)) + pbc_images(s, x0)
        self.g = borders(s, self.cutneighmax)
        self.foff, self.fnb = neigh_full(s.dim, self.g, s.ntypes, self.cns)
        if self.rev:  # (list rows reordered: the reference's own reordering spread)
            self.fnb = _reorder_rows(self.foff, self.fnb, self.rev)
            self.rev_builds += 1
        self.hoff, self.hnb = half_from_full(self.g, self.foff, self.fnb)
        # ghost copies of the border-packed per-atom fields
        self.vest_all = self.g.gather(self.vest)
        self.rho_all = self.g.gather(s.rho)
        self.e_all = self.g.gather(s.e)

    def _forward(self):
        g, s = self.g, self.s
        d = s.domain()
        xa = g.x
        xa[:s.n] = s.x
        self.vest_all = self.g.gather(self.vest)
        self.rho_all = self.g.gather(s.rho)
        self.e_all = self.g.gather(s.e)
        lib().orc_forward_comm(C.byref(d), g.nlocal, g.nghost, g.owner,
                               np.ascontiguousarray(g.image.ravel()), xa, None, None, None)

    def _force(self):
        s, g, ph = self.s, self.g, self.ph
        nt = s.ntypes
        nall = g.nall
        g.x[:s.n] = s.x
        if ph.rhosum_nstep > 0 and self.step % ph.rhosum_nstep == 0:
            with np.errstate(all="ignore"):      # (skipped types' self terms: h = 0)
                rho = rhosum(s.dim, g, nt, s.mass, ph.rhosum_cut, self.foff, self.fnb)
            upd = ~ph.rho_keep(nt)[s.type]
            s.rho[upd] = rho[upd]
            self.rho_all = g.gather(s.rho)       # forward_comm_pair
        f = np.zeros((nall, 3))
        drho = np.zeros(nall)
        de = np.zeros(nall)
        if ph.tait:
            f, drho, de = taitwater(s.dim, g, nt, 1, self.vest_all, self.rho_all, s.mass, ph.rho0,
                                    ph.c0, ph.visc, ph.tait_cut, self.hoff, self.hnb,
                                    morris=ph.morris, B=self.B)
        if ph.heat:
            de += heatconduction(s.dim, g, nt, 1, self.e_all, self.rho_all, s.mass, ph.alpha,
                                 ph.heat_cut, self.hoff, self.hnb)
        reverse_comm(g, f, drho, de)
        if any(a != 0.0 for a in ph.gravity):   # post_force
            lib().orc_gravity(s.n, s.type, ph.gravity_mask, s.mass, None,
                              np.asarray(ph.gravity, dtype=np.float64), f)
        self.f = f[:s.n].copy()
        self.drho = drho[:s.n].copy()
        self.de = de[:s.n].copy()

    # -- Verlet --------------------------------------------------------------------------
    def setup(self):
        self.step = 0
        self._build()                             # borders before setup_pre_force
        # FixMeso::setup_pre_force on the meso group (owned only; ghosts keep their
        # border-time vest); meso/stationary has none
        lib().orc_meso_setup_g(self.s.n, self.s.type, self._meso_mask(), self.s.v, self.vest)
        self.vest_all[:self.s.n] = self.vest
        self._force()
        self.last_build = 0
        for a in self.alts:
            a.setup()

    def _meso_mask(self):
        """fix meso's group: every type not under meso/stationary (0 = all)"""
        sm = self.ph.stationary_mask
        if sm == 0:
            return 0
        return sum(1 << t for t in range(1, self.s.ntypes + 1) if not (sm >> t) & 1)

    def run(self, nsteps):
        s, L = self.s, lib()
        mm, sm = self._meso_mask(), self.ph.stationary_mask
        for _ in range(nsteps):
            self.step += 1
            if mm or not sm:
                L.orc_meso_initial_g(s.n, self.ph.dt, self.dtf, s.type, mm, s.mass, None, s.x,
                                     s.v, self.f, self.vest, s.rho, self.drho, s.e, self.de)
            if sm:
                L.orc_meso_stationary(s.n, self.dtf, s.type, sm, s.rho, self.drho, s.e,
                                      self.de)
            if (self.step - self.last_build) % self.ph.every == 0:
                self._build()
                self.last_build = self.step
            else:
                self._forward()
            self._force()
            if mm or not sm:
                L.orc_meso_final_g(s.n, self.dtf, s.type, mm, s.mass, None, s.v, self.f,
                                   s.rho, self.drho, s.e, self.de)
            if sm:
                L.orc_meso_stationary(s.n, self.dtf, s.type, sm, s.rho, self.drho, s.e,
                                      self.de)
        for a in self.alts:
            a.run(nsteps)

    def numneigh_full(self):
        return np.diff(self.foff).astype(np.int32)


# ---------------------------------------------------------------------------------------
# C5: the multiphase stack of examples/USER/sph/bubble_growth/bubble.lmp:57-73 on atom_style
# meso/multiphase (per-atom rmass, cv, colorgradient), Verlet with fix meso (rmass) and
# fix phase_change (pre_exchange on its reneighbor steps), one process, newton on.
# ---------------------------------------------------------------------------------------
@dataclass
class MpPhysics:
    """pair_style hybrid/overlay sph/rhosum/multiphase N sph/colorgradient N
    sph/taitwater/multiphase sph/surfacetension sph/heatconduction/phasechange (tables are
    (nt+1, nt+1), upper triangle read) + fix phase_change (pc dict, or None)."""

    skin: float = 0.0
    dt: float = 1e-4
    every: int = 1
    rhosum_nstep: int = 1
    rhosum_cut: np.ndarray | None = None
    cg_nstep: int = 1
    cg_alpha: np.ndarray | None = None
    cg_cut: np.ndarray | None = None
    tait: bool = True
    rho0: np.ndarray | None = None
    c0: np.ndarray | None = None
    gamma: np.ndarray | None = None
    rbg: np.ndarray | None = None
    visc: np.ndarray | None = None
    tait_cut: np.ndarray | None = None
    st: bool = True
    st_cut: np.ndarray | None = None
    heat: bool = True
    heat_alpha: np.ndarray | None = None
    heat_cut: np.ndarray | None = None
    heat_fixflag: np.ndarray | None = None
    heat_tc: np.ndarray | None = None
    pc: dict | None = None
    # atom_modify sort N binsize (atom.cpp:63, 540-551): Atom::sort every N steps (0 = never);
    # binsize 0 = half the neighbor cutoff (setup_sort_bins, atom.cpp:1660-1726)
    sortfreq: int = 1000
    sort_binsize: float = 0.0

    def tables(self):
        return [(self.rhosum_nstep > 0, self.rhosum_cut), (self.cg_nstep > 0, self.cg_cut),
                (self.tait, self.tait_cut), (self.st, self.st_cut), (self.heat, self.heat_cut)]

    def cutmax(self, nt):
        cm = np.zeros((nt + 1, nt + 1))
        for on, c in self.tables():
            if on and c is not None:
                cm = np.maximum(cm, np.asarray(c))
        for i in range(nt + 1):
            for j in range(i):
                cm[i, j] = cm[j, i]
        return cm


def _sym(t):
    """coeff() upper triangle mirrored like init_one"""
    t = np.array(t, dtype=np.float64 if np.asarray(t).dtype.kind == "f" else np.int32)
    for i in range(t.shape[0]):
        for j in range(i):
            t[i, j] = t[j, i]
    return np.ascontiguousarray(t)


def pc_params(sysm: System, pc: dict, dt: float) -> PcParams:
    p = PcParams()
    p.dim = sysm.dim
    for k in ("Tc", "Tt", "Hwv", "dr", "to_mass", "cutoff"):
        setattr(p, k, float(pc[k]))
    p.from_type, p.to_type = int(pc["from_type"]), int(pc["to_type"])
    p.energy_chance = int(pc.get("energy_chance", 0))
    p.change_chance = float(pc.get("prob", 0.0))
    p.rate = float(pc.get("rate", 0.0))
    p.dt = dt
    p.maxattempt = int(pc.get("maxattempt", 10))
    for k in range(3):
        p.sublo[k], p.subhi[k], p.boxhi[k] = sysm.boxlo[k], sysm.boxhi[k], sysm.boxhi[k]
        p.top[k] = 1
    return p


# ---------------------------------------------------------------------------------------
# Brick decomposition (CommBrick on a uniform processor grid): the per-rank views fix
# phase_change sees when the box is split over several ranks
# ---------------------------------------------------------------------------------------
def brick_grid(sysm: System, pg):
    """Domain::set_local_box with uniform splits and CommBrick's procneigh, ranks x fastest
    (the engine's formula, sph_engine_create): per rank its grid location, sub-box and the
    lower/upper neighbour along each dimension."""
    P = int(pg[0] * pg[1] * pg[2])
    out = []
    for r in range(P):
        loc = [r % pg[0], (r // pg[0]) % pg[1], r // (pg[0] * pg[1])]
        lo, hi = np.zeros(3), np.zeros(3)
        nb = np.zeros((3, 2), dtype=np.int64)
        for k in range(3):
            prd = float(sysm.boxhi[k] - sysm.boxlo[k])
            lo[k] = sysm.boxlo[k] + prd * (loc[k] / pg[k])
            hi[k] = (sysm.boxhi[k] if loc[k] + 1 == pg[k]
                     else sysm.boxlo[k] + prd * ((loc[k] + 1) / pg[k]))
            for side, step in ((0, -1), (1, 1)):
                m = list(loc)
                m[k] = (m[k] + step) % pg[k]
                nb[k, side] = (m[2] * pg[1] + m[1]) * pg[0] + m[0]
        out.append(dict(loc=loc, lo=lo, hi=hi, neigh=nb))
    return out


def brick_owner(sysm: System, x: np.ndarray, pg) -> np.ndarray:
    """The rank owning each atom: sublo <= x < subhi per dimension (CommBrick::exchange)."""
    r = np.zeros(x.shape[0], dtype=np.int64)
    mult = 1
    for d in range(3):
        prd = float(sysm.boxhi[d] - sysm.boxlo[d])
        c = np.zeros(x.shape[0], dtype=np.int64)
        for k in range(1, pg[d]):
            c += (x[:, d] >= sysm.boxlo[d] + prd * (k / pg[d])).astype(np.int64)
        r += c * mult
        mult *= pg[d]
    return r


@dataclass
class BrickView:
    """One rank's atoms after CommBrick::borders over a processor grid: owned atoms in the
    rank's local order (borders_bricks' `local`), then each swap's ghosts in the order the
    sending rank scanned its atoms (comm_brick.cpp:733-800)."""

    rank: int
    nlocal: int
    gid: np.ndarray          # (nall,) global (tag-order) index of the atom or its origin
    x: np.ndarray            # (nall,3) at borders time
    type: np.ndarray
    image: np.ndarray        # (nall,3) periodic image of each copy (0 for owned)
    swap_first: list         # first ghost of each swap, + nghost
    src_rank: np.ndarray     # (nghost,) sending rank of each ghost
    src_idx: np.ndarray      # (nghost,) its index on the sending rank (sendlist entry)
    lo: np.ndarray = None
    hi: np.ndarray = None
    loc: list = None
    off: np.ndarray = None   # full list of the build (local indices)
    nb: np.ndarray = None
    hoff: np.ndarray = None  # its half list (half_from_full_newton on the rank's atoms)
    hnb: np.ndarray = None

    @property
    def nghost(self) -> int:
        return int(self.gid.shape[0]) - self.nlocal


def hole_fill(local: np.ndarray, leave: np.ndarray):
    """CommBrick::exchange's scan of one dimension (comm_brick.cpp:620-632): a departing
    atom's slot takes the last atom (avec->copy(nlocal-1, i)), which is examined next.
    local: atom ids in local order, leave: their flags -> (the kept ids in their new local
    order, the departed ids in send-buffer order)."""
    a = np.array(local, dtype=np.int64)
    lv = np.array(leave, dtype=bool)
    n, i, sent = a.size, 0, []
    while True:
        nz = np.flatnonzero(lv[i:n])
        if nz.size == 0:
            break
        i += int(nz[0])
        sent.append(int(a[i]))
        n -= 1
        a[i], lv[i] = a[n], lv[n]
    return a[:n].copy(), np.array(sent, dtype=np.int64)


def exchange_bricks(sysm: System, pg, local: list, x: np.ndarray | None = None) -> list:
    """CommBrick::exchange (comm_brick.cpp:573-680) over the grid: per dimension every rank
    sends the atoms outside its slab (hole fill, above) to its lower neighbour (and, with more
    than 2 ranks along the dimension, the same buffer to its upper one); a rank appends the
    received atoms inside its slab, the upper neighbour's buffer first.  local[r] = rank r's
    atom ids in local order; returns the new lists."""
    xo = sysm.x if x is None else x
    grid = brick_grid(sysm, pg)
    local = [np.asarray(l, dtype=np.int64) for l in local]
    for d in range(sysm.dim):
        if pg[d] == 1:
            continue   # (nothing leaves a periodic dimension after Domain::pbc)
        sent = []
        for r, b in enumerate(grid):
            xd = xo[local[r], d]
            local[r], snd = hole_fill(local[r], (xd < b["lo"][d]) | (xd >= b["hi"][d]))
            sent.append(snd)
        for r, b in enumerate(grid):
            srcs = [int(b["neigh"][d, 1])] + ([int(b["neigh"][d, 0])] if pg[d] > 2 else [])
            add = [local[r]]
            for src in srcs:
                g = sent[src]
                xd = xo[g, d]
                add.append(g[(xd >= b["lo"][d]) & (xd < b["hi"][d])])
            local[r] = np.concatenate(add)
    return local


def sort_bricks(sysm: System, pg, local: list, binsize: float, x: np.ndarray | None = None):
    """Atom::sort (atom.cpp:1555-1654) on every rank: bins of setup_sort_bins (:1660-1726)
    over the rank's sub-box, atoms listed bin by bin, in their current order within a bin;
    one bin = no sort."""
    xo = sysm.x if x is None else x
    out = []
    for r, b in enumerate(brick_grid(sysm, pg)):
        ids = np.asarray(local[r], dtype=np.int64)
        bininv = 1.0 / binsize
        nb, inv = [], []
        for k in range(3):
            ext = float(b["hi"][k] - b["lo"][k])
            m = int(ext * bininv)
            if k == 2 and sysm.dim == 2:
                m = 1
            m = max(m, 1)
            nb.append(m)
            inv.append(m / ext)
        if nb[0] * nb[1] * nb[2] == 1:
            out.append(ids)
            continue
        c = []
        for k in range(3):
            t = np.trunc((xo[ids, k] - b["lo"][k]) * inv[k])
            c.append(np.clip(t, 0, nb[k] - 1).astype(np.int64))
        ibin = c[2] * nb[1] * nb[0] + c[1] * nb[0] + c[0]
        out.append(ids[np.argsort(ibin, kind="stable")])
    return out


def borders_bricks(sysm: System, cutghost: float, pg, x: np.ndarray | None = None,
                   local: list | None = None):
    """CommBrick::borders (comm_brick.cpp:696-864, maxneed 1) on every rank of the grid at
    once: per dimension both swaps scan owned + earlier dimensions' ghosts, the lower swap's
    ghosts are appended before the upper one's; a brick at the periodic edge shifts the
    copies by the box length (one add per coordinate).  local[r]: rank r's owned atoms in
    their local order (default: the atoms inside its sub-box in tag order)."""
    xo = sysm.x if x is None else x
    grid = brick_grid(sysm, pg)
    own = brick_owner(sysm, xo, pg) if local is None else None
    V = []
    for r, b in enumerate(grid):
        idx = np.nonzero(own == r)[0] if local is None else np.asarray(local[r], np.int64)
        V.append(dict(gid=[idx], x=[xo[idx].copy()], type=[sysm.type[idx].copy()],
                      image=[np.zeros((idx.size, 3), dtype=np.int64)], sf=[], srank=[],
                      sidx=[], nlocal=int(idx.size)))
    cat = lambda v, k: np.concatenate(v[k]) if len(v[k]) > 1 else v[k][0]
    for d in range(sysm.dim):
        prd = float(sysm.boxhi[d] - sysm.boxlo[d])
        snap = [dict(gid=cat(v, "gid"), x=cat(v, "x"), type=cat(v, "type"),
                     image=cat(v, "image")) for v in V]
        incoming = [[None, None] for _ in V]
        for ineed in (0, 1):
            for r, b in enumerate(grid):
                loc = b["loc"][d]
                if sysm.periodic[d]:
                    sendflag = True
                else:
                    sendflag = loc > 0 if ineed == 0 else loc < pg[d] - 1
                if ineed == 0:
                    lo, hi = -1.0e20, b["lo"][d] + cutghost
                    pbc = 1 if loc == 0 else 0
                else:
                    lo, hi = b["hi"][d] - cutghost, 1.0e20
                    pbc = -1 if loc == pg[d] - 1 else 0
                sv = snap[r]
                xs = sv["x"]
                if sendflag:
                    sel = np.nonzero((xs[:, d] >= lo) & (xs[:, d] <= hi))[0]
                else:
                    sel = np.zeros(0, dtype=np.int64)
                xg = xs[sel].copy()
                if pbc:
                    xg[:, d] = xg[:, d] + pbc * prd
                img = sv["image"][sel].copy()
                img[:, d] += pbc
                incoming[int(b["neigh"][d, ineed])][ineed] = (
                    sv["gid"][sel], xg, sv["type"][sel], img, r, sel)
        for r, v in enumerate(V):
            for ineed in (0, 1):
                v["sf"].append(sum(a.shape[0] for a in v["gid"]) - v["nlocal"])
                inc = incoming[r][ineed]
                if inc is None:
                    continue
                g, xg, t, img, src, sel = inc
                v["gid"].append(g)
                v["x"].append(xg)
                v["type"].append(t)
                v["image"].append(img)
                v["srank"].append(np.full(sel.size, src, dtype=np.int64))
                v["sidx"].append(sel)
    out = []
    for r, v in enumerate(V):
        gid = cat(v, "gid")
        v["sf"].append(gid.shape[0] - v["nlocal"])
        sr = np.concatenate(v["srank"]) if v["srank"] else np.zeros(0, np.int64)
        si = np.concatenate(v["sidx"]) if v["sidx"] else np.zeros(0, np.int64)
        b = grid[r]
        out.append(BrickView(r, v["nlocal"], gid, cat(v, "x"), cat(v, "type").astype(np.int32),
                             cat(v, "image"), v["sf"], sr, si, b["lo"], b["hi"], b["loc"]))
    return out


class MpRefRun(_Spread):
    """C5 Verlet (verlet.cpp:222-308) over the C restatement: initial_integrate (fix meso,
    rmass) -> [pre_exchange: fix phase_change] -> pbc/borders/lists or forward comm (comm
    vel yes: x, v, rho, cg, rmass, e, vest) -> rhosum/multiphase, colorgradient (owned rows;
    the styles' misnamed pack_comm moves nothing, so ghosts keep their comm-time rho and cg,
    SURVEY A.6-1) -> taitwater/multiphase, surfacetension, heatconduction/phasechange on the
    half list with Newton-3 -> reverse comm (f, de) -> final_integrate.  The arrays are kept
    in tag order (new atoms appended); with fix phase_change each rank's LAMMPS local order is
    tracked beside them (self.local): read order, CommBrick::exchange's hole fill, Atom::sort
    at setup and every ph.sortfreq steps (verlet.cpp:106, 251), created atoms appended."""

    def __init__(self, sysm: System, ph: MpPhysics, cg=None, procgrid=None, spread=False,
                 read_order=None):
        self.s = sysm.copy()
        # read_order: the atom ids in the order LAMMPS read them (data-file lines), which is
        # its initial local order; default tag order
        self.read_order = None if read_order is None else np.asarray(read_order, np.int64)
        assert self.s.rmass is not None
        # procgrid: fix phase_change as it runs on a grid of ranks (each rank scans its owned
        # atoms in its local order with its own RanPark of the same seed,
        # fix_phase_change.cpp:116, creates atoms only in its sub-box, and the ghosts' dmass
        # goes back over the ranks' swaps); the pair styles, integrators and lists do not
        # depend on the decomposition
        self.pg = None if procgrid is None or int(np.prod(procgrid)) == 1 else tuple(procgrid)
        # the candidates' order is LAMMPS' local order: one process that sorts atoms runs the
        # per-rank path on a 1x1x1 grid, whose views list the owned atoms in that order
        if ph.pc is not None and ph.sortfreq > 0 and self.pg is None:
            self.pg = (1, 1, 1)
        self.local = None                    # per rank: atom ids in local order (pc only)
        self.nextsort = 0
        # rev: every list row walked backwards -- the same physics in another summation
        # order, so a test can size its tolerance to how far the reference's own result moves
        # under reordering where a sum nearly cancels (ill-conditioned atoms)
        self.rev = False
        self._init_spread(spread, lambda: MpRefRun(sysm, ph, cg=cg, procgrid=procgrid,
                                                   read_order=read_order),
                          lambda: MpRefRun(ulp_perturbed(sysm), ph, cg=cg, procgrid=procgrid,
                                           read_order=read_order), build=True)
        self.ph = ph
        nt = sysm.ntypes
        self.cns, self.cutneighmax = cutneighsq(nt, ph.cutmax(nt), ph.skin)
        n = sysm.n
        self.vest = np.zeros((n, 3))
        self.cg = np.zeros((n, 3)) if cg is None else np.array(cg, dtype=np.float64)
        self.f = np.zeros((n, 3))
        self.drho = np.zeros(n)
        self.de = np.zeros(n)
        self.step = 0
        self.last_build = 0
        self.dtf = 0.5 * ph.dt
        self.next_pc = 1                      # next_reneighbor = ntimestep + 1 (:120)
        self.seed = int(ph.pc["seed"]) if ph.pc else 0
        if self.pg:
            self.seeds = [self.seed] * int(np.prod(self.pg))
        self.ninserted = 0
        self.tabs = {}
        for name in ("rhosum_cut", "cg_alpha", "cg_cut", "visc", "tait_cut", "st_cut",
                     "heat_alpha", "heat_cut", "heat_tc"):
            v = getattr(ph, name)
            self.tabs[name] = _sym(v) if v is not None else np.zeros((nt + 1, nt + 1))
        ff = ph.heat_fixflag if ph.heat_fixflag is not None else np.zeros((nt + 1, nt + 1))
        self.tabs["heat_fixflag"] = _sym(np.asarray(ff, dtype=np.int32))
        if ph.tait:
            g = np.where(ph.gamma != 0, ph.gamma, 1.0)     # (type 0 unused)
            self.B = np.ascontiguousarray(ph.c0 * ph.c0 * ph.rho0 / g, dtype=np.float64)

    def _ghost_fields(self):
        s, g = self.s, self.g
        self.v_all = g.gather(s.v)
        self.vest_all = g.gather(self.vest)
        self.rho_all = g.gather(s.rho)
        self.e_all = g.gather(s.e)
        self.cv_all = g.gather(s.cv)
        self.rm_all = g.gather(s.rmass)
        self.cg_all = g.gather(self.cg)
        if self.pg:   # the owned values as communicated: what every rank's ghosts hold
            self.comm = dict(x=s.x.copy(), v=s.v.copy(), vest=self.vest.copy(),
                             rho=s.rho.copy(), e=s.e.copy(), cv=s.cv.copy(),
                             rmass=s.rmass.copy(), cg=self.cg.copy())

    def _build(self):
        s = self.s
        x0 = s.x.copy()
        lib().orc_pbc(C.byref(s.domain()), s.n, s.x)
        im = getattr(self, "image", np.zeros((0, 3), np.int64))
        if im.shape[0] < s.n:   # (created atoms: zero image, create_atom)
            im = np.concatenate([im, np.zeros((s.n - im.shape[0], 3), np.int64)])
        self.image = im + pbc_images(s, x0)
        self.g = borders(s, self.cutneighmax)
        self.foff, self.fnb = neigh_full(s.dim, self.g, s.ntypes, self.cns)
        if self.rev:
            self.fnb = _reorder_rows(self.foff, self.fnb, self.rev)
        self.hoff, self.hnb = half_from_full(self.g, self.foff, self.fnb)
        self._ghost_fields()
        if self.pg:
            if self.ph.pc is not None:
                self._local_order()
            self.bviews = borders_bricks(s, self.cutneighmax, self.pg, local=self.local)
            for bv in self.bviews:
                gh = Ghosted(bv.nlocal, bv.nghost, np.ascontiguousarray(bv.x), bv.type,
                             np.zeros(bv.nghost, np.int32), np.zeros((bv.nghost, 3), np.int32))
                bv.off, bv.nb = neigh_full(s.dim, gh, s.ntypes, self.cns)
                if self.rev:
                    bv.nb = _reorder_rows(bv.off, bv.nb, self.rev)
                bv.hoff, bv.hnb = half_from_full(gh, bv.off, bv.nb)

    def _local_order(self):
        """Between Domain::pbc and CommBrick::borders (verlet.cpp:100-107, 245-253): the
        exchange, then Atom::sort at setup and once step >= nextsort (nextsort =
        (step/sortfreq)*sortfreq + sortfreq, atom.cpp:1561).  The first call lists every
        rank's atoms in read order (read_order, default tag order, within the rank)."""
        s, ph = self.s, self.ph
        if self.local is None:
            own = brick_owner(s, s.x, self.pg)
            ro = self.read_order if self.read_order is not None else np.arange(s.n)
            self.local = [ro[own[ro] == r] for r in range(int(np.prod(self.pg)))]
        else:
            self.local = exchange_bricks(s, self.pg, self.local)
        if ph.sortfreq > 0 and (self.step == 0 or self.step >= self.nextsort):
            self.nextsort = (self.step // ph.sortfreq) * ph.sortfreq + ph.sortfreq
            bs = ph.sort_binsize if ph.sort_binsize > 0 else 0.5 * self.cutneighmax
            self.local = sort_bricks(s, self.pg, self.local, bs)
        assert sum(l.size for l in self.local) == s.n

    def _forward(self):
        g, s = self.g, self.s
        xa = g.x
        xa[:s.n] = s.x
        lib().orc_forward_comm(C.byref(s.domain()), g.nlocal, g.nghost, g.owner,
                               np.ascontiguousarray(g.image.ravel()), xa, None, None, None)
        self._ghost_fields()

    def _ghost_x(self, bv):
        """A rank's ghost positions as last communicated: the origin's x then plus its image
        (one add per coordinate, as every hop adds it)."""
        s = self.s
        prd = np.asarray(s.boxhi, dtype=np.float64) - np.asarray(s.boxlo, dtype=np.float64)
        nl = bv.nlocal
        xg = self.comm["x"][bv.gid[nl:]].copy()
        im = bv.image[nl:]
        for d in range(3):
            m = im[:, d] != 0
            xg[m, d] = xg[m, d] + im[m, d] * prd[d]
        return xg

    def _reverse_bricks(self, arrs):
        """CommBrick::reverse_comm over the grid: swaps in reverse order, every rank's ghost
        values added onto the atoms they were copied from on the sending rank."""
        nsw = len(self.bviews[0].swap_first) - 1
        for sw in range(nsw - 1, -1, -1):
            for bv in self.bviews:
                g0, g1 = bv.swap_first[sw], bv.swap_first[sw + 1]
                if g1 == g0:
                    continue
                src = int(bv.src_rank[g0])
                np.add.at(arrs[src], bv.src_idx[g0:g1],
                          arrs[bv.rank][bv.nlocal + g0:bv.nlocal + g1])

    def _force_bricks(self):
        """The stack rank by rank: every rank's styles see its owned atoms' fresh rho and
        colour gradient but its ghosts' values as communicated (the styles' pack_comm moves
        nothing) -- so which neighbours are ghosts, and hence the results,
        depend on the decomposition.  rhosum/multiphase itself reads only x and rmass."""
        s, ph, L = self.s, self.ph, lib()
        nt, n = s.ntypes, s.n
        T = self.tabs
        c = self.comm
        loc = []
        for bv in self.bviews:
            nl = bv.nlocal
            own, gg = bv.gid[:nl], bv.gid[nl:]
            loc.append(dict(x=np.ascontiguousarray(np.concatenate([s.x[own], self._ghost_x(bv)])),
                            rm=np.concatenate([s.rmass[own], c["rmass"][gg]]),
                            rho=np.concatenate([s.rho[own], c["rho"][gg]]),
                            v=np.concatenate([s.v[own], c["v"][gg]]),
                            e=np.concatenate([s.e[own], c["e"][gg]]),
                            cv=np.concatenate([s.cv[own], c["cv"][gg]]),
                            cg=np.concatenate([self.cg[own], c["cg"][gg]])))
        if ph.rhosum_nstep > 0 and self.step % ph.rhosum_nstep == 0:
            cc = T["rhosum_cut"]
            for bv, a in zip(self.bviews, loc):
                nl = bv.nlocal
                rho = np.zeros(a["x"].shape[0])
                L.orc_rhosum_multiphase(s.dim, nl, a["x"], bv.type, nt, a["rm"], cc, cc * cc,
                                        bv.off, _nz(bv.nb), rho)
                a["rho"][:nl] = rho[:nl]
                s.rho[bv.gid[:nl]] = rho[:nl]
        if ph.cg_nstep > 0 and self.step % ph.cg_nstep == 0:
            cc = T["cg_cut"]
            for bv, a in zip(self.bviews, loc):
                nl = bv.nlocal
                cgo = np.zeros((a["x"].shape[0], 3))
                L.orc_colorgradient(s.dim, nl, a["x"], a["rho"], a["rm"], bv.type, nt,
                                    T["cg_alpha"], cc, cc * cc, bv.off, _nz(bv.nb), cgo)
                a["cg"][:nl] = cgo[:nl]
                self.cg[bv.gid[:nl]] = cgo[:nl]
        fs, ds = [], []
        for bv, a in zip(self.bviews, loc):
            nl = bv.nlocal
            nall = a["x"].shape[0]
            f = np.zeros((nall, 3))
            de = np.zeros(nall)
            if ph.tait:
                cc = T["tait_cut"]
                L.orc_taitwater_multiphase(s.dim, nl, 1, a["x"], np.ascontiguousarray(a["v"]),
                                           a["rho"], bv.type, nt, a["rm"],
                                           np.ascontiguousarray(ph.rho0, dtype=np.float64),
                                           np.ascontiguousarray(ph.c0, dtype=np.float64), self.B,
                                           np.ascontiguousarray(ph.gamma, dtype=np.float64),
                                           np.ascontiguousarray(ph.rbg, dtype=np.float64),
                                           T["visc"], cc, cc * cc, bv.hoff, _nz(bv.hnb), f)
            if ph.st:
                cc = T["st_cut"]
                L.orc_surfacetension(s.dim, nl, 1, a["x"], a["rho"], a["rm"], bv.type, nt,
                                     np.ascontiguousarray(a["cg"]), cc, cc * cc, bv.hoff,
                                     _nz(bv.hnb), f)
            if ph.heat:
                cc = T["heat_cut"]
                L.orc_heatconduction_phasechange(s.dim, nl, 1, a["x"], a["e"], a["cv"],
                                                 a["rho"], a["rm"], bv.type, nt,
                                                 T["heat_alpha"], T["heat_fixflag"].ctypes.data,
                                                 T["heat_tc"].ctypes.data, cc, cc * cc, bv.hoff,
                                                 _nz(bv.hnb), de)
            fs.append(f)
            ds.append(de)
        self._reverse_bricks(fs)
        self._reverse_bricks(ds)
        self.f = np.zeros((n, 3))
        self.de = np.zeros(n)
        for bv, f, de in zip(self.bviews, fs, ds):
            self.f[bv.gid[:bv.nlocal]] = f[:bv.nlocal]
            self.de[bv.gid[:bv.nlocal]] = de[:bv.nlocal]
        self.drho = np.zeros(n)
        self.rho_all[:n] = s.rho
        self.cg_all[:n] = self.cg

    def _force(self):
        if self.pg:
            return self._force_bricks()
        s, g, ph, L = self.s, self.g, self.ph, lib()
        nt, n, nall = s.ntypes, s.n, g.nall
        T = self.tabs
        g.x[:n] = s.x
        if ph.rhosum_nstep > 0 and self.step % ph.rhosum_nstep == 0:
            rho = np.zeros(nall)
            c = T["rhosum_cut"]
            L.orc_rhosum_multiphase(s.dim, n, g.x, g.type, nt, self.rm_all, c, c * c,
                                    self.foff, _nz(self.fnb), rho)
            s.rho[:] = rho[:n]
            self.rho_all[:n] = s.rho           # ghosts keep their comm-time rho (A.6-1)
        if ph.cg_nstep > 0 and self.step % ph.cg_nstep == 0:
            cgo = np.zeros((nall, 3))
            c = T["cg_cut"]
            L.orc_colorgradient(s.dim, n, g.x, self.rho_all, self.rm_all, g.type, nt,
                                T["cg_alpha"], c, c * c, self.foff, _nz(self.fnb), cgo)
            self.cg[:] = cgo[:n]
            self.cg_all[:n] = self.cg          # ghosts keep their comm-time cg (A.6-1)
        f = np.zeros((nall, 3))
        de = np.zeros(nall)
        if ph.tait:
            c = T["tait_cut"]
            # the style reads atom->v (comm vel yes), pair_sph_taitwater_multiphase.cpp:103
            L.orc_taitwater_multiphase(s.dim, n, 1, g.x, np.ascontiguousarray(self.v_all),
                                       self.rho_all, g.type, nt, self.rm_all,
                                       np.ascontiguousarray(ph.rho0, dtype=np.float64),
                                       np.ascontiguousarray(ph.c0, dtype=np.float64), self.B,
                                       np.ascontiguousarray(ph.gamma, dtype=np.float64),
                                       np.ascontiguousarray(ph.rbg, dtype=np.float64),
                                       T["visc"], c, c * c, self.hoff, _nz(self.hnb), f)
        if ph.st:
            c = T["st_cut"]
            L.orc_surfacetension(s.dim, n, 1, g.x, self.rho_all, self.rm_all, g.type, nt,
                                 np.ascontiguousarray(self.cg_all), c, c * c, self.hoff,
                                 _nz(self.hnb), f)
        if ph.heat:
            c = T["heat_cut"]
            L.orc_heatconduction_phasechange(s.dim, n, 1, g.x, self.e_all, self.cv_all,
                                             self.rho_all, self.rm_all, g.type, nt,
                                             T["heat_alpha"], T["heat_fixflag"].ctypes.data,
                                             T["heat_tc"].ctypes.data,
                                             c, c * c, self.hoff, _nz(self.hnb), de)
        reverse_comm(g, f, None, de)
        self.f = f[:n].copy()
        self.drho = np.zeros(n)
        self.de = de[:n].copy()

    def _phase_change(self):
        """FixPhaseChange::pre_exchange (fix_phase_change.cpp:167-352) on the last build's
        full list: owned x as integrated, ghosts as last communicated.  self.pc_exact (the
        default): orc_pre_exchange_ref, the reference's own memory behaviour (created atoms
        over ghost slots, reverse comm along the swaps; pinned to the reference by
        tests/test_phasechange_golden.py).  Otherwise the port semantics (orc_phasechange:
        every candidate on the atoms as found)."""
        if self.pg:
            return self._phase_change_bricks()
        s, g, L = self.s, self.g, lib()
        n = s.n
        p = pc_params(s, self.ph.pc, self.ph.dt)
        arrays = dict(x=np.concatenate([s.x, g.x[n:]]), v=np.concatenate([s.v, self.v_all[n:]]),
                      vest=np.concatenate([self.vest, self.vest_all[n:]]),
                      cg=np.concatenate([self.cg, self.cg_all[n:]]),
                      e=np.concatenate([s.e, self.e_all[n:]]),
                      rmass=np.concatenate([s.rmass, self.rm_all[n:]]),
                      rho=np.concatenate([s.rho, self.rho_all[n:]]),
                      cv=np.concatenate([s.cv, self.cv_all[n:]]), type=g.type)
        arrays = {k: np.ascontiguousarray(v) for k, v in arrays.items()}
        if getattr(self, "pc_exact", True):
            self.seed, nnew, out = pre_exchange_ref(p, self.seed, g, arrays, self.foff, self.fnb)
            nins = nnew - n
            s.x, s.v, s.e, s.rmass = out["x"], out["v"], out["e"], out["rmass"]
            s.rho, s.cv, s.type = out["rho"], out["cv"], out["type"]
            self.vest, self.cg = out["vest"], out["cg"]
        else:
            e_all = arrays["e"]
            seed, nins, rec, par, dmass = phasechange(
                p, self.seed, n, arrays["x"], arrays["v"], arrays["vest"], arrays["cg"], e_all,
                arrays["rmass"], arrays["rho"], arrays["cv"], g.type, self.foff, self.fnb)
            self.seed = seed
            s.e[:] = e_all[:n]
            L.orc_reverse_swaps(n, len(g.swap_first) - 1, g.swap_first, _nz(g.src), dmass)
            L.orc_phasechange_finish(n, dmass, s.rmass, s.e)
            if nins:
                to = int(self.ph.pc["to_type"])
                s.x = np.concatenate([s.x, rec[:, 0:3]])
                s.v = np.concatenate([s.v, rec[:, 3:6]])
                self.vest = np.concatenate([self.vest, rec[:, 6:9]])
                s.e = np.concatenate([s.e, rec[:, 9]])
                s.rmass = np.concatenate([s.rmass, rec[:, 10]])
                s.rho = np.concatenate([s.rho, rec[:, 11]])
                s.cv = np.concatenate([s.cv, rec[:, 12]])
                s.type = np.concatenate([s.type, np.full(nins, to, dtype=np.int32)])
                self.cg = np.concatenate([self.cg, np.zeros((nins, 3))])   # create_atom
        if nins:
            self.f = np.concatenate([self.f, np.zeros((nins, 3))])
            self.drho = np.concatenate([self.drho, np.zeros(nins)])
            self.de = np.concatenate([self.de, np.zeros(nins)])
            self.ninserted += nins
        return nins

    def _phase_change_bricks(self):
        """pre_exchange on every rank of the grid (orc_pre_exchange_ref up to the reverse
        comm, on the rank's view: owned atoms as integrated, ghosts as last communicated,
        the last build's full list), then reverse_comm_fix over the ranks' swaps in reverse
        order, the finish loop per rank, and Atom::tag_extend: the created atoms take the
        next tags rank by rank (atom.cpp:598-630, MPI_Scan order)."""
        s, L = self.s, lib()
        c = self.comm
        res = []
        for bv in self.bviews:
            nl = bv.nlocal
            own, gg = bv.gid[:nl], bv.gid[nl:]
            xg = self._ghost_x(bv)
            arrays = dict(x=np.concatenate([s.x[own], xg]),
                          v=np.concatenate([s.v[own], c["v"][gg]]),
                          vest=np.concatenate([self.vest[own], c["vest"][gg]]),
                          cg=np.concatenate([self.cg[own], c["cg"][gg]]),
                          e=np.concatenate([s.e[own], c["e"][gg]]),
                          rmass=np.concatenate([s.rmass[own], c["rmass"][gg]]),
                          rho=np.concatenate([s.rho[own], c["rho"][gg]]),
                          cv=np.concatenate([s.cv[own], c["cv"][gg]]), type=bv.type)
            p = pc_params(s, self.ph.pc, self.ph.dt)
            for k in range(3):
                p.sublo[k], p.subhi[k] = bv.lo[k], bv.hi[k]
                p.top[k] = int(bv.loc[k] == self.pg[k] - 1)
            extra = 64
            while True:
                nmax = bv.nlocal + bv.nghost + extra
                a = {}
                for k in ("x", "v", "vest", "cg"):
                    a[k] = np.zeros((nmax, 3))
                    a[k][:arrays[k].shape[0]] = arrays[k]
                for k in ("e", "rmass", "rho", "cv"):
                    a[k] = np.zeros(nmax)
                    a[k][:arrays[k].shape[0]] = arrays[k]
                a["type"] = np.zeros(nmax, dtype=np.int32)
                a["type"][:bv.type.shape[0]] = bv.type
                sd = C.c_int(int(self.seeds[bv.rank]))
                dm = np.zeros(nmax)
                ncur = L.orc_pre_exchange_ref(C.byref(p), C.byref(sd), nl, bv.nghost, nmax,
                                              a["x"], a["v"], a["vest"], a["cg"], a["e"],
                                              a["rmass"], a["rho"], a["cv"], a["type"], bv.off,
                                              _nz(bv.nb), -1, np.zeros(1, np.int32),
                                              np.zeros(1, np.int32), dm)
                if ncur >= 0:
                    break
                extra *= 4
            self.seeds[bv.rank] = sd.value
            res.append((a, dm, ncur))
        self._reverse_bricks([r[1] for r in res])   # reverse_comm_fix of dmass
        new = []
        nxt = s.n
        for bv, (a, dm, ncur) in zip(self.bviews, res):
            nl = bv.nlocal
            own = bv.gid[:nl]
            rm, e = a["rmass"][:nl].copy(), a["e"][:nl].copy()
            L.orc_phasechange_finish(nl, np.ascontiguousarray(dm[:nl]), rm, e)
            s.rmass[own] = rm
            s.e[own] = e
            if ncur > nl:
                new.append({k: v[nl:ncur].copy() for k, v in a.items()})
                if self.local is not None:   # created at the end of the rank's local list
                    self.local[bv.rank] = np.concatenate(
                        [self.local[bv.rank], np.arange(nxt, nxt + ncur - nl)])
                nxt += ncur - nl
        nins = sum(d["x"].shape[0] for d in new)
        if nins:
            cat = lambda k: np.concatenate([d[k] for d in new])
            s.x = np.concatenate([s.x, cat("x")])
            s.v = np.concatenate([s.v, cat("v")])
            self.vest = np.concatenate([self.vest, cat("vest")])
            s.e = np.concatenate([s.e, cat("e")])
            s.rmass = np.concatenate([s.rmass, cat("rmass")])
            s.rho = np.concatenate([s.rho, cat("rho")])
            s.cv = np.concatenate([s.cv, cat("cv")])
            s.type = np.concatenate([s.type, cat("type")])
            self.cg = np.concatenate([self.cg, cat("cg")])
            self.f = np.concatenate([self.f, np.zeros((nins, 3))])
            self.drho = np.concatenate([self.drho, np.zeros(nins)])
            self.de = np.concatenate([self.de, np.zeros(nins)])
            self.ninserted += nins
        return nins

    def setup(self):
        self.step = 0
        self._qf(True)
        self._build()
        lib().orc_meso_setup(self.s.n, self.s.v, self.vest)   # FixMeso::setup_pre_force
        self._force()
        self._qf(False)
        self.last_build = 0
        for a in self.alts:
            a.setup()

    def run(self, nsteps):
        self._qf(True)
        try:
            self._run(nsteps)
        finally:
            self._qf(False)
        for a in self.alts:
            a.run(nsteps)

    def _run(self, nsteps):
        s, L, ph = self.s, lib(), self.ph
        for _ in range(nsteps):
            self.step += 1
            L.orc_meso_initial_g(s.n, ph.dt, self.dtf, s.type, 0, s.mass, s.rmass.ctypes.data,
                                 s.x, s.v, self.f, self.vest, s.rho, self.drho, s.e, self.de)
            pc_due = ph.pc is not None and self.step == self.next_pc
            if pc_due or (self.step - self.last_build) % ph.every == 0:
                if pc_due:
                    self._phase_change()
                    self.next_pc += int(ph.pc.get("nevery", 1))
                self._build()
                self.last_build = self.step
            else:
                self._forward()
            self._force()
            L.orc_meso_final_g(s.n, self.dtf, s.type, 0, s.mass, s.rmass.ctypes.data, s.v,
                               self.f, s.rho, self.drho, s.e, self.de)

    def numneigh_full(self):
        return np.diff(self.foff).astype(np.int32)


# ---------------------------------------------------------------------------------------
# Restart records (the per-atom layout of the reference's restart files) and image flags
# ---------------------------------------------------------------------------------------
IMGMAX, IMGBITS = 512, 10   # lmptype.h (LAMMPS_SMALLBIG): imageint = int, 10 bits per dim


def img_pack(image):
    """(n, 3) image counts -> packed imageint, lmptype.h / atom.cpp"""
    im = np.asarray(image, dtype=np.int64) + IMGMAX
    return ((im[:, 2] << (2 * IMGBITS)) | (im[:, 1] << IMGBITS) | im[:, 0]).astype(np.int64)


def pbc_images(sysm: System, x_before: np.ndarray) -> np.ndarray:
    """The image change Domain::pbc (domain.cpp:478-560) applied: -1 for a wrap from below
    lo (x += prd), +1 for one from at/above hi (x -= prd)."""
    prd = sysm.boxhi - sysm.boxlo
    d = np.zeros(x_before.shape, dtype=np.int64)
    for k in range(3):
        if sysm.periodic[k] and prd[k] > 0:
            d[:, k] = np.rint((x_before[:, k] - sysm.x[:, k]) / prd[k]).astype(np.int64)
    return d


def _ubuf(a):
    return np.asarray(a, dtype=np.int64).view(np.float64)


def pack_restart_meso(x, tag, type_, image, v, rho, e, cv, vest, mask=None):
    """AtomVecMeso::pack_restart (atom_vec_meso.cpp:726-757): 17 doubles per atom, the ints
    as ubuf bit patterns (lmptype.h)."""
    n = x.shape[0]
    mask = np.ones(n, np.int64) if mask is None else mask
    out = np.zeros((n, 17))
    out[:, 0] = 17
    out[:, 1:4] = x
    out[:, 4] = _ubuf(tag)
    out[:, 5] = _ubuf(type_)
    out[:, 6] = _ubuf(mask)
    out[:, 7] = _ubuf(image)
    out[:, 8:11] = v
    out[:, 11] = rho
    out[:, 12] = e
    out[:, 13] = cv
    out[:, 14:17] = vest
    return out


def pack_restart_multiphase(x, tag, type_, image, v, rho, cg, rmass, e, cv, vest, mask=None):
    """AtomVecMesoMultiPhase::pack_restart (atom_vec_meso_multiphase.cpp:887-916): 21 doubles
    per atom, the ints as plain doubles (that routine assigns them directly)."""
    n = x.shape[0]
    mask = np.ones(n) if mask is None else mask
    out = np.zeros((n, 21))
    out[:, 0] = 21
    out[:, 1:4] = x
    out[:, 4] = tag
    out[:, 5] = type_
    out[:, 6] = mask
    out[:, 7] = image
    out[:, 8:11] = v
    out[:, 11] = rho
    out[:, 12:15] = cg
    out[:, 15] = rmass
    out[:, 16] = e
    out[:, 17] = cv
    out[:, 18:21] = vest
    return out


def unpack_restart(buf):
    """AtomVecMeso{,MultiPhase}::unpack_restart (atom_vec_meso.cpp:763-800,
    atom_vec_meso_multiphase.cpp:922-960) of a (n, 17 | 21) record array."""
    buf = np.asarray(buf)
    mp = buf.shape[1] == 21
    ints = (lambda c: buf[:, c].astype(np.int64)) if mp else (lambda c: buf[:, c].view(np.int64))
    d = dict(x=buf[:, 1:4], tag=ints(4), type=ints(5), mask=ints(6), image=ints(7),
             v=buf[:, 8:11], rho=buf[:, 11])
    if mp:
        d.update(cg=buf[:, 12:15], rmass=buf[:, 15], e=buf[:, 16], cv=buf[:, 17],
                 vest=buf[:, 18:21])
    else:
        d.update(e=buf[:, 12], cv=buf[:, 13], vest=buf[:, 14:17])
    return d
