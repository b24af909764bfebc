"""Python bindings of libsph_hip.so (include/sph_hip.h) -- the MI355X USER-SPH engine.

This is host plumbing for tests and bench.py; the product is the C ABI.  There is no CPU
fallback: if libsph_hip.so is missing, or no HIP device is usable, every compute call
raises ``HipError``.

Loaded by path because the directory name is not a Python identifier::

    spec = importlib.util.spec_from_file_location("sph_amd", ".../lammps-sph-multiphase_amd/__init__.py")
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# (SPH_HIP_LIB: another build of the same library, e.g. the study build of `make STUDY=1`)
LIB_PATH = os.environ.get("SPH_HIP_LIB") or os.path.join(HERE, "libsph_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "sph_hip.h")

SPH_LIST_FULL, SPH_LIST_HALF = 0, 1
SPH_VISC_MONAGHAN, SPH_VISC_MORRIS = 0, 1
SPH_MAXTYPES = 8
_NT2 = (SPH_MAXTYPES + 1) ** 2

ERRORS = {-1: "EINVAL", -2: "ENODEV", -3: "ERUNTIME", -4: "ENOMEM", -5: "ECOMM",
          -6: "EOVERFLOW"}


class HipError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"sph_hip {ERRORS.get(code, code)}: {msg}")
        self.code = code


_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_lp = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_i, _d, _vp = C.c_int, C.c_double, C.c_void_p

_lib = None


class EngineMpConfig(C.Structure):
    """sph_engine_mp_config (include/sph_hip.h section 2): the bubble_growth stack."""
    _fields_ = [
        ("rhosum_nstep", C.c_int), ("rhosum_cut", C.c_double * _NT2),
        ("cg_nstep", C.c_int), ("cg_alpha", C.c_double * _NT2), ("cg_cut", C.c_double * _NT2),
        ("tait_on", C.c_int), ("rho0", C.c_double * (SPH_MAXTYPES + 1)),
        ("soundspeed", C.c_double * (SPH_MAXTYPES + 1)),
        ("gamma", C.c_double * (SPH_MAXTYPES + 1)),
        ("rbackground", C.c_double * (SPH_MAXTYPES + 1)),
        ("tait_visc", C.c_double * _NT2), ("tait_cut", C.c_double * _NT2),
        ("st_on", C.c_int), ("st_cut", C.c_double * _NT2),
        ("heat_on", C.c_int), ("heat_alpha", C.c_double * _NT2),
        ("heat_cut", C.c_double * _NT2), ("heat_tc", C.c_double * _NT2),
        ("heat_fixflag", C.c_int * _NT2),
    ]


class EngineConfig(C.Structure):
    _fields_ = [
        ("dim", C.c_int), ("ntypes", C.c_int),
        ("boxlo", C.c_double * 3), ("boxhi", C.c_double * 3), ("periodic", C.c_int * 3),
        ("skin", C.c_double), ("neigh_every", C.c_int), ("dt", C.c_double),
        ("ftm2v", C.c_double), ("mass", C.c_double * (SPH_MAXTYPES + 1)),
        ("stationary_mask", C.c_int),
        ("rhosum_nstep", C.c_int), ("rhosum_cut", C.c_double * _NT2),
        ("tait_on", C.c_int), ("tait_visc", C.c_int),
        ("rho0", C.c_double * (SPH_MAXTYPES + 1)),
        ("soundspeed", C.c_double * (SPH_MAXTYPES + 1)),
        ("B", C.c_double * (SPH_MAXTYPES + 1)),
        ("tait_visc_coef", C.c_double * _NT2), ("tait_cut", C.c_double * _NT2),
        ("heat_on", C.c_int), ("heat_alpha", C.c_double * _NT2), ("heat_cut", C.c_double * _NT2),
        ("gravity", C.c_double * 3), ("gravity_mask", C.c_int),
        ("procgrid", C.c_int * 3), ("rank", C.c_int), ("sort", C.c_int),
        ("kernel_path", C.c_int),
        ("mp", C.POINTER(EngineMpConfig)),
    ]


class EngineStats(C.Structure):
    _fields_ = [
        ("step", C.c_int64), ("nlocal", C.c_int), ("nghost", C.c_int),
        ("nbr_full", C.c_int64), ("nbr_builds", C.c_int), ("nbr_maxrow", C.c_int),
        ("staged", C.c_int), ("stage_max", C.c_int),
        ("ms_rhosum", C.c_double), ("ms_tait", C.c_double), ("ms_heat", C.c_double),
        ("ms_integrate", C.c_double), ("ms_comm", C.c_double), ("ms_neigh", C.c_double),
        ("n_rhosum", C.c_int64), ("n_tait", C.c_int64), ("n_heat", C.c_int64),
        ("n_neigh", C.c_int64), ("blk_nbig", C.c_int), ("inner_rows", C.c_int),
        ("inner_live", C.c_int), ("flags", C.c_int), ("inner_refresh", C.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


EXPORTS = {
    # name: (restype, argtypes)
    "sph_hip_last_error": (C.c_char_p, []),
    "sph_hip_abi_version": (_i, []),
    "sph_hip_device_count": (_i, []),
    "sph_hip_create": (_i, [_i, _i, _i, _i, C.POINTER(_vp)]),
    "sph_hip_destroy": (_i, [_vp]),
    "sph_hip_rhosum_coeff": (_i, [_vp, _dp, _dp]),
    "sph_hip_taitwater_coeff": (_i, [_vp, _i, _dp, _dp, _dp, _dp, _dp, _dp]),
    "sph_hip_heatconduction_coeff": (_i, [_vp, _dp, _dp, _dp]),
    "sph_hip_atoms": (_i, [_vp, _i, _i, _dp, _vp, _vp, _vp, _ip]),
    "sph_hip_list": (_i, [_vp, _i, _i, _vp, _vp, _vp]),
    "sph_hip_list_keyed": (_i, [_vp, _i, C.c_int64, _i, _vp, _vp, _vp]),
    "sph_hip_atoms_rho": (_i, [_vp, _dp]),
    "sph_hip_atoms_update": (_i, [_vp, _dp, _vp, _vp, _vp]),
    "sph_hip_host_arrays": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sph_hip_list_csr": (_i, [_vp, _i, _i, _lp, _ip]),
    "sph_hip_build_list": (_i, [_vp, _i, C.c_int64, _dp]),
    "sph_hip_list_numneigh": (_i, [_vp, _ip]),
    "sph_hip_rhosum": (_i, [_vp, _dp]),
    "sph_hip_taitwater": (_i, [_vp, _dp, _dp, _dp, _vp]),
    "sph_hip_heatconduction": (_i, [_vp, _dp]),
    "sph_hip_atoms_multiphase": (_i, [_vp, _dp, _vp]),
    "sph_hip_rhosum_multiphase_coeff": (_i, [_vp, _dp]),
    "sph_hip_rhosum_multiphase": (_i, [_vp, _dp]),
    "sph_hip_taitwater_multiphase_coeff": (_i, [_vp, _dp, _dp, _dp, _dp, _dp, _dp]),
    "sph_hip_taitwater_multiphase": (_i, [_vp, _dp]),
    "sph_hip_heatconduction_phasechange_coeff": (_i, [_vp, _dp, _vp, _vp, _dp]),
    "sph_hip_heatconduction_phasechange": (_i, [_vp, _dp]),
    "sph_hip_colorgradient_coeff": (_i, [_vp, _dp, _dp]),
    "sph_hip_colorgradient": (_i, [_vp, _dp]),
    "sph_hip_set_timing": (_i, [_vp, _i]),
    "sph_hip_last_kernel_ms": (_i, [_vp, _dp]),
    "sph_hip_surfacetension_coeff": (_i, [_vp, _dp]),
    "sph_hip_surfacetension": (_i, [_vp, _dp, _dp]),
    "sph_hip_phasechange": (_i, [_vp, _vp, C.POINTER(_i), _dp, _dp, _dp, _dp, _i,
                                 C.POINTER(_i), _vp, _vp]),
    "sph_hip_phasechange_finish": (_i, [_i, _dp, _dp, _dp]),
    "sph_engine_create": (_i, [_i, C.POINTER(EngineConfig), C.POINTER(_vp)]),
    "sph_engine_destroy": (_i, [_vp]),
    "sph_engine_comm_uid": (_i, [_vp]),
    "sph_engine_comm_init": (_i, [_vp, _vp, _i, _i]),
    "sph_engine_comm_loopback": (_i, [_vp, _i]),
    "sph_local_world_create": (_i, [_i, C.POINTER(_vp)]),
    "sph_local_world_destroy": (_i, [_vp]),
    "sph_engine_comm_local": (_i, [_vp, _vp, _i]),
    "sph_engine_comm_ipc": (_i, [_vp, C.c_char_p, _i, _i, _i]),
    "sph_engine_tune": (_i, [_vp, _i, _i]),
    "sph_engine_set_tags": (_i, [_vp, _ip]),
    "sph_engine_set_atoms": (_i, [_vp, _i, _dp, _dp, _ip, _dp, _vp, _vp]),
    "sph_engine_setup": (_i, [_vp]),
    "sph_engine_run": (_i, [_vp, _i]),
    "sph_engine_nlocal": (_i, [_vp]),
    "sph_engine_get_atoms": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sph_engine_neighbor_counts": (_i, [_vp, _ip]),
    "sph_engine_stats_get": (_i, [_vp, C.POINTER(EngineStats)]),
    "sph_engine_set_timing": (_i, [_vp, _i]),
    "sph_engine_sync": (_i, [_vp]),
    "sph_engine_pair_passes": (_i, [_vp, _i]),
    "sph_engine_rebuild_passes": (_i, [_vp, _i]),
    "sph_engine_set_atoms_multiphase": (_i, [_vp, _dp, _vp, _vp]),
    "sph_engine_phase_change": (_i, [_vp, _vp, _i, _i]),
    "sph_engine_atom_sort": (_i, [_vp, _i, C.c_double]),
    "sph_engine_get_atoms_multiphase": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "sph_engine_write_restart": (_i, [_vp, _vp, C.c_int64, C.POINTER(_i)]),
    "sph_engine_read_restart": (_i, [_vp, _i, _dp]),
}


def load() -> C.CDLL:
    """Load libsph_hip.so (raises if it was not built -- there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HipError(-2, f"{LIB_PATH} not built (run `make -C lammps-sph-multiphase_amd`)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _chk(rc: int):
    if rc != 0:
        raise HipError(rc, load().sph_hip_last_error().decode(errors="replace"))


def device_count() -> int:
    return load().sph_hip_device_count()


def phasechange_finish(nlocal, dmass, rmass, e):
    """sph_hip_phasechange_finish: rmass -= dmass, e renormalised (fix_phase_change.cpp:
    325-332), in place on the owned atoms."""
    _chk(load().sph_hip_phasechange_finish(int(nlocal), dmass, rmass, e))


def _ptr(a):
    return None if a is None else a.ctypes.data


class PhaseChangeParams(C.Structure):
    """sph_phasechange_params (include/sph_hip.h section 1c)."""
    _fields_ = [("Tc", C.c_double), ("Tt", C.c_double), ("Hwv", C.c_double),
                ("dr", C.c_double), ("to_mass", C.c_double), ("cutoff", C.c_double),
                ("from_type", C.c_int), ("to_type", C.c_int), ("energy_chance", C.c_int),
                ("change_chance", C.c_double), ("rate", C.c_double), ("dt", C.c_double),
                ("maxattempt", C.c_int), ("sublo", C.c_double * 3),
                ("subhi", C.c_double * 3), ("boxhi", C.c_double * 3), ("top", C.c_int * 3)]


# ------------------------------------------------------------------------------------------
# 1. Pair-style layer
# ------------------------------------------------------------------------------------------
class NeighList:
    """A LAMMPS NeighList (ilist, numneigh, firstneigh) over one CSR array, built without a
    per-row Python loop: firstneigh[i] points into `neigh` at off[i] (row i of owned atom i,
    ilist = identity).  What the shim passes to sph_hip_list[_keyed]."""

    def __init__(self, off, neigh):
        off = np.asarray(off, dtype=np.int64)
        self.neigh = np.ascontiguousarray(neigh if len(neigh) else np.zeros(1), dtype=np.int32)
        self.inum = len(off) - 1
        self.ilist = np.arange(self.inum, dtype=np.int32)
        self.numneigh = np.diff(off).astype(np.int32)
        self.ptrs = (self.neigh.ctypes.data + 4 * off[:-1]).astype(np.uint64)
        if self.inum == 0:
            self.ptrs = np.zeros(1, np.uint64)


class PairContext:
    """One sph_hip_ctx: what the LAMMPS sph/<style>/hip Pair classes drive."""

    def __init__(self, dim: int, ntypes: int, newton_pair: int = 1, device: int = 0):
        self.L = load()
        h = _vp()
        _chk(self.L.sph_hip_create(device, dim, ntypes, newton_pair, C.byref(h)))
        self.h = h
        self.ntypes = ntypes
        self.nlocal = self.nghost = 0

    def close(self):
        if self.h:
            self.L.sph_hip_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _t(a):
        return np.ascontiguousarray(a, dtype=np.float64).ravel()

    def rhosum_coeff(self, cut, mass):
        _chk(self.L.sph_hip_rhosum_coeff(self.h, self._t(cut), self._t(mass)))

    def taitwater_coeff(self, rho0, c0, B, visc, cut, mass, morris=False):
        _chk(self.L.sph_hip_taitwater_coeff(self.h, SPH_VISC_MORRIS if morris else SPH_VISC_MONAGHAN,
                                            self._t(rho0), self._t(c0), self._t(B), self._t(visc),
                                            self._t(cut), self._t(mass)))

    def heatconduction_coeff(self, alpha, cut, mass):
        _chk(self.L.sph_hip_heatconduction_coeff(self.h, self._t(alpha), self._t(cut),
                                                 self._t(mass)))

    def atoms(self, nlocal, nghost, x, type_, vest=None, rho=None, e=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        t = np.ascontiguousarray(type_, dtype=np.int32)
        vest = None if vest is None else np.ascontiguousarray(vest, dtype=np.float64)
        rho = None if rho is None else np.ascontiguousarray(rho, dtype=np.float64)
        e = None if e is None else np.ascontiguousarray(e, dtype=np.float64)
        _chk(self.L.sph_hip_atoms(self.h, nlocal, nghost, x, _ptr(vest), _ptr(rho), _ptr(e), t))
        self._keep = (x, t, vest, rho, e)
        self.nlocal, self.nghost = nlocal, nghost

    def list_csr(self, kind, off, neigh):
        off = np.ascontiguousarray(off, dtype=np.int64)
        neigh = np.ascontiguousarray(neigh if len(neigh) else np.zeros(1), dtype=np.int32)
        _chk(self.L.sph_hip_list_csr(self.h, kind, len(off) - 1, off, neigh))

    def list_lammps(self, kind, ilist, numneigh, firstneigh_rows, key=None):
        """LAMMPS NeighList form: ilist, numneigh (per atom), list of per-atom int32 rows.
        key (the list build, e.g. neighbor->ncalls): sph_hip_list_keyed, which reuses the
        staged list of this kind when the key matches."""
        ilist = np.ascontiguousarray(ilist, dtype=np.int32)
        numneigh = np.ascontiguousarray(numneigh, dtype=np.int32)
        rows = [np.ascontiguousarray(r, dtype=np.int32) for r in firstneigh_rows]
        ptrs = (C.c_void_p * max(len(rows), 1))(*[r.ctypes.data for r in rows])
        if key is None:
            _chk(self.L.sph_hip_list(self.h, kind, len(ilist), ilist.ctypes.data,
                                     numneigh.ctypes.data, C.cast(ptrs, C.c_void_p)))
        else:
            _chk(self.L.sph_hip_list_keyed(self.h, kind, int(key), len(ilist), ilist.ctypes.data,
                                           numneigh.ctypes.data, C.cast(ptrs, C.c_void_p)))

    def atoms_update(self, x, vest=None, rho=None, e=None):
        """Same atom set as the last atoms(): restage positions (and vest/rho/e)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        vest = None if vest is None else np.ascontiguousarray(vest, dtype=np.float64)
        rho = None if rho is None else np.ascontiguousarray(rho, dtype=np.float64)
        e = None if e is None else np.ascontiguousarray(e, dtype=np.float64)
        _chk(self.L.sph_hip_atoms_update(self.h, x, _ptr(vest), _ptr(rho), _ptr(e)))
        self._keep_u = (x, vest, rho, e)

    def host_arrays(self, nmax, x=None, vest=None, rho=None, e=None, f=None, drho=None,
                    de=None):
        """Register the caller's arrays as mapped host memory (sph_hip_host_arrays); they must
        stay alive (and in place) until host_arrays(0) or close()."""
        arrs = [x, vest, rho, e, f, drho, de]
        for a in arrs:
            assert a is None or (a.dtype == np.float64 and a.flags["C_CONTIGUOUS"])
        _chk(self.L.sph_hip_host_arrays(self.h, int(nmax),
                                        *[None if a is None else a.ctypes.data for a in arrs]))
        self._keep_h = arrs

    def atoms_rho(self, rho):
        """Restage rho only (sph_hip_atoms_rho)."""
        _chk(self.L.sph_hip_atoms_rho(self.h, np.ascontiguousarray(rho, dtype=np.float64)))

    def build_list(self, kind, cutneighsq, key=-1):
        """The list built on the device from the staged atoms (sph_hip_build_list):
        cutneighsq = Neighbor::cutneighsq, (ntypes+1)^2; key as list_neighlist."""
        c = np.ascontiguousarray(cutneighsq, dtype=np.float64).ravel()
        _chk(self.L.sph_hip_build_list(self.h, kind, int(key), c))

    def numneigh(self, inum):
        out = np.zeros(max(inum, 1), dtype=np.int32)
        _chk(self.L.sph_hip_list_numneigh(self.h, out))
        return out[:inum]

    def list_neighlist(self, kind, nl, key=-1):
        """Stage a NeighList (sph_hip_list_keyed; key < 0: always upload)."""
        _chk(self.L.sph_hip_list_keyed(self.h, kind, int(key), nl.inum, nl.ilist.ctypes.data,
                                       nl.numneigh.ctypes.data, nl.ptrs.ctypes.data))

    def rhosum(self, rho):
        _chk(self.L.sph_hip_rhosum(self.h, rho))
        return rho

    def taitwater(self, f, drho, de, virial=None):
        _chk(self.L.sph_hip_taitwater(self.h, f, drho, de, _ptr(virial)))

    def heatconduction(self, de):
        _chk(self.L.sph_hip_heatconduction(self.h, de))

    # -- multiphase styles (section 1b) --------------------------------------------------
    def atoms_multiphase(self, rmass, cv=None):
        rmass = np.ascontiguousarray(rmass, dtype=np.float64)
        cv = None if cv is None else np.ascontiguousarray(cv, dtype=np.float64)
        _chk(self.L.sph_hip_atoms_multiphase(self.h, rmass, _ptr(cv)))
        self._keep_mp = (rmass, cv)

    def rhosum_multiphase_coeff(self, cut):
        _chk(self.L.sph_hip_rhosum_multiphase_coeff(self.h, self._t(cut)))

    def rhosum_multiphase(self, rho):
        _chk(self.L.sph_hip_rhosum_multiphase(self.h, rho))
        return rho

    def taitwater_multiphase_coeff(self, rho0, c0, gamma, rbackground, visc, cut):
        _chk(self.L.sph_hip_taitwater_multiphase_coeff(
            self.h, self._t(rho0), self._t(c0), self._t(gamma), self._t(rbackground),
            self._t(visc), self._t(cut)))

    def taitwater_multiphase(self, f):
        _chk(self.L.sph_hip_taitwater_multiphase(self.h, f))

    def heatconduction_phasechange_coeff(self, alpha, cut, fixflag=None, tc=None):
        ff = None if fixflag is None else np.ascontiguousarray(fixflag, dtype=np.int32).ravel()
        tcv = None if tc is None else self._t(tc)
        self._keep_hpc = (ff, tcv)
        _chk(self.L.sph_hip_heatconduction_phasechange_coeff(self.h, self._t(alpha), _ptr(ff),
                                                            _ptr(tcv), self._t(cut)))

    def heatconduction_phasechange(self, de):
        _chk(self.L.sph_hip_heatconduction_phasechange(self.h, de))

    def colorgradient_coeff(self, alpha, cut):
        _chk(self.L.sph_hip_colorgradient_coeff(self.h, self._t(alpha), self._t(cut)))

    def phasechange(self, params, seed, v, cg, e, cap=None):
        """One FixPhaseChange::pre_exchange.  Returns (seed, nins, new_atoms (nins, 13),
        parent, dmass); e is updated in place."""
        nall = self.nlocal + self.nghost
        cap = nall if cap is None else cap
        sd = _i(int(seed))
        nins = _i(0)
        dmass = np.zeros(nall)
        rec = np.zeros((max(cap, 1), 13))
        par = np.zeros(max(cap, 1), dtype=np.int32)
        _chk(self.L.sph_hip_phasechange(self.h, C.byref(params), C.byref(sd),
                                        np.ascontiguousarray(v, dtype=np.float64),
                                        np.ascontiguousarray(cg, dtype=np.float64), e, dmass,
                                        cap, C.byref(nins), rec.ctypes.data, par.ctypes.data))
        n = nins.value
        return sd.value, n, rec[:min(n, cap)].copy(), par[:min(n, cap)].copy(), dmass

    def colorgradient(self, cg):
        _chk(self.L.sph_hip_colorgradient(self.h, cg))
        return cg

    def set_timing(self, on=True):
        _chk(self.L.sph_hip_set_timing(self.h, 1 if on else 0))

    def last_kernel_ms(self) -> float:
        v = np.zeros(1)
        _chk(self.L.sph_hip_last_kernel_ms(self.h, v))
        return float(v[0])

    def surfacetension_coeff(self, cut):
        _chk(self.L.sph_hip_surfacetension_coeff(self.h, self._t(cut)))

    def surfacetension(self, cg, f):
        """cg: (nall, 3) colorgradient of every atom; f (nall, 3) is accumulated."""
        _chk(self.L.sph_hip_surfacetension(self.h, np.ascontiguousarray(cg, dtype=np.float64),
                                           f))
        return f


# ------------------------------------------------------------------------------------------
# 2. Device-resident engine
# ------------------------------------------------------------------------------------------
def _pair_table(dst, tab, ntypes):
    tab = np.asarray(tab, dtype=np.float64)
    for i in range(ntypes + 1):
        for j in range(ntypes + 1):
            dst[i * (SPH_MAXTYPES + 1) + j] = float(tab[i, j])


def make_config(dim, ntypes, boxlo, boxhi, periodic, mass, skin, dt, neigh_every=10,
                rhosum=None, tait=None, heat=None, gravity=(0.0, 0.0, 0.0),
                stationary_mask=0, sort=1, procgrid=(1, 1, 1), rank=0,
                kernel_path=0, gravity_mask=0, mp=None) -> EngineConfig:
    """kernel_path: 0 = the production pair passes (block-staged LDS unions + 16-bit slot
    rows; bench.py's path), 1 = the row path (row2 gathers over strided global lists).
    rhosum = dict(nstep, cut); tait = dict(rho0, c0, visc, cut, morris[, B]);
    heat = dict(alpha, cut); per-type arrays (ntypes+1), per-pair (ntypes+1, ntypes+1)."""
    c = EngineConfig()
    c.dim, c.ntypes = dim, ntypes
    for k in range(3):
        c.boxlo[k], c.boxhi[k], c.periodic[k] = float(boxlo[k]), float(boxhi[k]), int(periodic[k])
        c.gravity[k] = float(gravity[k])
        c.procgrid[k] = int(procgrid[k])
    c.rank = rank
    c.skin, c.dt, c.neigh_every, c.ftm2v = skin, dt, neigh_every, 1.0
    for t in range(ntypes + 1):
        c.mass[t] = float(mass[t])
    c.stationary_mask = stationary_mask
    c.gravity_mask = gravity_mask
    c.sort = sort
    c.kernel_path = kernel_path
    if rhosum:
        c.rhosum_nstep = int(rhosum.get("nstep", 1))
        _pair_table(c.rhosum_cut, rhosum["cut"], ntypes)
    if tait:
        c.tait_on = 1
        c.tait_visc = SPH_VISC_MORRIS if tait.get("morris") else SPH_VISC_MONAGHAN
        rho0 = np.asarray(tait["rho0"], dtype=np.float64)
        c0 = np.asarray(tait["c0"], dtype=np.float64)
        B = np.asarray(tait["B"], dtype=np.float64) if "B" in tait else c0 * c0 * rho0 / 7.0
        for t in range(ntypes + 1):
            c.rho0[t], c.soundspeed[t], c.B[t] = float(rho0[t]), float(c0[t]), float(B[t])
        _pair_table(c.tait_visc_coef, tait["visc"], ntypes)
        _pair_table(c.tait_cut, tait["cut"], ntypes)
    if heat:
        c.heat_on = 1
        _pair_table(c.heat_alpha, heat["alpha"], ntypes)
        _pair_table(c.heat_cut, heat["cut"], ntypes)
    if mp is not None:
        m = mp_config(ntypes, **mp)
        c.mp = C.pointer(m)
        c._mp_keep = m  # (the engine copies it at create)
    return c


def mp_config(ntypes, rhosum_nstep=1, rhosum_cut=None, cg_nstep=1, cg_alpha=None, cg_cut=None,
              rho0=None, c0=None, gamma=None, rbg=None, visc=None, tait_cut=None, st_cut=None,
              heat_alpha=None, heat_cut=None, heat_fixflag=None, heat_tc=None) -> EngineMpConfig:
    """The multiphase stack: tables (ntypes+1, ntypes+1), per-type arrays (ntypes+1); a style
    is on when its cut table is given (rhosum/colorgradient also need nstep > 0)."""
    m = EngineMpConfig()
    if rhosum_cut is not None and rhosum_nstep > 0:
        m.rhosum_nstep = int(rhosum_nstep)
        _pair_table(m.rhosum_cut, rhosum_cut, ntypes)
    if cg_cut is not None and cg_nstep > 0:
        m.cg_nstep = int(cg_nstep)
        _pair_table(m.cg_cut, cg_cut, ntypes)
        _pair_table(m.cg_alpha, cg_alpha, ntypes)
    if tait_cut is not None:
        m.tait_on = 1
        for t in range(ntypes + 1):
            m.rho0[t], m.soundspeed[t] = float(rho0[t]), float(c0[t])
            m.gamma[t], m.rbackground[t] = float(gamma[t]), float(rbg[t])
        _pair_table(m.tait_visc, visc, ntypes)
        _pair_table(m.tait_cut, tait_cut, ntypes)
    if st_cut is not None:
        m.st_on = 1
        _pair_table(m.st_cut, st_cut, ntypes)
    if heat_cut is not None:
        m.heat_on = 1
        _pair_table(m.heat_alpha, heat_alpha, ntypes)
        _pair_table(m.heat_cut, heat_cut, ntypes)
        if heat_tc is not None:
            _pair_table(m.heat_tc, heat_tc, ntypes)
        if heat_fixflag is not None:
            ff = np.asarray(heat_fixflag)
            for i in range(ntypes + 1):
                for j in range(ntypes + 1):
                    m.heat_fixflag[i * (SPH_MAXTYPES + 1) + j] = int(ff[i, j])
    return m


def comm_uid() -> bytes:
    """ncclUniqueId (128 bytes) for sph_engine_comm_init; make it on rank 0, broadcast."""
    buf = C.create_string_buffer(128)
    _chk(load().sph_engine_comm_uid(buf))
    return buf.raw


class LocalWorld:
    """Several bricks in one process (sph_local_world): one host thread per brick."""

    def __init__(self, nranks: int):
        self.L = load()
        h = _vp()
        _chk(self.L.sph_local_world_create(nranks, C.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            self.L.sph_local_world_destroy(self.h)
            self.h = None


class Engine:
    def __init__(self, cfg: EngineConfig, device: int = 0):
        self.L = load()
        h = _vp()
        self.cfg = cfg
        _chk(self.L.sph_engine_create(device, C.byref(cfg), C.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            self.L.sph_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_atoms(self, x, v, type_, rho, e=None, cv=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        v = np.ascontiguousarray(v, dtype=np.float64)
        t = np.ascontiguousarray(type_, dtype=np.int32)
        rho = np.ascontiguousarray(rho, dtype=np.float64)
        e = None if e is None else np.ascontiguousarray(e, dtype=np.float64)
        cv = None if cv is None else np.ascontiguousarray(cv, dtype=np.float64)
        _chk(self.L.sph_engine_set_atoms(self.h, x.shape[0], x, v, t, rho, _ptr(e), _ptr(cv)))

    def set_atoms_multiphase(self, rmass, cv=None, cg=None):
        rmass = np.ascontiguousarray(rmass, dtype=np.float64)
        cv = None if cv is None else np.ascontiguousarray(cv, dtype=np.float64)
        cg = None if cg is None else np.ascontiguousarray(cg, dtype=np.float64)
        _chk(self.L.sph_engine_set_atoms_multiphase(self.h, rmass, _ptr(cv), _ptr(cg)))

    def phase_change(self, Tc, Tt, Hwv, dr, to_mass, cutoff, from_type, to_type, nevery=1,
                     seed=123456, prob=0.0, energy_chance=0, rate=0.0, maxattempt=10):
        """fix phase_change Tc Tt Hwv dr mass cutoff from to nevery seed prob|ENERGY rate."""
        p = PhaseChangeParams()
        p.Tc, p.Tt, p.Hwv, p.dr, p.to_mass, p.cutoff = Tc, Tt, Hwv, dr, to_mass, cutoff
        p.from_type, p.to_type = from_type, to_type
        p.energy_chance, p.change_chance, p.rate = energy_chance, prob, rate
        p.maxattempt = maxattempt
        _chk(self.L.sph_engine_phase_change(self.h, C.byref(p), nevery, seed))

    def atom_sort(self, sortfreq=1000, binsize=0.0):
        """atom_modify sort sortfreq binsize: the LAMMPS local order fix phase_change meets its
        candidates in (Atom::sort at setup and every sortfreq steps; 0 = never)."""
        _chk(self.L.sph_engine_atom_sort(self.h, int(sortfreq), float(binsize)))

    def get_atoms_multiphase(self):
        n = self.nlocal
        out = dict(rmass=np.zeros(n), cv=np.zeros(n), cg=np.zeros((n, 3)), vest=np.zeros((n, 3)),
                   type=np.zeros(n, dtype=np.int32))
        ni = C.c_int64(0)
        _chk(self.L.sph_engine_get_atoms_multiphase(
            self.h, out["rmass"].ctypes.data, out["cv"].ctypes.data, out["cg"].ctypes.data,
            out["vest"].ctypes.data, out["type"].ctypes.data, C.byref(ni)))
        out["ninserted"] = ni.value
        return out

    def write_restart(self) -> np.ndarray:
        """(nlocal, 17 | 21) restart records, AtomVecMeso{,MultiPhase}::pack_restart layout."""
        rec = _i(0)
        _chk(self.L.sph_engine_write_restart(self.h, None, 0, C.byref(rec)))
        buf = np.zeros((self.nlocal, rec.value))
        _chk(self.L.sph_engine_write_restart(self.h, buf.ctypes.data, buf.size, C.byref(rec)))
        return buf

    def read_restart(self, buf):
        buf = np.ascontiguousarray(buf, dtype=np.float64)
        _chk(self.L.sph_engine_read_restart(self.h, buf.shape[0], buf))

    def dump_custom(self, fp, step, columns, boxlo, boxhi, boundary="pp pp pp"):
        """One 'dump custom' snapshot of the owned atoms (write_dump_custom) from the engine
        state; per-atom columns by name (see write_dump_custom)."""
        g = self.get_atoms()
        try:
            g.update(self.get_atoms_multiphase())
        except Exception:
            pass
        try:
            rec = unpack_restart_records(self.write_restart())
            g["image"] = rec["image_xyz"]
        except Exception:
            pass
        write_dump_custom(fp, step, g, columns, boxlo, boxhi, boundary)

    def setup(self):
        _chk(self.L.sph_engine_setup(self.h))

    def run(self, n):
        _chk(self.L.sph_engine_run(self.h, n))

    def pair_passes(self, n):
        _chk(self.L.sph_engine_pair_passes(self.h, n))

    def rebuild_passes(self, n):
        _chk(self.L.sph_engine_rebuild_passes(self.h, n))

    def sync(self):
        _chk(self.L.sph_engine_sync(self.h))

    # timer classes of sph_engine_set_timing
    T_RHO, T_TAIT, T_HEAT, T_INT, T_COMM, T_NEIGH = range(6)

    def set_timing(self, on, classes=None):
        """on: every kernel class timed with hipEvents; classes: only these (T_* bits)."""
        if on and classes is not None:
            mask = 0
            for c in classes:
                mask |= 1 << c
            _chk(self.L.sph_engine_set_timing(self.h, mask << 1))
        else:
            _chk(self.L.sph_engine_set_timing(self.h, 1 if on else 0))

    @property
    def nlocal(self):
        return self.L.sph_engine_nlocal(self.h)

    def get_atoms(self):
        """Owned atoms: set_atoms order for a single brick, else local order; "tag" always."""
        n = self.nlocal
        out = {k: np.zeros((n, 3)) for k in ("x", "v", "f")}
        out.update({k: np.zeros(n) for k in ("rho", "e", "drho", "de")})
        out["tag"] = np.zeros(n, dtype=np.int32)
        _chk(self.L.sph_engine_get_atoms(self.h, out["x"].ctypes.data, out["v"].ctypes.data,
                                         out["rho"].ctypes.data, out["e"].ctypes.data,
                                         out["f"].ctypes.data, out["drho"].ctypes.data,
                                         out["de"].ctypes.data, out["tag"].ctypes.data))
        return out

    def set_tags(self, tags):
        tags = np.ascontiguousarray(tags, dtype=np.int32)
        _chk(self.L.sph_engine_set_tags(self.h, tags))

    def comm_local(self, world: "LocalWorld", rank: int):
        _chk(self.L.sph_engine_comm_local(self.h, world.h, rank))
        self._world = world

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = C.create_string_buffer(bytes(uid), 128)
        _chk(self.L.sph_engine_comm_init(self.h, buf, nranks, rank))

    TUNE_OVERLAP, TUNE_BLKUMF = 1, 2

    def tune(self, key: int, value: int):
        """sph_engine_tune: a schedule choice that does not change results (before setup)."""
        _chk(self.L.sph_engine_tune(self.h, key, int(value)))

    IPC_DEVICE, IPC_HOST = 0, 1

    def comm_ipc(self, name: str, nranks: int, rank: int, mode: int = 0):
        """Node-local world of processes (sph_engine_comm_ipc): `name` = "/word" chosen by
        rank 0 and shared by the launcher; mode IPC_DEVICE (hipIpc outboxes, device copies)
        or IPC_HOST (host shared-memory staging).  Collective over the ranks."""
        _chk(self.L.sph_engine_comm_ipc(self.h, name.encode(), nranks, rank, int(mode)))

    def comm_loopback(self, on: bool = True):
        """One brick, self swaps through the attached communicator (RCCL send/recv to self)."""
        _chk(self.L.sph_engine_comm_loopback(self.h, 1 if on else 0))

    def neighbor_counts(self):
        c = np.zeros(self.nlocal, dtype=np.int32)
        _chk(self.L.sph_engine_neighbor_counts(self.h, c))
        return c

    def stats(self) -> dict:
        s = EngineStats()
        _chk(self.L.sph_engine_stats_get(self.h, C.byref(s)))
        return s.as_dict()


# ------------------------------------------------------------------------------------------
# dump custom / restart records on the host
# ------------------------------------------------------------------------------------------
def unpack_restart_records(buf):
    """Fields of (n, 17 | 21) restart records (include/sph_hip.h, sph_engine_write_restart);
    image_xyz = the unpacked image counts (lmptype.h: 10 bits per dimension, 512 = zero)."""
    buf = np.asarray(buf)
    mp = buf.shape[1] == 21
    ints = (lambda c: buf[:, c].astype(np.int64)) if mp else (lambda c: buf[:, c].view(np.int64))
    img = ints(7)
    d = {"x": buf[:, 1:4], "tag": ints(4), "type": ints(5), "image": img,
         "image_xyz": np.stack([(img & 1023) - 512, ((img >> 10) & 1023) - 512,
                                ((img >> 20) & 1023) - 512], 1)}
    return d


def write_dump_custom(fp, step, atoms, columns, boxlo, boxhi, boundary="pp pp pp"):
    """LAMMPS 'dump custom' text (dump_custom.cpp: header_item :351-362, ints '%d ', floats
    '%g ' per value then a newline, write_text).  atoms: get_atoms()-style dict ("tag" 0-based
    -> id = tag + 1).  Columns: id type x y z xs ys zs xu yu zu ix iy iz vx vy vz fx fy fz, and
    the USER-SPH per-atom computes by what they return: rho (compute meso_rho/atom), e
    (meso_e/atom), t (meso_t/atom = e / cv), cv, rmass, drho, de."""
    lo, hi = np.asarray(boxlo, float), np.asarray(boxhi, float)
    prd = hi - lo
    n = atoms["x"].shape[0]
    img = atoms.get("image", np.zeros((n, 3), np.int64))
    cols = []
    for c in columns:
        if c == "id":
            cols.append((atoms["tag"] + 1, True))
        elif c == "type":
            cols.append((atoms["type"], True))
        elif c in ("x", "y", "z"):
            cols.append((atoms["x"][:, "xyz".index(c)], False))
        elif c in ("xs", "ys", "zs"):   # pack_xs: (x - boxlo) * (1/prd)
            k = "xyz".index(c[0])
            cols.append(((atoms["x"][:, k] - lo[k]) * (1.0 / prd[k]), False))
        elif c in ("xu", "yu", "zu"):
            k = "xyz".index(c[0])
            cols.append((atoms["x"][:, k] + img[:, k] * prd[k], False))
        elif c in ("ix", "iy", "iz"):
            cols.append((img[:, "xyz".index(c[1])], True))
        elif c in ("vx", "vy", "vz", "fx", "fy", "fz"):
            cols.append((atoms[c[0]][:, "xyz".index(c[1])], False))
        elif c == "t":
            cols.append((atoms["e"] / atoms["cv"], False))
        else:
            cols.append((atoms[c], False))
    close = isinstance(fp, str)
    f = open(fp, "a") if close else fp
    f.write(f"ITEM: TIMESTEP\n{int(step)}\nITEM: NUMBER OF ATOMS\n{n}\n")
    f.write(f"ITEM: BOX BOUNDS {boundary}\n")
    for k in range(3):
        f.write("%g %g\n" % (lo[k], hi[k]))
    f.write("ITEM: ATOMS " + " ".join(columns) + "\n")
    order = np.argsort(atoms["tag"], kind="stable")
    for i in order:
        f.write("".join(("%d " % int(a[i])) if is_int else ("%g " % float(a[i]))
                        for a, is_int in cols) + "\n")
    if close:
        f.close()
