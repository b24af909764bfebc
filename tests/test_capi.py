"""CPU checks of the C ABI: libsph_hip.so loads, exports exactly what include/sph_hip.h
declares, and fails loudly (no CPU fallback) when no HIP device is usable."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "sph_hip.h")
LIB = os.path.join(ROOT, "lammps-sph-multiphase_amd", "libsph_hip.so")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sph_(?:hip|engine|local_world)_\w+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib_built():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.dirname(LIB)], check=True)
    return LIB


def test_header_declares_api():
    names = declared_functions()
    for must in ("sph_hip_create", "sph_hip_rhosum", "sph_hip_taitwater",
                 "sph_hip_heatconduction", "sph_engine_create", "sph_engine_run"):
        assert must in names


def test_library_exports_every_declared_symbol(lib_built):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_built], capture_output=True,
                         text=True, check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if " T " in l)
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, f"declared but not exported: {missing}"
    lib = ctypes.CDLL(lib_built)
    for n in declared_functions():
        assert getattr(lib, n) is not None


def test_bindings_cover_header(sph_amd):
    assert set(declared_functions()) == set(sph_amd.EXPORTS)


def test_abi_version(sph_amd):
    assert sph_amd.load().sph_hip_abi_version() == 2


def test_no_silent_cpu_fallback(sph_amd):
    """Without a device every compute entry point fails with ENODEV (GPU box: skipped)."""
    if sph_amd.device_count() > 0:
        pytest.skip("a HIP device is present")
    with pytest.raises(sph_amd.HipError) as ei:
        sph_amd.PairContext(3, 1, 1)
    assert ei.value.code == -2
    cfg = sph_amd.make_config(3, 1, [0, 0, 0], [10, 10, 10], [1, 1, 1], [0, 1], 0.3, 1e-3,
                              rhosum=dict(nstep=1, cut=np.array([[0, 0], [0, 3.0]])))
    with pytest.raises(sph_amd.HipError) as ei:
        sph_amd.Engine(cfg)
    assert ei.value.code == -2


def test_config_struct_layout_matches_header(sph_amd):
    """EngineConfig mirrors sph_engine_config field-for-field (checked by compiling a
    probe against the header)."""
    probe = r"""
#include <stdio.h>
#include <stddef.h>
#include "sph_hip.h"
int main(void){
  printf("%zu %zu %zu %zu %zu\n", sizeof(sph_engine_config), offsetof(sph_engine_config, tait_on),
         offsetof(sph_engine_config, heat_cut), offsetof(sph_engine_config, sort),
         sizeof(sph_engine_stats));
  return 0;
}
"""
    import tempfile
    d = tempfile.mkdtemp()
    src = os.path.join(d, "probe.c")
    exe = os.path.join(d, "probe")
    open(src, "w").write(probe)
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), src, "-o", exe], check=True)
    vals = list(map(int, subprocess.run([exe], capture_output=True, text=True).stdout.split()))
    C = sph_amd.EngineConfig
    assert vals == [ctypes.sizeof(C), C.tait_on.offset, C.heat_cut.offset, C.sort.offset,
                    ctypes.sizeof(sph_amd.EngineStats)]


def test_neighlist_row_pointers(sph_amd):
    """NeighList (what the shim hands to sph_hip_list_keyed): firstneigh[i] points at row i
    of the CSR array, numneigh = row lengths, ilist = identity -- no per-row Python arrays."""
    off = np.array([0, 3, 3, 7, 8], dtype=np.int64)
    nb = np.arange(8, dtype=np.int32) + 100
    nl = sph_amd.NeighList(off, nb)
    assert nl.inum == 4
    assert list(nl.numneigh) == [3, 0, 4, 1]
    assert list(nl.ilist) == [0, 1, 2, 3]
    for i in range(4):
        row = np.ctypeslib.as_array(ctypes.cast(int(nl.ptrs[i]), ctypes.POINTER(ctypes.c_int32)),
                                    shape=(int(nl.numneigh[i]) or 1,))
        assert list(row[:nl.numneigh[i]]) == list(nb[off[i]:off[i + 1]])
    empty = sph_amd.NeighList(np.zeros(1, np.int64), np.zeros(0, np.int32))
    assert empty.inum == 0 and len(empty.ptrs) == 1
