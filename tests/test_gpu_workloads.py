"""The pair-layer workloads of bench.py (c2pair, c5pair) and the layer's kernel timing
(sph_hip_set_timing / sph_hip_last_kernel_ms) on small blocks: they run, time something,
and report consistent JSON.  Parity of the styles themselves is test_gpu_pair.py /
test_gpu_multiphase.py."""
import argparse
import contextlib
import importlib.util
import io
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("workload", ["c2pair", "c5pair"])
def test_pair_layer_workload(gpu, sph_amd, workload):
    bench = load_bench()
    args = argparse.Namespace(edge=14, steps=2, warmup=1, no_cpu=True)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        (bench.c2_pair_main if workload == "c2pair" else bench.c5_pair_main)(args, sph_amd)
    out = json.loads(buf.getvalue().strip().splitlines()[-1])
    assert out["value"] > 0 and out["ms_per_step"] > 0
    for k, v in out["kernels"].items():
        assert v["ms_per_call"] > 0, k
    assert 0 < out["roofline"]["frac"] < 1


def test_kernel_timing_api(gpu, sph_amd):
    x = np.array([[0.0, 0, 0], [0.5, 0, 0], [0, 0.5, 0]])
    t = np.ones(3, dtype=np.int32)
    ctx = sph_amd.PairContext(3, 1, 1)
    ctx.atoms(3, 0, x, t, vest=np.zeros((3, 3)), rho=np.ones(3), e=np.zeros(3))
    cut = np.array([[0.0, 0.0], [0.0, 1.0]])
    ctx.rhosum_coeff(cut, np.array([0.0, 1.0]))
    ctx.list_csr(sph_amd.SPH_LIST_FULL, np.array([0, 2, 4, 6]), np.array([1, 2, 0, 2, 0, 1]))
    ctx.rhosum(np.zeros(3))
    assert ctx.last_kernel_ms() == 0.0          # timing off
    ctx.set_timing(True)
    ctx.rhosum(np.zeros(3))
    assert ctx.last_kernel_ms() > 0.0
    ctx.close()
