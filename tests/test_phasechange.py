"""fix phase_change (FixPhaseChange::pre_exchange, fix_phase_change.cpp:167-352).

CPU: the oracle against the reference's own KAT geometry
(examples/USER/sph/multiphase_two_atoms/phase_change.lmp: 2 atoms, every probability 1)
whose outcome follows from the fix's arithmetic without the random stream, against the
Park-Miller minimal-standard sequence, and for exact mass conservation on a larger box.
GPU: sph_hip_phasechange against the oracle with the same seed -- the same candidates must
change phase in the same order (identical stream consumption), new atoms and the mass
taken from donors within 1e-10."""
import numpy as np
import pytest

import pyoracle as po
from conftest import rel_err
from scenarios import c3_system


def kat_system():
    x = np.array([[5, 5, 5], [5.6, 5, 5]], dtype=np.float64)
    t = np.array([1, 2], dtype=np.int32)
    m = np.array([10.0, 2.0])
    e = np.array([10.0, 2.0])
    cv = np.array([3.0, 1.0])
    rho = np.ones(2)
    off = np.array([0, 1, 2], dtype=np.int64)
    nb = np.array([1, 0], dtype=np.int32)
    return x, t, m, e, cv, rho, off, nb


def kat_params():
    p = po.PcParams()
    p.dim = 3
    p.Tc, p.Tt, p.Hwv, p.dr, p.to_mass, p.cutoff = 1.0, 1.0, 1.0, 1.0, 1.0, 1.0
    p.from_type, p.to_type = 1, 2
    p.energy_chance = 0
    p.change_chance = 1.0
    p.dt = 0.0
    p.maxattempt = 10
    for k, (lo, hi) in enumerate([(0, 10), (0, 10), (-10, 10)]):
        p.sublo[k], p.subhi[k], p.boxhi[k] = lo, hi, hi
        p.top[k] = 1
    return p


def kat_cg(x, t, m, rho, off, nb):
    cut = np.zeros((3, 3))
    cut[1:, 1:] = 1.0
    alpha = np.zeros((3, 3))
    alpha[1, 2] = alpha[2, 1] = 1.0
    cg = np.zeros((2, 3))
    po.lib().orc_colorgradient(3, 2, x, rho, m, t, 2, alpha, cut, cut * cut, off, nb, cg)
    return cg


def test_park_miller_minimal_standard(po):
    """RanPark is Park & Miller's minimal standard: 16807^k mod (2^31-1)."""
    s = po.C.c_int(1)
    vals = [po.lib().orc_park_uniform(po.C.byref(s)) for _ in range(3)]
    assert s.value == pow(16807, 3, 2 ** 31 - 1)
    assert vals[0] == 16807 / 2147483647.0
    s2 = po.C.c_int(123456)
    for _ in range(10000):
        po.lib().orc_park_uniform(po.C.byref(s2))
    assert s2.value == (123456 * pow(16807, 10000, 2 ** 31 - 1)) % (2 ** 31 - 1)


def test_phase_change_kat(po):
    x, t, m, e, cv, rho, off, nb = kat_system()
    cg = kat_cg(x, t, m, rho, off, nb)
    assert abs(cg[1, 0]) > 0 and abs(cg[1, 1]) < 1e-15 and abs(cg[1, 2]) < 1e-15
    v = np.zeros((2, 3))
    seed, n, rec, par, dmass = po.phasechange(kat_params(), 123456, 2, x, v, v.copy(), cg, e,
                                              m.copy(), rho, cv, t, off, nb)
    assert n == 1 and par[0] == 1                 # the vapour atom (T = 2 >= Tc) evaporates
    assert np.allclose(dmass, [1.0, 0.0])          # all of to_mass from the only donor
    rm = m.copy()
    po.lib().orc_phasechange_finish(2, dmass, rm, e)
    assert np.allclose(rm, [9.0, 2.0])
    assert np.isclose(e[0], 10.0 * 10.0 / 9.0)      # energy renormalised, :331-333
    assert np.isclose(e[1], 0.5)                    # 0.5 (e - Hwv), :317-320
    r = rec[0]
    assert np.isclose(r[9], 0.5) and r[10] == 1.0 and r[11] == 1.0 and r[12] == 1.0
    # cg of the vapour atom points along x only: create_newpos' b2 is 0/0 (the reference
    # normalises b2 under the b1abs test, :494), every one of the 10 attempts yields NaN
    # coordinates that insert_one_atom rejects, and create_newpos_simple places the atom:
    # 1 draw for the decision + 10 x 2 + 3 = 24 draws, first simple attempt accepted
    M = 2 ** 31 - 1
    assert seed == (123456 * pow(16807, 24, M)) % M
    s = po.C.c_int(123456)
    u = [po.lib().orc_park_uniform(po.C.byref(s)) for _ in range(24)]
    want = x[1] + (np.array(u[21:24]) - 0.5) * 1.0
    assert np.array_equal(r[:3], want)
    assert rm.sum() + r[10] == m.sum()              # mass conserved


def two_phase_box(nside=7, seed=99):
    """bubble_growth-like scales (bubble.lmp:107-114): dx = 0.1, h = pcutoff = 3 dx."""
    s = c3_system(nside, seed=seed)
    dx = 0.1
    s.x *= dx
    s.boxlo = s.boxlo * dx
    s.boxhi = s.boxhi * dx
    nt = 2
    h = 3 * dx
    cut = np.zeros((3, 3))
    cut[1:, 1:] = h
    cns, cmax = po.cutneighsq(nt, cut, 0.02)
    g = po.borders(s, cmax)
    foff, fnb = po.neigh_full(3, g, nt, cns)
    rng = np.random.default_rng(seed)
    liq = s.type == 1
    own = dict(rmass=np.where(liq, 1.0, 0.3) * (1 + 0.05 * rng.uniform(-1, 1, s.n)),
               rho=np.where(liq, 1.0, 0.3), cv=np.where(liq, 1.0, 0.5),
               e=np.where(liq, 1.0, 2.0) * (1 + 0.5 * rng.uniform(-1, 1, s.n)),
               v=s.v, vest=s.v + 0.01 * rng.normal(size=s.v.shape))
    d = {k: np.ascontiguousarray(g.gather(v)) for k, v in own.items()}
    alpha = np.zeros((3, 3))
    alpha[1, 2] = alpha[2, 1] = 1.0
    cg = np.zeros((g.nall, 3))
    po.lib().orc_colorgradient(3, g.nlocal, g.x, d["rho"], d["rmass"], g.type, 2, alpha, cut,
                               cut * cut, foff, fnb, cg)
    cg[g.nlocal:] = cg[g.owner]
    d.update(g=g, foff=foff, fnb=fnb, cg=cg, cut=cut)
    p = kat_params()
    p.Tc, p.Tt, p.Hwv, p.dr, p.to_mass, p.cutoff = 3.0, 3.2, 0.5, 0.5 * dx, 0.1, h
    p.change_chance = 0.3
    for k in range(3):
        p.sublo[k], p.subhi[k], p.boxhi[k] = s.boxlo[k], s.boxhi[k], s.boxhi[k]
    return d, p


def test_phase_change_mass_conservation(po):
    d, p = two_phase_box()
    g = d["g"]
    e = d["e"].copy()
    seed, n, rec, par, dmass = po.phasechange(p, 4242, g.nlocal, g.x, d["v"], d["vest"],
                                              d["cg"], e, d["rmass"], d["rho"], d["cv"], g.type,
                                              d["foff"], d["fnb"])
    assert n > 5
    dm = dmass[:g.nlocal].copy()
    np.add.at(dm, g.owner, dmass[g.nlocal:])         # reverse_comm_fix
    rm = d["rmass"][:g.nlocal].copy()
    po.lib().orc_phasechange_finish(g.nlocal, dm, rm, e)
    total0 = d["rmass"][:g.nlocal].sum()
    assert abs(rm.sum() + rec[:, 10].sum() - total0) < 1e-12 * total0
    assert (rm > 0).all()


def _pair_layer_call(sph_amd, p, seed, g, arrays, off, nb):
    """sph_hip_phasechange (the pair-style layer, atoms staged in LAMMPS order) followed by
    what fix phase_change/hip does around it: create the atoms, reverse comm of dmass along
    CommBrick's swaps, sph_hip_phasechange_finish."""
    ctx = sph_amd.PairContext(int(p.dim), 2, 1)
    ctx.atoms(g.nlocal, g.nghost, arrays["x"], arrays["type"], vest=arrays["vest"],
              rho=arrays["rho"], e=arrays["e"])
    ctx.atoms_multiphase(arrays["rmass"], arrays["cv"])
    ctx.list_csr(sph_amd.SPH_LIST_FULL, off, nb)
    hp = sph_amd.PhaseChangeParams()
    for name, _ in sph_amd.PhaseChangeParams._fields_:
        val = getattr(p, name)
        if hasattr(val, "__len__"):
            for k in range(3):
                getattr(hp, name)[k] = val[k]
        else:
            setattr(hp, name, val)
    e = arrays["e"].copy()
    sd, nins, rec, par, dm = ctx.phasechange(hp, seed, arrays["v"], arrays["cg"], e)
    po.lib().orc_reverse_swaps(g.nlocal, len(g.swap_first) - 1, g.swap_first,
                               g.src if g.src.size else np.zeros(1, np.int32), dm)
    rm = arrays["rmass"][:g.nlocal].copy()
    sph_amd.phasechange_finish(g.nlocal, dm, rm, e)
    return sd, nins, rec, par, rm, e[:g.nlocal]


@pytest.mark.gpu
@pytest.mark.parametrize("energy", [0, 1])
def test_gpu_phase_change_vs_oracle(gpu, sph_amd, energy):
    """Against the restatement with the reference's memory behaviour (created atoms over the
    ghost slots later candidates read; orc_pre_exchange_ref, pinned to the reference by
    test_phasechange_golden.py): the same stream, insertions and donors' mass."""
    d, p = two_phase_box()
    g = d["g"]
    if energy:
        p.energy_chance = 1
        p.rate = 4.0
        p.dt = 0.5
    arrays = dict(x=g.x, v=d["v"], vest=d["vest"], cg=d["cg"], e=d["e"], rmass=d["rmass"],
                  rho=d["rho"], cv=d["cv"], type=g.type)
    so, no, out = po.pre_exchange_ref(p, 4242, g, arrays, d["foff"], d["fnb"])
    assert no > g.nlocal
    sg, ng, rg, pg, rm, e = _pair_layer_call(sph_amd, p, 4242, g, arrays, d["foff"], d["fnb"])
    n = g.nlocal
    assert (sg, ng) == (so, no - n)                   # same stream consumption
    assert np.array_equal(rg[:, :3], out["x"][n:])    # host-side positions: bit-identical
    for c, k in ((3, "v"), (6, "vest")):
        assert rel_err(rg[:, c:c + 3], out[k][n:]) < 1e-10, k
    assert rel_err(rg[:, 9], out["e"][n:]) < 1e-12
    assert rel_err(rm, out["rmass"][:n]) < 1e-12
    assert rel_err(e, out["e"][:n]) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["kat", "slab", "bubble", "slab2d"])
def test_gpu_phase_change_vs_reference_fixture(gpu, sph_amd, name):
    """The pair-style layer on the inputs of the reference's own FixPhaseChange calls
    (tests/golden/pc_*.npz, first call): the same insertions at bit-identical positions,
    the new atoms' fields and the donors' rmass and energies as the reference left them --
    including the slab case, where created atoms overwrite ghost donors (sph_pc.h)."""
    import os
    from test_phasechange_golden import call_inputs, load
    d = load(name)
    p = po.pc_params_from_args(d["args"], int(d["dim"]), d["boxlo"], d["boxhi"], float(d["dt"]))
    g, arrays, off, nb = call_inputs(d, 0)
    sg, ng, rg, pg, rm, e = _pair_layer_call(sph_amd, p, int(d["args"][12]), g, arrays, off, nb)
    n = g.nlocal
    assert ng == int(d["c0_out_nlocal"]) - n
    assert np.array_equal(rg[:, :3], d["c0_out_x"][n:])
    for c, k in ((3, "v"), (6, "vest")):
        assert rel_err(rg[:, c:c + 3], d["c0_out_" + k][n:]) < 1e-10, k
    assert rel_err(rg[:, 9], d["c0_out_e"][n:]) < 1e-12
    assert np.array_equal(rg[:, 10], d["c0_out_rmass"][n:])
    assert rel_err(rm, d["c0_out_rmass"][:n]) < 1e-12
    assert rel_err(e, d["c0_out_e"][:n]) < 1e-12


@pytest.mark.gpu
def test_gpu_phase_change_dmass_deterministic(gpu, sph_amd):
    """The donors' dmass is summed per donor in candidate order (the reference's order,
    fix_phase_change.cpp:289-299) after a sort of the donations, not with fp64 atomics: two
    calls on the same staged atoms and list give bit-identical rmass and e."""
    d, p = two_phase_box()
    g = d["g"]
    arrays = dict(x=g.x, v=d["v"], vest=d["vest"], cg=d["cg"], e=d["e"], rmass=d["rmass"],
                  rho=d["rho"], cv=d["cv"], type=g.type)
    a = _pair_layer_call(sph_amd, p, 4242, g, arrays, d["foff"], d["fnb"])
    b = _pair_layer_call(sph_amd, p, 4242, g, arrays, d["foff"], d["fnb"])
    assert a[1] > 0
    assert np.array_equal(a[4], b[4]) and np.array_equal(a[5], b[5])
