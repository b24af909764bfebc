"""fix phase_change pinned to the reference's own FixPhaseChange (tests/golden/pc_*.npz,
written by tests/golden/make_phase_change.py from oracle/_ref: fix_phase_change.cpp,
random_park.cpp and region_block.cpp compiled from the reference sources).

The oracle's orc_pre_exchange_ref restates pre_exchange (fix_phase_change.cpp:167-352) with
the reference's memory behaviour -- created atoms written over the ghost slots that later
candidates' lists still name, their drho (= dmass) zeroed, reverse comm along CommBrick's
swaps -- and must reproduce every fixture call bit for bit, including the RanPark stream
carried from one call to the next.  The slab fixture is one where that aliasing changes the
outcome (donations to overwritten ghost slots are lost; the reference does not conserve mass
there), which the test asserts so the fixture keeps covering it."""
import glob
import os

import numpy as np
import pytest

import pyoracle as po

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["kat", "slab", "bubble", "slab2d"]


def load(name):
    return dict(np.load(os.path.join(GOLD, f"pc_{name}.npz")))


def call_inputs(d, c):
    p = f"c{c}_"
    n, ng = int(d[p + "nlocal"]), int(d[p + "nghost"])
    g = po.Ghosted(n, ng, d[p + "in_x"], d[p + "in_type"], d[p + "owner"], None,
                   d[p + "src"].astype(np.int32), d[p + "swap_first"].astype(np.int32))
    arrays = {k: d[p + "in_" + k] for k in ("x", "v", "vest", "cg", "e", "rmass", "rho", "cv",
                                           "type")}
    return g, arrays, d[p + "full_off"], d[p + "full_nbr"].astype(np.int32)


def test_fixtures_present():
    have = {os.path.basename(f)[3:-4] for f in glob.glob(os.path.join(GOLD, "pc_*.npz"))}
    assert set(CASES) <= have


@pytest.mark.parametrize("name", CASES)
def test_oracle_pre_exchange_bit_exact(po, name):
    d = load(name)
    p = po.pc_params_from_args(d["args"], int(d["dim"]), d["boxlo"], d["boxhi"], float(d["dt"]))
    seed = int(d["args"][12])
    for c in range(int(d["ncalls"])):
        g, arrays, off, nb = call_inputs(d, c)
        seed, n, out = po.pre_exchange_ref(p, seed, g, arrays, off, nb)
        pre = f"c{c}_out_"
        assert n == int(d[f"c{c}_out_nlocal"])
        for k, v in out.items():
            assert np.array_equal(v, d[pre + k]), (name, c, k)


def test_kat_outcome(po):
    """phase_change.lmp: the vapour atom evaporates, taking all of to_mass from the liquid
    atom; e renormalised (:325-332), new atom e = (e - Hwv)/2 (:316-318)."""
    d = load("kat")
    assert int(d["c0_out_nlocal"]) == 3
    assert np.array_equal(d["c0_out_rmass"], [9.0, 2.0, 1.0])
    assert d["c0_out_e"][0] == 10.0 * 10.0 / 9.0 and d["c0_out_e"][1] == 0.5
    assert d["c0_out_type"][2] == 2


def test_slab_pins_the_aliasing(po):
    """On the slab fixture the reference's created atoms overwrite ghost slots that hold
    donors of the same call: the donations recorded there are zeroed (create_atom,
    atom_vec_meso_multiphase.cpp:994) and never reach their owners, so the owned mass plus
    the created mass exceeds the mass before the call.  The port-semantics restatement
    (orc_phasechange: every candidate on the atoms as found) conserves it exactly."""
    d = load("slab")
    g, arrays, off, nb = call_inputs(d, 0)
    n0 = g.nlocal
    before = arrays["rmass"][:n0].sum()
    after = d["c0_out_rmass"].sum()
    assert after - before > 1e-3
    p = po.pc_params_from_args(d["args"], 3, d["boxlo"], d["boxhi"], float(d["dt"]))
    e = arrays["e"].copy()
    _, nins, rec, _, dm = po.phasechange(p, 123456, n0, arrays["x"], arrays["v"], arrays["vest"],
                                         arrays["cg"], e, arrays["rmass"], arrays["rho"],
                                         arrays["cv"], arrays["type"], off, nb)
    assert nins == int(d["c0_out_nlocal"]) - n0
    po.lib().orc_reverse_swaps(n0, len(g.swap_first) - 1, g.swap_first, g.src, dm)
    rm = arrays["rmass"][:n0].copy()
    po.lib().orc_phasechange_finish(n0, dm, rm, e)
    assert abs(rm.sum() + rec[:, 10].sum() - before) < 1e-12 * before


@pytest.mark.parametrize("name", ["bubble", "slab2d"])
def test_port_semantics_equal_reference_without_aliasing(po, name):
    """Where no created atom lands on a slot a later candidate reads, the two restatements
    agree: same insertions, same stream, same donors' mass (to rounding)."""
    d = load(name)
    p = po.pc_params_from_args(d["args"], int(d["dim"]), d["boxlo"], d["boxhi"], float(d["dt"]))
    g, arrays, off, nb = call_inputs(d, 0)
    n0 = g.nlocal
    e = arrays["e"].copy()
    _, nins, rec, par, dm = po.phasechange(p, int(d["args"][12]), n0, arrays["x"], arrays["v"],
                                           arrays["vest"], arrays["cg"], e, arrays["rmass"],
                                           arrays["rho"], arrays["cv"], arrays["type"], off, nb)
    assert nins == int(d["c0_out_nlocal"]) - n0
    po.lib().orc_reverse_swaps(n0, len(g.swap_first) - 1, g.swap_first, g.src, dm)
    rm = arrays["rmass"][:n0].copy()
    po.lib().orc_phasechange_finish(n0, dm, rm, e)
    assert np.array_equal(rec[:, :3], d["c0_out_x"][n0:])
    assert np.abs(rm - d["c0_out_rmass"][:n0]).max() < 1e-14
    assert np.abs(e[:n0] - d["c0_out_e"][:n0]).max() < 1e-13 * np.abs(e).max()
