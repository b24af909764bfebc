"""Debug helper: one sph/taitwater/hip compute through the linked shim on the golden c2_n6."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "oracle")); sys.path.insert(0, os.path.join(R, "tests"))
import numpy as np
import pyoracle as po
from test_oracle_golden import load
S = po.shim()
d = load(sys.argv[1] if len(sys.argv) > 1 else "c2_n6")
dim, nt, n, ng = int(d["dim"]), int(d["ntypes"]), int(d["nlocal"]), int(d["nghost"])
if "out_rho" in d:
    rho = d["rho"].copy()
    S.ref_rhosum(dim, nt, n, ng, d["x"], d["type"], d["mass"], d["rhosum_cut"], d["full_off"], d["full_nbr"], rho)
    print("rhosum err", np.abs(rho[:n] - d["out_rho"]).max(), flush=True)
f, drho, de = np.zeros((n + ng, 3)), np.zeros(n + ng), np.zeros(n + ng)
(S.ref_taitwater_morris if int(d["morris"]) else S.ref_taitwater)(dim, nt, n, ng, 1, d["x"], d["vest"], d["rho"], d["type"], d["mass"], d["rho0"], d["c0"], d["visc"], d["tait_cut"], d["half_off"], d["half_nbr"], f, drho, de)
print("tait err", np.abs(f - d["out_f"]).max() / np.abs(d["out_f"]).max(), flush=True)
if "out_de_heat" in d:
    print("heat", flush=True)
    de = np.zeros(n + ng)
    S.ref_heatconduction(dim, nt, n, ng, 1, d["x"], d["e"], d["rho"], d["type"], d["mass"], d["alpha"], d["heat_cut"], d["half_off"], d["half_nbr"], de)
    print("heat err", np.abs(de - d["out_de_heat"]).max() / np.abs(d["out_de_heat"]).max(), flush=True)
