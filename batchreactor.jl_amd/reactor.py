"""batch_reactor entry points, mirroring BatchReactor.jl's public API on the HIP engine.

  batch_reactor(input_file, lib_dir; sens, surfchem, gaschem)   src/BatchReactor.jl:67-70
  batch_reactor(input_file, lib_dir, udf; sens)                 src/BatchReactor.jl:51-54
  batch_reactor(inlet_comp, T, p, time; Asv, chem, thermo_obj, md)  src/BatchReactor.jl:86-147
  batch_reactor_ensemble(...)  -- new: N reactors, each with its own T, p, composition, Asv, tf

The file-driven path writes gas_profile.{dat,csv} and surface_covg.{dat,csv} next to the input
(src/BatchReactor.jl:168-180) and returns the CVODE retcode symbol as the string "Success".
"""
import os
from dataclasses import dataclass

import numpy as np

from .engine import Engine
from .mechanism import Mechanism, read_batch_xml, R_GAS


@dataclass
class Chemistry:
    """ReactionCommons.Chemistry(surfchem, gaschem, userchem, udf) (src/BatchReactor.jl:52,:68)."""
    surfchem: bool = False
    gaschem: bool = False
    userchem: bool = False
    udf: object = None


_ENGINES = {}


def _engine(mech: Mechanism, device=0) -> Engine:
    key = (id(mech), device)
    if key not in _ENGINES:
        _ENGINES[key] = Engine(mech, device)
    return _ENGINES[key]


def compile_mechanism(input_file, lib_dir, chem: Chemistry, conv=0):
    """input_data (src/BatchReactor.jl:238-306): mechanism + inlet state from batch.xml."""
    d = read_batch_xml(input_file)
    gas_mech = d.get("gas_mech") if chem.gaschem else None
    surf_mech = d.get("surface_mech") if chem.surfchem else None
    mech = Mechanism.from_files(lib_dir, gas_mech=gas_mech, surface_mech=surf_mech,
                                gasphase=None if gas_mech else d.get("gasphase"), conv=conv)
    if "molefractions" in d:
        x = mech.mole_fractions(d["molefractions"])
    else:  # <massfractions>
        y = np.zeros(mech.ng)
        for k, v in d["massfractions"].items():
            y[mech.gas_species.index(k.upper())] = v
        t = y / mech.molwt
        x = t / t.sum()
    # RxnHelperUtils.get_value_from_xml on a missing <Asv> behaves as Asv = 1
    return mech, x, d["T"], d["p"], d.get("Asv", 1.0), d["time"]


def _fmt_dat(v):
    return "%.4e\t" % v


def _write_headers(folder, mech, surf):
    g_dat = open(os.path.join(folder, "gas_profile.dat"), "w")
    g_csv = open(os.path.join(folder, "gas_profile.csv"), "w")
    s_dat = open(os.path.join(folder, "surface_covg.dat"), "w")
    s_csv = open(os.path.join(folder, "surface_covg.csv"), "w")
    hdr = ["t", "T", "p", "rho"] + mech.gas_species
    g_dat.write("".join("%10s\t" % h for h in hdr) + "\n")
    g_csv.write(",".join(hdr) + "\n")
    if surf:
        sh = ["t", "T"] + mech.surf_species
        s_dat.write("".join("%10s\t" % h for h in sh) + "\n")
        s_csv.write(",".join(sh) + "\n")
    return g_dat, g_csv, s_dat, s_csv


def _row(streams, mech, surf, t, T, p, rho, x, th):
    g_dat, g_csv, s_dat, s_csv = streams
    vals = [t, T, p, rho] + list(x)
    g_dat.write("".join(_fmt_dat(v) for v in vals) + "\n")
    g_csv.write(",".join(repr(float(v)) for v in vals) + "\n")
    if surf:
        sv = [t, T] + list(th)
        s_dat.write("".join(_fmt_dat(v) for v in sv) + "\n")
        s_csv.write(",".join(repr(float(v)) for v in sv) + "\n")


def batch_reactor(input_file, lib_dir, udf=None, *, sens=False, surfchem=False, gaschem=False, device=0,
                  conv=0):
    """File-driven batch reactor (src/BatchReactor.jl:51-54, :67-70, :152-217)."""
    if udf is not None:
        raise NotImplementedError("user-defined chemistry (udf) is host-only in the reference and is not "
                                  "part of the GPU hot path; see DESIGN.md")
    chem = Chemistry(surfchem=surfchem, gaschem=gaschem)
    mech, x, T, p0, Asv, tf = compile_mechanism(input_file, lib_dir, chem, conv)
    u0 = mech.initial_state(T, p0, x)
    if sens:
        return (dict(mech=mech, T=T, Asv=Asv, chem=chem), u0, (0.0, tf))
    eng = _engine(mech, device)
    # one row per accepted step (save_data callback, :383-402): rho from the accepted state u,
    # x, p and coverages from the step's last RHS evaluation (the engine's trace rows carry both)
    cap = 4096
    while True:
        u, st, tr = eng.integrate([T], [Asv], u0[None, :], [tf], trace_cap=cap)
        nst = int(st["nsteps"][0])
        if nst < cap:
            break
        cap = 2 * nst
    n, ng = mech.n, mech.ng
    folder = os.path.dirname(os.path.abspath(input_file))
    streams = _write_headers(folder, mech, surfchem)
    try:
        for k in range(nst + 1):
            row = tr[0, k]
            uk, yk = row[4:4 + n], row[4 + n:4 + 2 * n]
            _row(streams, mech, surfchem, row[0], T, row[3], uk[:ng].sum(), mech.state_to_molefrac(yk), yk[ng:])
    finally:
        for s in streams:
            s.close()
    return "Success" if st["status"][0] == 0 else "Failure"


def batch_reactor_programmatic(inlet_comp, T, p, time, *, Asv=1.0, chem: Chemistry, mech: Mechanism, device=0):
    """batch_reactor(inlet_comp, T, p, time; Asv, chem, thermo_obj, md) (src/BatchReactor.jl:86-147).
    Returns (t, Dict(species => x_end)) with t = [0, time] (save_everystep=false)."""
    x = mech.mole_fractions(inlet_comp)
    u0 = mech.initial_state(T, p, x)
    u, st = _engine(mech, device).integrate([T], [Asv], u0[None, :], [time])
    if st["status"][0] != 0:
        raise RuntimeError(f"integration failed with status {st['status'][0]}")
    xf = mech.state_to_molefrac(u[0])
    return [0.0, float(time)], dict(zip(mech.gas_species, xf))


def batch_reactor_ensemble(mech: Mechanism, T, p, X, time, *, Asv=1.0, theta0=None, device=0, rtol=1e-6,
                           atol=1e-10):
    """N independent reactors in one call. X: [N, ng] inlet mole fractions. Returns
    (x_end [N, ng], theta_end [N, ns], stats dict of [N] arrays)."""
    X = np.atleast_2d(np.asarray(X, float))
    N = X.shape[0]
    T = np.broadcast_to(np.asarray(T, float), (N,))
    p = np.broadcast_to(np.asarray(p, float), (N,))
    U0 = np.stack([mech.initial_state(T[i], p[i], X[i], theta0) for i in range(N)])
    u, st = _engine(mech, device).integrate(T, np.broadcast_to(np.asarray(Asv, float), (N,)), U0,
                                            np.broadcast_to(np.asarray(time, float), (N,)), rtol, atol)
    return mech.state_to_molefrac(u), u[:, mech.ng:], st
