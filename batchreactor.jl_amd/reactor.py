"""batch_reactor entry points, mirroring BatchReactor.jl's public API on the HIP engine.

  batch_reactor(input_file, lib_dir; sens, surfchem, gaschem)   src/BatchReactor.jl:67-70
  batch_reactor(input_file, lib_dir, udf; sens)                 src/BatchReactor.jl:51-54
  batch_reactor(inlet_comp, T, p, time; Asv, chem, thermo_obj, md)  src/BatchReactor.jl:86-147
  batch_reactor_ensemble(...)  -- new: N reactors, each with its own T, p, composition, Asv, tf

The file-driven path writes gas_profile.{dat,csv} and surface_covg.{dat,csv} next to the input
(src/BatchReactor.jl:168-180) and returns the CVODE retcode symbol as the string "Success".
The user-defined-chemistry path (udf) runs the user's host function, as the reference does
(src/BatchReactor.jl:358-360); it is host code outside the GPU hot path.
"""
import decimal
import os
from dataclasses import dataclass, field

import numpy as np

from .engine import Engine
from .mechanism import CONV_REFERENCE, Mechanism, read_batch_xml


@dataclass
class Chemistry:
    """ReactionCommons.Chemistry(surfchem, gaschem, userchem, udf) (src/BatchReactor.jl:52,:68)."""
    surfchem: bool = False
    gaschem: bool = False
    userchem: bool = False
    udf: object = None


@dataclass
class ConstantParams:
    """ConstantParams(Asv, T) (src/BatchReactor.jl:14-17)."""
    Asv: float
    T: float


@dataclass
class UserDefinedState:
    """ReactionCommons.UserDefinedState(T, p, mole_frac, molwt, species, source) as built at
    src/BatchReactor.jl:197-200: the udf fills `source` [mol/m3/s]; du = source .* molwt (:371-372)."""
    T: float
    p: float
    mole_frac: np.ndarray
    molwt: np.ndarray
    species: list
    source: np.ndarray


@dataclass
class ODEProblem:
    """The problem object `sens=true` returns (ODEProblem(residual!, soln, t_span, params),
    src/BatchReactor.jl:204-207): f(du, u, p, t) is residual!, evaluated on the GPU (br_rhs)."""
    f: object
    u0: np.ndarray
    tspan: tuple
    p: dict = field(default_factory=dict)


# SciML return codes of a CVODE_BDF solve (Symbol(sol.retcode), src/BatchReactor.jl:216), from the
# engine's per-reactor status (include/brhip.h): Sundials.jl's interpret_sundials_retcode maps CVODE's
# flags -1 (CV_TOO_MUCH_WORK) -> MaxIters, -2 / -3 (CV_TOO_MUCH_ACC, CV_ERR_FAILURE) -> Unstable,
# -4 (CV_CONV_FAILURE) -> ConvergenceFailure, any other failure -> Failure; SciML's unstable_check (a
# NaN state) ends the solve with Unstable (status -7). Restated from the published packages, which are
# not in the image: the mapping itself is parity-unpinned (no reference fixture fails).
RETCODES = {0: "Success", -1: "MaxIters", -2: "Unstable", -3: "Unstable", -4: "ConvergenceFailure",
            -7: "Unstable"}


def retcode(status) -> str:
    """The retcode symbol's name for an engine status code (0 -> "Success")."""
    return RETCODES.get(int(status), "Failure")


def _engine(mech: Mechanism, device=0) -> Engine:
    """One engine per (mechanism object, device), owned by the mechanism: it lives as long as the
    mechanism does (no global cache, so repeated file-driven calls do not accumulate handles)."""
    cache = mech.__dict__.setdefault("_engines", {})
    if device not in cache:
        cache[device] = Engine(mech, device)
    return cache[device]


def compile_mechanism(input_file, lib_dir, chem: Chemistry, conv=CONV_REFERENCE):
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


# ---------------------------------------------------------------------------------------------
# output files (save_data, src/BatchReactor.jl:383-402; RxnHelperUtils create_header /
# write_to_file / write_csv)
# ---------------------------------------------------------------------------------------------
def julia_string(x) -> str:
    """Julia's string(::Float64): the shortest round-trip digits (as Python's repr), printed in
    plain notation when the decimal exponent e (x = d.ddd x 10^e) satisfies -4 <= e <= 5 and as
    d.ddde<exp> otherwise, always with a fractional part: 0.0001, 1.0e-5, 100000.0, 1.0e6,
    4.3211443386069156e-16 (the format of test/batch_gas_and_surf/gas_profile.csv)."""
    x = float(x)
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Inf" if x > 0 else "-Inf"
    if x == 0.0:
        return "-0.0" if str(x).startswith("-") else "0.0"
    sign, digits, exp = decimal.Decimal(repr(x)).as_tuple()
    ds = "".join(map(str, digits)).rstrip("0") or "0"
    e10 = exp + len(digits) - 1                      # decimal exponent of the leading digit
    s = "-" if sign else ""
    if -4 <= e10 <= 5:
        if e10 >= 0:
            ip, fp = ds[:e10 + 1].ljust(e10 + 1, "0"), ds[e10 + 1:]
        else:
            ip, fp = "0", "0" * (-e10 - 1) + ds
        return f"{s}{ip}.{fp or '0'}"
    return f"{s}{ds[0]}.{ds[1:] or '0'}e{e10}"


def _fmt_dat(v):
    return "%.4e\t" % v


def _open_streams(folder, mech, surf):
    g_dat = open(os.path.join(folder, "gas_profile.dat"), "w")
    s_dat = open(os.path.join(folder, "surface_covg.dat"), "w")
    g_csv = open(os.path.join(folder, "gas_profile.csv"), "w")
    s_csv = open(os.path.join(folder, "surface_covg.csv"), "w")
    hdr = ["t", "T", "p", "rho"] + mech.gas_species
    g_dat.write("".join("%10s\t" % h for h in hdr) + "\n")
    g_csv.write(",".join(hdr) + "\n")
    if surf:
        sh = ["t", "T"] + mech.surf_species
        s_dat.write("".join("%10s\t" % h for h in sh) + "\n")
        s_csv.write(",".join(sh) + "\n")
    return g_dat, g_csv, s_dat, s_csv


def _row(streams, surf, t, T, p, rho, x, th, progress=False):
    g_dat, g_csv, s_dat, s_csv = streams
    vals = [t, T, p, rho] + list(x)
    g_dat.write("".join(_fmt_dat(v) for v in vals) + "\n")
    g_csv.write(",".join(julia_string(v) for v in vals) + "\n")
    if surf:
        sv = [t, T] + list(th)
        s_dat.write("".join(_fmt_dat(v) for v in sv) + "\n")
        s_csv.write(",".join(julia_string(v) for v in sv) + "\n")
    if progress:
        print("%4e" % t)                             # @printf("%4e\n", t) (:401)


# ---------------------------------------------------------------------------------------------
# file-driven entry point
# ---------------------------------------------------------------------------------------------
def _gpu_rhs_problem(mech, eng, T, Asv, u0, tf, chem):
    """(params, prob, t_span) of sens=true: residual! evaluated by the engine (br_rhs)."""
    def residual(du, u, p, t):
        du[:] = eng.rhs([T], [Asv], np.asarray(u, float)[None, :])[0]
    params = dict(s_state=None, g_state=None, u_state=None, thermo=mech, smd=mech if chem.surfchem else None,
                  gmd=mech if chem.gaschem else None, cp=ConstantParams(Asv, T), chem=chem)
    t_span = (0.0, tf)
    return params, ODEProblem(residual, u0, t_span, params), t_span


def _udf_run(mech, x0, T, p0, tf, chem, folder, progress, max_steps=100000):
    """userchem path (src/BatchReactor.jl:197-200,:358-360,:371-372): the user's host function fills
    state.source; du = source .* molwt. As in the reference, the state handed to the udf keeps the
    inlet T, p and mole fractions (residual! never updates u_state). The reference solves it with
    CVODE_BDF() (:204-210); a Python function cannot run in a kernel, so it is integrated on the CPU
    by br_integrate_host -- the engine's CVODE 5.x restatement with CVODE's DQ Jacobian, the same solver
    the Julia host calls -- with one save_data row per accepted step (:383-402)."""
    from . import _lib
    ng = mech.ng
    state = UserDefinedState(T, p0, np.array(x0, float), mech.molwt, list(mech.gas_species), np.zeros(ng))
    u0 = mech.initial_state(T, p0, x0)

    def f(t, u):
        chem.udf(state)
        return np.asarray(state.source[:ng], float) * mech.molwt

    streams = _open_streams(folder, mech, False)
    try:
        status, _, _ = _lib.integrate_host(
            f, u0[:ng], tf, max_steps=max_steps,
            on_step=lambda t, u: _row(streams, False, t, T, state.p, float(np.sum(u)), state.mole_frac, (), progress))
    finally:
        for s in streams:
            s.close()
    return retcode(status)


def batch_reactor(input_file, lib_dir, udf=None, *, sens=False, surfchem=False, gaschem=False, device=0,
                  conv=CONV_REFERENCE, progress=False, max_steps=100000):
    """File-driven batch reactor (src/BatchReactor.jl:51-54, :67-70, :152-217). Returns "Success"
    (Symbol(sol.retcode)) or, with sens=True, (params, prob, t_span) (:205-207)."""
    chem = Chemistry(surfchem=surfchem and udf is None, gaschem=gaschem and udf is None, userchem=udf is not None,
                     udf=udf)
    mech, x, T, p0, Asv, tf = compile_mechanism(input_file, lib_dir, chem, conv)
    folder = os.path.dirname(os.path.abspath(input_file))
    u0 = mech.initial_state(T, p0, x)
    if chem.userchem:
        if sens:
            state = UserDefinedState(T, p0, np.array(x, float), mech.molwt, list(mech.gas_species),
                                     np.zeros(mech.ng))

            def residual(du, u, p, t):
                udf(state)
                du[:mech.ng] = np.asarray(state.source[:mech.ng], float) * mech.molwt
            params = dict(s_state=None, g_state=None, u_state=state, thermo=mech, smd=None, gmd=None,
                          cp=ConstantParams(Asv, T), chem=chem)
            return params, ODEProblem(residual, u0, (0.0, tf), params), (0.0, tf)
        return _udf_run(mech, x, T, p0, tf, chem, folder, progress, max_steps)
    eng = _engine(mech, device)
    if sens:
        return _gpu_rhs_problem(mech, eng, T, Asv, u0, tf, chem)
    # one row per accepted step (save_data callback, :383-402): rho from the accepted state u,
    # x, p and coverages from the step's last RHS evaluation (the engine's trace rows carry both).
    # The trace starts at 4096 rows; a run that took more steps is repeated once with exactly its
    # step count (the integration is deterministic, so the repeat takes the same steps)
    cap = min(4096, max_steps)
    u, st, tr = eng.integrate([T], [Asv], u0[None, :], [tf], trace_cap=cap, max_steps=max_steps)
    nst = int(st["nsteps"][0])
    if nst > cap:
        u, st, tr = eng.integrate([T], [Asv], u0[None, :], [tf], trace_cap=nst, max_steps=max_steps)
        nst = int(st["nsteps"][0])
    n, ng = mech.n, mech.ng
    streams = _open_streams(folder, mech, chem.surfchem)
    try:
        for k in range(nst + 1):
            row = tr[0, k]
            uk, yk = row[4:4 + n], row[4 + n:4 + 2 * n]
            _row(streams, chem.surfchem, row[0], T, row[3], uk[:ng].sum(), mech.state_to_molefrac(yk), yk[ng:],
                 progress)
    finally:
        for s in streams:
            s.close()
    return retcode(st["status"][0])


def batch_reactor_programmatic(inlet_comp, T, p, time, *, Asv=1.0, chem: Chemistry, mech: Mechanism, device=0):
    """batch_reactor(inlet_comp, T, p, time; Asv, chem, thermo_obj, md) (src/BatchReactor.jl:86-147).
    Returns (t, Dict(species => x_end)) with t = [0, time] (save_everystep=false). Species are
    matched by name, so the Julia Dict key order of the surface case (species =
    collect(keys(inlet_comp)), :103) does not change the result. As the reference (which does not
    check sol.retcode here), a failed integration still returns: t ends at the time reached and x is
    that of the last accepted state (batch_reactor_ensemble returns the status codes)."""
    x = mech.mole_fractions(inlet_comp)
    u0 = mech.initial_state(T, p, x)
    u, st = _engine(mech, device).integrate([T], [Asv], u0[None, :], [time])
    t_end = float(time) if st["status"][0] == 0 else float(st["t_end"][0])
    xf = dict(zip(mech.gas_species, mech.state_to_molefrac(u[0])))
    if chem.surfchem and not chem.gaschem:   # species = collect(keys(inlet_comp)) (:103, :145)
        return [0.0, t_end], {k: xf[k.upper()] for k in inlet_comp}
    return [0.0, t_end], xf


def batch_reactor_ensemble(mech: Mechanism, T, p, X, time, *, Asv=1.0, theta0=None, device=0, rtol=1e-6,
                           atol=1e-10, tout=None):
    """N independent reactors in one call. X: [N, ng] inlet mole fractions. Returns
    (x_end [N, ng], theta_end [N, ns], stats dict of [N] arrays, including t_ign, and "yout"
    [N, nout, n] when output times are given)."""
    X = np.atleast_2d(np.asarray(X, float))
    N = X.shape[0]
    T = np.broadcast_to(np.asarray(T, float), (N,))
    p = np.broadcast_to(np.asarray(p, float), (N,))
    U0 = np.stack([mech.initial_state(T[i], p[i], X[i], theta0) for i in range(N)]) if N else np.zeros((0, mech.n))
    u, st = _engine(mech, device).integrate(T, np.broadcast_to(np.asarray(Asv, float), (N,)), U0,
                                            np.broadcast_to(np.asarray(time, float), (N,)), rtol, atol, tout=tout)
    return mech.state_to_molefrac(u), u[:, mech.ng:], st
