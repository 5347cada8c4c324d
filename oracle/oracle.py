"""ctypes wrapper of the CPU oracle (oracle/liboracle.so). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module;
the product package (batchreactor.jl_amd/) never does. See oracle.h for the reference
file:line each function restates.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

CONV_KC_UNIT_SLIP = 1
CONV_FALLOFF_XM = 2
CONV_DOC_COVG = 4
CONV_TROE_C4 = 16
CONV_REFERENCE = CONV_KC_UNIT_SLIP | CONV_FALLOFF_XM | CONV_TROE_C4   # GasphaseReactions (golden)


class Opts(C.Structure):
    _fields_ = [("rtol", C.c_double), ("atol", C.c_double), ("analytic_jac", C.c_int),
                ("max_steps", C.c_int), ("hmax", C.c_double), ("unstable_factor", C.c_double),
                ("ignition_species", C.c_int)]


class Stats(C.Structure):
    _fields_ = [("nsteps", C.c_long), ("nfe", C.c_long), ("nje", C.c_long), ("nsetups", C.c_long),
                ("nni", C.c_long), ("ncfn", C.c_long), ("netf", C.c_long), ("nfeDQ", C.c_long),
                ("status", C.c_int), ("qlast", C.c_int), ("hlast", C.c_double), ("tcur", C.c_double),
                ("t_ign", C.c_double), ("ign_rate", C.c_double), ("ign_dt", C.c_double)]

    def asdict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


STEP_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_double, C.POINTER(C.c_double), C.c_double,
                      C.POINTER(C.c_double), C.POINTER(C.c_double))


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        dp = C.POINTER(C.c_double)
        L.orc_load.restype = C.c_void_p
        L.orc_load.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int, C.c_double]
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_errmsg.restype = C.c_char_p
        for f in ("orc_ng", "orc_ns", "orc_nrg", "orc_nrs"):
            getattr(L, f).argtypes = [C.c_void_p]
            getattr(L, f).restype = C.c_int
        L.orc_species_name.argtypes = [C.c_void_p, C.c_int]
        L.orc_species_name.restype = C.c_char_p
        L.orc_molwt.argtypes = [C.c_void_p, C.c_int]
        L.orc_molwt.restype = C.c_double
        L.orc_site_density.argtypes = [C.c_void_p]
        L.orc_site_density.restype = C.c_double
        L.orc_initial_coverage.argtypes = [C.c_void_p, dp]
        L.orc_set_conv.argtypes = [C.c_void_p, C.c_int]
        L.orc_set_rxn_mult.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double]
        L.orc_initial_state.argtypes = [C.c_void_p, C.c_double, C.c_double, dp, dp]
        L.orc_rates.argtypes = [C.c_void_p, C.c_double, C.c_double, dp, dp, dp, dp]
        L.orc_rop.argtypes = [C.c_void_p, C.c_double, C.c_double, dp, dp, dp, dp]
        L.orc_rhs.argtypes = [C.c_void_p, C.c_double, C.c_double, dp, dp, dp, dp]
        L.orc_jac.argtypes = [C.c_void_p, C.c_double, C.c_double, dp, dp]
        L.orc_integrate.argtypes = [C.c_void_p, C.c_double, C.c_double, dp, C.c_double,
                                    C.POINTER(Opts), C.POINTER(Stats), STEP_CB, C.c_void_p]
        L.orc_integrate.restype = C.c_int
        L.orc_integrate_out.argtypes = [C.c_void_p, C.c_double, C.c_double, dp, C.c_double, C.POINTER(Opts),
                                        C.POINTER(Stats), C.c_int, dp, dp]
        L.orc_integrate_out.restype = C.c_int
        L.orc_integrate_batch.argtypes = [C.c_void_p, C.c_int, dp, dp, dp, dp, C.POINTER(Opts),
                                          C.POINTER(Stats), C.c_int]
        L.orc_integrate_batch.restype = C.c_int
        L.orc_integrate_batch_out.argtypes = [C.c_void_p, C.c_int, dp, dp, dp, dp, C.POINTER(Opts),
                                              C.POINTER(Stats), C.c_int, C.c_int, dp, dp]
        L.orc_integrate_batch_out.restype = C.c_int
        L.orc_set_rop_jitter.argtypes = [C.c_double]
        L.orc_set_rop_jitter.restype = None
        L.orc_set_rop_jitter_seed.argtypes = [C.c_ulonglong]
        L.orc_set_rop_jitter_seed.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _enc(s):
    return None if s is None else s.encode()


class Mech:
    """One compiled mechanism (gas and/or surface) for the oracle."""

    def __init__(self, gas_mech=None, therm=None, surf_mech=None, gas_species=None, conv=CONV_REFERENCE,
                 p_std=1e5):
        L = lib()
        gs = " ".join(gas_species) if gas_species else None
        self.h = L.orc_load(_enc(gas_mech), _enc(therm), _enc(surf_mech), _enc(gs), conv, p_std)
        if not self.h:
            raise RuntimeError("oracle load failed: " + L.orc_errmsg().decode())
        self.ng, self.ns = L.orc_ng(self.h), L.orc_ns(self.h)
        self.nrg, self.nrs = L.orc_nrg(self.h), L.orc_nrs(self.h)
        self.n = self.ng + self.ns
        self.names = [L.orc_species_name(self.h, k).decode() for k in range(self.n)]
        self.M = np.array([L.orc_molwt(self.h, k) for k in range(self.ng)])
        self.site_density = L.orc_site_density(self.h)
        self.theta0 = np.zeros(self.ns)
        self.ign1 = self.names.index("OH") + 1 if "OH" in self.names[:self.ng] else 0   # ignition marker
        if self.ns:
            L.orc_initial_coverage(self.h, _p(self.theta0))

    def __del__(self):
        try:
            lib().orc_free(self.h)
        except Exception:
            pass

    def set_conv(self, conv):
        lib().orc_set_conv(self.h, conv)

    def set_rxn_mult(self, i, fmul, rmul):
        lib().orc_set_rxn_mult(self.h, i, fmul, rmul)

    def initial_state(self, T, p, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        u = np.zeros(self.n)
        lib().orc_initial_state(self.h, T, p, _p(x), _p(u))
        return u

    def rates(self, T, p, x, theta=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        th = np.ascontiguousarray(theta if theta is not None else np.zeros(max(self.ns, 1)), dtype=np.float64)
        w = np.zeros(max(self.ng, 1))
        s = np.zeros(max(self.n, 1))
        lib().orc_rates(self.h, T, p, _p(x), _p(th), _p(w), _p(s))
        return w[:self.ng], s[:self.n]

    def rop(self, T, p, x, theta=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        th = np.ascontiguousarray(theta if theta is not None else np.zeros(max(self.ns, 1)), dtype=np.float64)
        qg = np.zeros(max(self.nrg, 1))
        qs = np.zeros(max(self.nrs, 1))
        lib().orc_rop(self.h, T, p, _p(x), _p(th), _p(qg), _p(qs))
        return qg[:self.nrg], qs[:self.nrs]

    def rhs(self, T, Asv, u):
        u = np.ascontiguousarray(u, dtype=np.float64)
        du = np.zeros(self.n)
        p = np.zeros(1)
        x = np.zeros(max(self.ng, 1))
        lib().orc_rhs(self.h, T, Asv, _p(u), _p(du), _p(p), _p(x))
        return du, p[0], x[:self.ng]

    def jac(self, T, Asv, u):
        u = np.ascontiguousarray(u, dtype=np.float64)
        J = np.zeros((self.n, self.n))
        lib().orc_jac(self.h, T, Asv, _p(u), _p(J))
        return J

    def integrate(self, T, Asv, u0, tf, rtol=1e-6, atol=1e-10, analytic_jac=False, max_steps=100000,
                  record=False):
        u = np.array(u0, dtype=np.float64)
        o = Opts(rtol, atol, int(analytic_jac), max_steps, 0.0, 0.0, self.ign1)
        st = Stats()
        rows = []
        ng, ns = self.ng, self.ns

        def cb(_user, t, up, p, xp, thp):
            rows.append((t, np.ctypeslib.as_array(up, (self.n,)).copy(), p,
                         np.ctypeslib.as_array(xp, (max(ng, 1),))[:ng].copy(),
                         np.ctypeslib.as_array(thp, (max(ns, 1),))[:ns].copy() if ns else np.zeros(0)))

        fcb = STEP_CB(cb) if record else STEP_CB()
        r = lib().orc_integrate(self.h, T, Asv, _p(u), tf, C.byref(o), C.byref(st), fcb, None)
        return u, st.asdict(), rows

    def integrate_out(self, T, Asv, u0, tf, tout, rtol=1e-6, atol=1e-10, analytic_jac=False, max_steps=100000):
        """State at the output times `tout` (ascending), CVODE CV_NORMAL + CVodeGetDky semantics."""
        u = np.array(u0, dtype=np.float64)
        tout = np.ascontiguousarray(tout, dtype=np.float64)
        Y = np.zeros((len(tout), self.n))
        o = Opts(rtol, atol, int(analytic_jac), max_steps, 0.0, 0.0, self.ign1)
        st = Stats()
        lib().orc_integrate_out(self.h, T, Asv, _p(u), tf, C.byref(o), C.byref(st), len(tout), _p(tout), _p(Y))
        return u, st.asdict(), Y

    def integrate_batch(self, T, Asv, U0, tf, rtol=1e-6, atol=1e-10, analytic_jac=True, nthreads=0, tout=None):
        """OpenMP ensemble; with `tout`, also returns the states there (Y[N][len(tout)][n])."""
        N = len(T)
        U = np.array(U0, dtype=np.float64, order="C").reshape(N, self.n)
        T = np.ascontiguousarray(T, dtype=np.float64)
        Asv = np.ascontiguousarray(Asv, dtype=np.float64)
        tf = np.ascontiguousarray(np.broadcast_to(tf, (N,)), dtype=np.float64)
        o = Opts(rtol, atol, int(analytic_jac), 100000, 0.0, 0.0, self.ign1)
        st = (Stats * N)()
        if tout is None:
            bad = lib().orc_integrate_batch(self.h, N, _p(T), _p(Asv), _p(U), _p(tf), C.byref(o), st, nthreads)
            return U, [s.asdict() for s in st], bad
        tout = np.ascontiguousarray(tout, dtype=np.float64)
        Y = np.zeros((N, len(tout), self.n))
        bad = lib().orc_integrate_batch_out(self.h, N, _p(T), _p(Asv), _p(U), _p(tf), C.byref(o), st, nthreads,
                                            len(tout), _p(tout), _p(Y))
        return U, [s.asdict() for s in st], bad, Y
