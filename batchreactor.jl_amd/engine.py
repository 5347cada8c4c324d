"""Engine: a compiled mechanism resident on one GPU (br_mech handle) and the batched hot-path
operators on it. This is the host mirror of the reference's operator interface:

  rates(...)      <- GasphaseReactions / SurfaceReactions.calculate_molar_production_rates!
                     (src/BatchReactor.jl:344,:355), batched
  rhs(...)        <- residual!(du,u,p,t) (src/BatchReactor.jl:312-376), batched
  jacobian(...)   <- the dense Jacobian CVODE forms inside CVODE_BDF() (:138-141,:210)
  integrate(...)  <- solve(ODEProblem(residual!,u0,(0,tf),params), CVODE_BDF();
                     reltol=1e-6, abstol=1e-10, save_everystep=false) (:138-141,:204-210)

Arrays are reactor-major: u[N, n], n = ng + ns, u = [rho*Y_k ; theta_k].
"""
import ctypes as C

import numpy as np

from . import _lib
from .mechanism import Mechanism

STAT_FIELDS = ("nsteps", "nfe", "nje", "nsetups", "nni", "ncfn", "netf", "status", "cyc_total", "cyc_rhs",
               "cyc_jac", "cyc_lu", "cyc_sol", "t_end", "cyc_ctl", "cyc_clk", "t_ign", "ign_rate", "ign_dt",
               "nfe_dq")
IGNITION_MARKER = "OH"   # the reference golden's ignition marker: max dX_OH/dt


class Engine:
    def __init__(self, mech: Mechanism, device: int = 0):
        L = _lib.lib()
        self.mech = mech
        self.device = device
        t = mech.tables
        self._keep = []

        def d(a):
            a = np.ascontiguousarray(a, dtype=np.float64)
            self._keep.append(a)
            return _lib.dptr(a)

        def i(a):
            a = np.ascontiguousarray(a, dtype=np.int32)
            self._keep.append(a)
            return _lib.iptr(a)

        desc = _lib.MechDesc(
            mech.ng, mech.ns, mech.nrg, mech.nrs, mech.conv, mech.p_std,
            d(mech.molwt), d(mech.nasa),
            i(t["g_nf"]), i(t["g_nr"]), i(t["g_f"]), i(t["g_r"]), i(t["g_rev"]), i(t["g_tb"]),
            d(t["g_arr"]), d(t["g_low"]), i(t["g_troe_n"]), d(t["g_troe"]), d(t["g_eff"]),
            mech.site_density, d(mech.sigma),
            i(t["s_nf"]), i(t["s_np"]), i(t["s_f"]), i(t["s_p"]), i(t["s_stick"]), d(t["s_arr"]),
            i(t["s_ncov"]), i(t["s_cov_sp"]), d(t["s_cov_eps"]))
        h = C.c_void_p()
        _lib.check(L.br_mech_create(C.byref(desc), device, C.byref(h)))
        self.h = h
        self.n, self.ng, self.ns = mech.n, mech.ng, mech.ns
        # 1-based br_opts.ignition_species (0: the mechanism has no OH, t_ign not tracked)
        self.ign1 = mech.gas_species.index(IGNITION_MARKER) + 1 if IGNITION_MARKER in mech.gas_species else 0
        self.nmax = 16 if self.n <= 16 else 32 if self.n <= 32 else 56 if self.n <= 56 else 64 if self.n <= 64 else 72   # kernel tile

    @property
    def kernel_name(self) -> str:
        """the integrator kernel br_integrate_dev launches for this mechanism"""
        nm = _lib.lib().br_mech_engine(self.h)
        if nm < 0:   # group engine: -(100 * group width + register width)
            return f"k_group<{-nm // 100}, {-nm % 100}>"
        return f"k_lane<{nm}>" if nm > 0 else f"k_integrate<{self.nmax}>"

    @property
    def engine(self) -> str:
        """'lane' (one reactor per lane, small gas mechanisms), 'quad' / 'pair' (four / two reactors
        per wavefront, one per 16- / 32-lane group, n <= 16 / 32) or 'wave' (one reactor per wavefront)"""
        nm = _lib.lib().br_mech_engine(self.h)
        if nm < 0:
            return "quad" if -nm // 100 == 16 else "pair"
        return "lane" if nm > 0 else "wave"

    @property
    def launch_info(self) -> dict:
        """launch geometry of the engine in use (wave / group / lane): reactors per workgroup, resident
        waves per CU, LDS bytes per workgroup (br_mech_launch_info)"""
        rpb, wpc, lds = C.c_int(), C.c_int(), C.c_longlong()
        _lib.check(_lib.lib().br_mech_launch_info(self.h, C.byref(rpb), C.byref(wpc), C.byref(lds)))
        return {"reactors_per_workgroup": rpb.value, "waves_per_cu": wpc.value, "lds_bytes_per_workgroup": lds.value}

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().br_mech_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _arr(a, N, dtype=np.float64):
        return np.ascontiguousarray(np.broadcast_to(np.asarray(a, dtype), (N,)))

    def rates(self, T, p, x, theta=None):
        x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float64)
        N = x.shape[0]
        T, p = self._arr(T, N), self._arr(p, N)
        th = None if (theta is None or self.ns == 0) else np.ascontiguousarray(np.atleast_2d(theta), dtype=np.float64)
        w = np.zeros((N, self.ng))
        s = np.zeros((N, self.n))
        _lib.check(_lib.lib().br_rates(self.h, N, _lib.dptr(T), _lib.dptr(p), _lib.dptr(x), _lib.dptr(th),
                                       _lib.dptr(w), _lib.dptr(s)))
        return w, s

    def rhs(self, T, Asv, u):
        u = np.ascontiguousarray(np.atleast_2d(u), dtype=np.float64)
        N = u.shape[0]
        T, A = self._arr(T, N), self._arr(Asv, N)
        du = np.zeros_like(u)
        _lib.check(_lib.lib().br_rhs(self.h, N, _lib.dptr(T), _lib.dptr(A), _lib.dptr(u), _lib.dptr(du)))
        return du

    def jacobian(self, T, Asv, u):
        u = np.ascontiguousarray(np.atleast_2d(u), dtype=np.float64)
        N = u.shape[0]
        T, A = self._arr(T, N), self._arr(Asv, N)
        J = np.zeros((N, self.n, self.n))
        _lib.check(_lib.lib().br_jacobian(self.h, N, _lib.dptr(T), _lib.dptr(A), _lib.dptr(u), _lib.dptr(J)))
        return J

    def _opts(self, rtol, atol, max_steps, trace_cap=0, unstable_factor=0.0, tout=None, yout=None, dq_jacobian=False):
        nout = 0 if tout is None else len(tout)
        return _lib.Opts(rtol, atol, max_steps, self.device, 0.0, trace_cap, unstable_factor, self.ign1, nout,
                         _lib.dptr(tout) if nout else None, _lib.dptr(yout) if nout else None, int(dq_jacobian))

    def integrate(self, T, Asv, u0, tf, rtol=1e-6, atol=1e-10, max_steps=100000, trace_cap=0, tout=None,
                  unstable_factor=0.0, dq_jacobian=False):
        """Integrate N reactors 0 -> tf. With trace_cap > 0 also returns the per-step rows
        trace[N, trace_cap+1, 2n+4] = (t, h, q, p_last, u[n], y_last[n]): u the accepted state, y_last
        and p_last the state and pressure of the step's last RHS evaluation (save_data semantics).
        With tout (ascending output times) the stats dict also carries "yout" [N, nout, n], the
        states at those times (CVODE CV_NORMAL output, the step sequence is unchanged).
        dq_jacobian: CVODE's difference-quotient Jacobian (the reference's setting), both engines."""
        u = np.array(np.atleast_2d(u0), dtype=np.float64, order="C")
        N = u.shape[0]
        T, A, tf = self._arr(T, N), self._arr(Asv, N), self._arr(tf, N)
        st = np.zeros((N, _lib.NSTAT))
        to = None if tout is None else np.ascontiguousarray(tout, dtype=np.float64)
        yo = None if tout is None else np.zeros((N, len(to), self.n))
        o = self._opts(rtol, atol, max_steps, trace_cap, unstable_factor, to, yo, dq_jacobian)
        L = _lib.lib()
        if trace_cap > 0:
            tr = np.zeros((N, trace_cap + 1, 2 * self.n + 4))
            _lib.check(L.br_integrate_traced(self.h, N, _lib.dptr(T), _lib.dptr(A), _lib.dptr(u), _lib.dptr(tf),
                                             C.byref(o), _lib.dptr(st), _lib.dptr(tr)))
        else:
            tr = None
            _lib.check(L.br_integrate(self.h, N, _lib.dptr(T), _lib.dptr(A), _lib.dptr(u), _lib.dptr(tf),
                                      C.byref(o), _lib.dptr(st)))
        stats = {k: st[:, i] for i, k in enumerate(STAT_FIELDS)}
        if yo is not None:
            stats["yout"] = yo
        return (u, stats, tr) if trace_cap > 0 else (u, stats)

    def integrate_device(self, T_ptr, Asv_ptr, u_ptr, tf_ptr, stats_ptr, N, stream_ptr=None, rtol=1e-6,
                         atol=1e-10, max_steps=100000):
        """Device-resident variant: raw device pointers (e.g. torch tensor data_ptr())."""
        o = self._opts(rtol, atol, max_steps)
        _lib.check(_lib.lib().br_integrate_dev(self.h, N, C.c_void_p(T_ptr), C.c_void_p(Asv_ptr),
                                               C.c_void_p(u_ptr), C.c_void_p(tf_ptr), C.byref(o),
                                               C.c_void_p(stats_ptr), C.c_void_p(stream_ptr or 0)))

    def last_kernel_ms(self):
        ms = np.zeros(1)
        _lib.check(_lib.lib().br_last_kernel_ms(self.h, _lib.dptr(ms)))
        return float(ms[0])


def integrate_multi(engines, T, Asv, u0, tf, rtol=1e-6, atol=1e-10, max_steps=100000, tout=None):
    """br_integrate_multi: the ensemble split into contiguous slices over `engines` (one Engine per
    GPU, same mechanism), integrated concurrently; returns (u, stats) in ensemble order."""
    L = _lib.lib()
    e0 = engines[0]
    u = np.array(np.atleast_2d(u0), dtype=np.float64, order="C")
    N = u.shape[0]
    T, A, tf = e0._arr(T, N), e0._arr(Asv, N), e0._arr(tf, N)
    st = np.zeros((N, _lib.NSTAT))
    to = None if tout is None else np.ascontiguousarray(tout, dtype=np.float64)
    yo = None if tout is None else np.zeros((N, len(to), e0.n))
    o = e0._opts(rtol, atol, max_steps, 0, 0.0, to, yo)
    hs = (C.c_void_p * len(engines))(*[e.h.value for e in engines])
    _lib.check(L.br_integrate_multi(hs, len(engines), N, _lib.dptr(T), _lib.dptr(A), _lib.dptr(u), _lib.dptr(tf),
                                    C.byref(o), _lib.dptr(st)))
    stats = {k: st[:, i] for i, k in enumerate(STAT_FIELDS)}
    if yo is not None:
        stats["yout"] = yo
    return u, stats
