"""ctypes binding of libbrhip.so (include/brhip.h). Fails loudly when the library is absent:
there is no CPU fallback in the product path."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBPATH = os.environ.get("BRHIP_LIB") or os.path.join(HERE, "libbrhip.so")

dp = C.POINTER(C.c_double)
ip = C.POINTER(C.c_int)


class MechDesc(C.Structure):
    _fields_ = [
        ("ng", C.c_int), ("ns", C.c_int), ("nrg", C.c_int), ("nrs", C.c_int),
        ("conv", C.c_int), ("p_std", C.c_double),
        ("molwt", dp), ("nasa", dp),
        ("g_nf", ip), ("g_nr", ip), ("g_f", ip), ("g_r", ip), ("g_rev", ip), ("g_tb", ip),
        ("g_arr", dp), ("g_low", dp), ("g_troe_n", ip), ("g_troe", dp), ("g_eff", dp),
        ("site_density", C.c_double), ("sigma", dp),
        ("s_nf", ip), ("s_np", ip), ("s_f", ip), ("s_p", ip), ("s_stick", ip), ("s_arr", dp),
        ("s_ncov", ip), ("s_cov_sp", ip), ("s_cov_eps", dp),
    ]


class Opts(C.Structure):
    _fields_ = [("rtol", C.c_double), ("atol", C.c_double), ("max_steps", C.c_int), ("device", C.c_int),
                ("hmax", C.c_double), ("trace_cap", C.c_int), ("unstable_factor", C.c_double),
                ("ignition_species", C.c_int), ("nout", C.c_int), ("tout", dp), ("yout", dp),
                ("dq_jacobian", C.c_int)]


NSTAT = 20
BATCH_MAXCOMP = 64


class BatchInput(C.Structure):
    """br_batch_input (br_read_batch_xml)"""
    _fields_ = [("gas_mech", C.c_char * 256), ("surface_mech", C.c_char * 256), ("gasphase", C.c_char * 1024),
                ("T", C.c_double), ("p", C.c_double), ("Asv", C.c_double), ("time", C.c_double),
                ("has_T", C.c_int), ("has_p", C.c_int), ("has_Asv", C.c_int), ("has_time", C.c_int),
                ("ncomp", C.c_int), ("comp_is_mass", C.c_int),
                ("comp_names", (C.c_char * 32) * BATCH_MAXCOMP), ("comp_values", C.c_double * BATCH_MAXCOMP)]


EXPORTS = ["br_version", "br_last_error", "br_device_count", "br_mech_create", "br_mech_destroy", "br_mech_info", "br_mech_engine", "br_mech_launch_info",
           "br_rates", "br_rhs", "br_jacobian", "br_integrate", "br_integrate_traced", "br_integrate_multi", "br_integrate_dev",
           "br_last_kernel_ms", "br_debug_lu_solve", "br_mech_parse", "br_host_mech_desc", "br_host_mech_sizes",
           "br_host_mech_species", "br_host_mech_theta0", "br_host_mech_free", "br_mech_compile", "br_read_batch_xml",
           "br_integrate_host"]

# br_integrate_host callbacks: int f(void* user, double t, const double* u, double* du);
# void cb(void* user, double t, const double* u)
RHS_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double))
STEP_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_double, C.POINTER(C.c_double))

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIBPATH):
        raise RuntimeError(f"libbrhip.so not built ({LIBPATH}); run __graft_entry__.build()")
    L = C.CDLL(LIBPATH)
    vp = C.c_void_p
    L.br_version.restype = C.c_int
    L.br_last_error.restype = C.c_char_p
    L.br_device_count.restype = C.c_int
    L.br_mech_create.argtypes = [C.POINTER(MechDesc), C.c_int, C.POINTER(vp)]
    L.br_mech_destroy.argtypes = [vp]
    L.br_mech_info.argtypes = [vp, ip, ip, ip, ip]
    L.br_mech_engine.argtypes = [vp]
    L.br_mech_engine.restype = C.c_int
    L.br_mech_launch_info.argtypes = [vp, ip, ip, C.POINTER(C.c_longlong)]
    L.br_rates.argtypes = [vp, C.c_int, dp, dp, dp, dp, dp, dp]
    L.br_rhs.argtypes = [vp, C.c_int, dp, dp, dp, dp]
    L.br_jacobian.argtypes = [vp, C.c_int, dp, dp, dp, dp]
    L.br_integrate.argtypes = [vp, C.c_int, dp, dp, dp, dp, C.POINTER(Opts), dp]
    L.br_integrate_traced.argtypes = [vp, C.c_int, dp, dp, dp, dp, C.POINTER(Opts), dp, dp]
    L.br_integrate_dev.argtypes = [vp, C.c_int, vp, vp, vp, vp, C.POINTER(Opts), vp, vp]
    L.br_integrate_multi.argtypes = [C.POINTER(vp), C.c_int, C.c_int, dp, dp, dp, dp, C.POINTER(Opts), dp]
    L.br_last_kernel_ms.argtypes = [vp, dp]
    L.br_debug_lu_solve.argtypes = [C.c_int, C.c_int, dp, dp, dp, dp, ip]
    L.br_debug_lu_solve.restype = C.c_int
    cs = C.c_char_p
    L.br_mech_parse.argtypes = [cs, cs, cs, cs, C.c_int, C.POINTER(vp)]
    L.br_host_mech_desc.argtypes = [vp, C.POINTER(MechDesc)]
    L.br_host_mech_sizes.argtypes = [vp, ip, ip, ip, ip]
    L.br_host_mech_species.argtypes = [vp, C.c_int, C.c_char_p, C.c_size_t]
    L.br_host_mech_theta0.argtypes = [vp, dp]
    L.br_host_mech_free.argtypes = [vp]
    L.br_mech_compile.argtypes = [cs, cs, cs, cs, C.c_int, C.c_int, C.POINTER(vp)]
    L.br_read_batch_xml.argtypes = [cs, C.POINTER(BatchInput)]
    L.br_integrate_host.argtypes = [C.c_int, RHS_FN, vp, dp, C.c_double, C.c_double, C.c_double, C.c_int, STEP_FN, vp,
                                    dp]
    for f in ("br_mech_create", "br_mech_destroy", "br_mech_info", "br_rates", "br_rhs", "br_jacobian",
              "br_integrate", "br_integrate_traced", "br_integrate_multi", "br_integrate_dev", "br_last_kernel_ms",
              "br_mech_parse", "br_host_mech_desc", "br_host_mech_sizes", "br_host_mech_species",
              "br_host_mech_theta0", "br_host_mech_free", "br_mech_compile", "br_read_batch_xml", "br_integrate_host"):
        getattr(L, f).restype = C.c_int
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise RuntimeError(f"libbrhip error {rc}: {lib().br_last_error().decode()}")


def dptr(a):
    return a.ctypes.data_as(dp) if a is not None else None


def iptr(a):
    return a.ctypes.data_as(ip)


def integrate_host(f, u0, tf, rtol=1e-6, atol=1e-10, max_steps=100000, on_step=None):
    """br_integrate_host: CVODE_BDF (the engine's CVODE 5.x restatement, DQ Jacobian) on the CPU with
    a Python right-hand side f(t, u) -> du; on_step(t, u) after every accepted step and at t = 0 / tf
    (save_data's rows). Returns (status, u_end, stats[BR_NSTAT]). An exception in f ends the solve
    with BR_ERR_RHS and is re-raised here."""
    import numpy as np
    u = np.array(u0, dtype=np.float64)
    n = len(u)
    err = []

    def rhs(_user, t, up, dup):
        try:
            du = np.asarray(f(t, np.ctypeslib.as_array(up, (n,)).copy()), dtype=np.float64)
            np.ctypeslib.as_array(dup, (n,))[:] = du
            return 0
        except BaseException as e:   # noqa: BLE001  (handed back after the C solver returns)
            err.append(e)
            return 1

    def step(_user, t, up):
        if on_step is not None and not err:
            try:
                on_step(t, np.ctypeslib.as_array(up, (n,)).copy())
            except BaseException as e:   # noqa: BLE001
                err.append(e)

    st = np.zeros(NSTAT)
    fr, fs = RHS_FN(rhs), STEP_FN(step)   # (kept alive for the call)
    status = lib().br_integrate_host(n, fr, None, dptr(u), float(tf), float(rtol), float(atol), int(max_steps), fs,
                                     None, dptr(st))
    if err:
        raise err[0]
    return status, u, st
