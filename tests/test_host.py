"""Host-side checks that need no GPU: the mechanism compiler, the batch.xml reader, the C-ABI
library's exports, and agreement of the product's independent parser with the oracle's."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, LIB, ROOT


def test_parse_grimech(pkg):
    m = pkg.Mechanism.from_files(LIB, gas_mech="grimech.dat")
    assert (m.ng, m.nrg, m.ns, m.nrs) == (53, 325, 0, 0)
    t = m.tables
    assert int((t["g_tb"] == 2).sum()) == 29           # falloff
    assert int((t["g_troe_n"] > 0).sum()) == 26          # Troe
    assert int((t["g_tb"] == 1).sum()) == 12             # +M
    assert int(t["g_rev"].sum()) == 309
    assert int(t["g_nf"].sum()) == 649 and int(t["g_nr"].sum()) == 639
    nondefault = sum(len(r.efficiencies) for r in m.gas_rxns)
    assert nondefault == 278


def test_parse_h2o2_and_surface(pkg):
    h = pkg.Mechanism.from_files(LIB, gas_mech="h2o2.dat")
    assert (h.ng, h.nrg) == (9, 18)
    assert int((h.tables["g_tb"] == 1).sum()) == 5
    s = pkg.Mechanism.from_files(LIB, surface_mech="ch4ni.xml", gasphase="CH4 H2O H2 CO CO2 O2 N2".split())
    assert (s.ng, s.ns, s.nrs) == (7, 13, 42)
    assert int(s.tables["s_stick"].sum()) == 6
    assert int((s.tables["s_ncov"] > 0).sum()) == 4
    assert s.site_density == 2.66e-9
    np.testing.assert_array_equal(s.theta0[[0, 4]], [0.6, 0.4])


def test_molwt_matches_oracle(pkg, orc):
    m = pkg.Mechanism.from_files(LIB, gas_mech="grimech.dat")
    o = orc.Mech(os.path.join(LIB, "grimech.dat"), os.path.join(LIB, "therm.dat"))
    assert m.gas_species == o.names[:o.ng]
    np.testing.assert_array_equal(m.molwt, o.M)


def test_initial_state_matches_oracle(pkg, orc):
    m = pkg.Mechanism.from_files(LIB, gas_mech="grimech.dat", surface_mech="ch4ni.xml")
    o = orc.Mech(os.path.join(LIB, "grimech.dat"), os.path.join(LIB, "therm.dat"), os.path.join(LIB, "ch4ni.xml"))
    x = m.mole_fractions({"CH4": 0.25, "O2": 0.5, "N2": 0.25})
    np.testing.assert_array_equal(m.initial_state(1173.0, 1e5, x), o.initial_state(1173.0, 1e5, x))


def test_batch_xml(pkg):
    d = pkg.read_batch_xml(os.path.join(GOLDEN, "batch_surf", "batch.xml"))
    assert d["T"] == 1073.15 and d["Asv"] == 10 and d["time"] == 10
    assert d["gasphase"] == ["CH4", "H2O", "H2", "CO", "CO2", "O2", "N2"]
    assert d["molefractions"] == {"CH4": 0.25, "H2O": 0.25, "N2": 0.5}
    d = pkg.read_batch_xml(os.path.join(GOLDEN, "batch_gas_and_surf", "batch.xml"))
    assert d["gas_mech"] == "grimech.dat" and d["surface_mech"] == "ch4ni.xml" and "Asv" not in d


def test_library_exports_every_declared_symbol(pkg):
    """libbrhip.so loads without a GPU and exports every function include/brhip.h declares."""
    hdr = open(os.path.join(ROOT, "include", "brhip.h")).read()
    declared = set(re.findall(r"^\s*(?:int|const char\*)\s+(br_\w+)\s*\(", hdr, re.M))
    assert len(declared) >= 12
    lib = ctypes.CDLL(pkg._lib.LIBPATH)
    for name in declared:
        assert hasattr(lib, name), name
    assert set(pkg._lib.EXPORTS) == declared
    assert pkg._lib.lib().br_version() >= 100


def test_library_is_gfx950_code_object(pkg):
    """The embedded device code object targets gfx950 (MI355X)."""
    data = open(pkg._lib.LIBPATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_state_to_molefrac_roundtrip(pkg):
    m = pkg.Mechanism.from_files(LIB, gas_mech="h2o2.dat")
    x = m.mole_fractions({"H2": 0.25, "O2": 0.25, "N2": 0.5})
    u = m.initial_state(1173.0, 1e5, x)
    np.testing.assert_allclose(m.state_to_molefrac(u), x, rtol=1e-15, atol=1e-16)


def test_csv_writer_is_julia_string_format(pkg):
    """save_data writes CSV through Julia's string(::Float64) (src/BatchReactor.jl:395-399,
    RxnHelperUtils.write_csv): every number token of the reference's own gas+surf CSVs (committed
    fixture rows, tokens verbatim) is reproduced character for character (e-5, not e-05; 1.0e-5;
    100000.0; 0.0001)."""
    import csv
    n = 0
    for name in ("gas_and_surf_golden.csv", "gas_and_surf_covg_golden.csv"):
        for r in list(csv.reader(open(os.path.join(GOLDEN, name))))[1:]:
            for tok in r[1:]:
                assert pkg.julia_string(float(tok)) == tok, tok
                n += 1
    assert n > 20000
    for v, s in ((1e6, "1.0e6"), (123456.7, "123456.7"), (1e-5, "1.0e-5"), (-2.5e-7, "-2.5e-7"), (0.0, "0.0"),
                 (1173.0, "1173.0"), (10.0, "10.0")):
        assert pkg.julia_string(v) == s


def _udf_dir(tmp_path):
    import shutil
    d = tmp_path / "batch_udf"
    d.mkdir()
    shutil.copy(os.path.join(GOLDEN, "batch_udf", "batch.xml"), d / "batch.xml")
    return d


def test_udf_zero_source_success(pkg, tmp_path):
    """Reference testset "Testing user defined chemistry" (test/runtests.jl:70-77): a udf that sets
    state.source to zero returns Success; the gas profile rows keep the inlet state."""
    d = _udf_dir(tmp_path)

    def udf(state):
        state.source[:] = 0.0
    assert pkg.batch_reactor(str(d / "batch.xml"), LIB, udf) == "Success"
    rows = open(d / "gas_profile.csv").read().splitlines()
    assert rows[0] == "t,T,p,rho,CH4,H2O,H2,CO,CO2,O2,N2"
    last = rows[-1].split(",")
    assert float(last[0]) == 10.0 and last[4:] == ["0.25", "0.25", "0.0", "0.0", "0.0", "0.0", "0.5"]
    assert open(d / "surface_covg.csv").read() == ""          # opened, never written (:171-173)


def test_udf_source_integrates(pkg, tmp_path):
    """A constant udf source S_k [mol/m3/s] gives rho_k(t) = rho_k(0) + S_k M_k t exactly
    (du = source .* molwt, src/BatchReactor.jl:371-372); the state handed to the udf keeps the inlet
    T, p and mole fractions (residual! never updates u_state, :358-360)."""
    d = _udf_dir(tmp_path)
    seen = []

    def udf(state):
        seen.append((state.T, state.p, state.mole_frac.copy()))
        state.source[:] = 0.0
        state.source[state.species.index("H2")] = 1e-3
        state.source[state.species.index("CH4")] = -1e-4
    assert pkg.batch_reactor(str(d / "batch.xml"), LIB, udf) == "Success"
    rows = [r.split(",") for r in open(d / "gas_profile.csv").read().splitlines()[1:]]
    m = pkg.Mechanism.from_files(LIB, gasphase="CH4 H2O H2 CO CO2 O2 N2".split())
    rho0 = m.initial_state(1073.15, 1e5, m.mole_fractions({"CH4": 0.25, "H2O": 0.25, "N2": 0.5})).sum()
    dM = 1e-3 * m.molwt[2] - 1e-4 * m.molwt[0]
    for r in rows:
        assert abs(float(r[3]) - (rho0 + dM * float(r[0]))) <= 1e-9 * rho0
    assert all(s[0] == 1073.15 and s[1] == 1e5 for s in seen)


def test_sens_returns_params_prob_tspan(pkg, tmp_path):
    """sens=true returns (params, prob, t_span) (src/BatchReactor.jl:205-207): params carries the
    reference's fields, prob.f is residual!(du, u, p, t)."""
    d = _udf_dir(tmp_path)

    def udf(state):
        state.source[:] = 2.0
    params, prob, t_span = pkg.batch_reactor(str(d / "batch.xml"), LIB, udf, sens=True)
    assert t_span == (0.0, 10.0) and prob.tspan == t_span
    assert set(params) == {"s_state", "g_state", "u_state", "thermo", "smd", "gmd", "cp", "chem"}
    assert params["cp"].Asv == 10.0 and params["cp"].T == 1073.15 and params["chem"].userchem
    du = np.zeros_like(prob.u0)
    prob.f(du, prob.u0, prob.p, 0.0)
    np.testing.assert_allclose(du, 2.0 * params["thermo"].molwt)


def test_reference_conventions_are_default(pkg, orc):
    """The reference's gas-kinetics conventions (CONV_REFERENCE) are the
    default of the product compiler and of the oracle; textbook CHEMKIN stays available (conv=0)."""
    m = pkg.Mechanism.from_files(LIB, gas_mech="grimech.dat")
    assert m.conv == pkg.CONV_REFERENCE == orc.CONV_REFERENCE == 19
    assert pkg.Mechanism.from_files(LIB, gas_mech="h2o2.dat", conv=0).conv == 0


# --------------------------------------------------------------------------------------------
# native (C++) mechanism compiler of libbrhip.so: br_mech_parse / br_read_batch_xml, the path a
# Julia host uses (julia/BatchReactorHIP.jl) -- must give the Python compiler's tables bit for bit
# --------------------------------------------------------------------------------------------
_DESC_SHAPES = {  # field -> shape from (ng, ns, nrg, nrs)
    "molwt": lambda g, s, r, q: (g,), "nasa": lambda g, s, r, q: (g, 15),
    "g_nf": lambda g, s, r, q: (r,), "g_nr": lambda g, s, r, q: (r,), "g_f": lambda g, s, r, q: (r, 4),
    "g_r": lambda g, s, r, q: (r, 4), "g_rev": lambda g, s, r, q: (r,), "g_tb": lambda g, s, r, q: (r,),
    "g_arr": lambda g, s, r, q: (r, 3), "g_low": lambda g, s, r, q: (r, 3), "g_troe_n": lambda g, s, r, q: (r,),
    "g_troe": lambda g, s, r, q: (r, 4), "g_eff": lambda g, s, r, q: (r, g), "sigma": lambda g, s, r, q: (s,),
    "s_nf": lambda g, s, r, q: (q,), "s_np": lambda g, s, r, q: (q,), "s_f": lambda g, s, r, q: (q, 6),
    "s_p": lambda g, s, r, q: (q, 6), "s_stick": lambda g, s, r, q: (q,), "s_arr": lambda g, s, r, q: (q, 3),
    "s_ncov": lambda g, s, r, q: (q,), "s_cov_sp": lambda g, s, r, q: (q, 4), "s_cov_eps": lambda g, s, r, q: (q, 4),
}


def _native(pkg, gas=None, surf=None, gasphase=None, conv=None):
    L = pkg._lib.lib()
    h = ctypes.c_void_p()
    enc = lambda s: None if s is None else s.encode()
    rc = L.br_mech_parse(enc(gas and os.path.join(LIB, gas)), enc(os.path.join(LIB, "therm.dat")),
                         enc(surf and os.path.join(LIB, surf)), enc(gasphase),
                         pkg.CONV_REFERENCE if conv is None else conv, ctypes.byref(h))
    if rc:
        return rc, L.br_last_error().decode()
    d = pkg._lib.MechDesc()
    assert L.br_host_mech_desc(h, ctypes.byref(d)) == 0
    sizes = (d.ng, d.ns, d.nrg, d.nrs)
    out = {"sizes": sizes, "conv": d.conv, "p_std": d.p_std, "site_density": d.site_density}
    for f, shp in _DESC_SHAPES.items():
        s = shp(*sizes)
        p = getattr(d, f)
        out[f] = np.ctypeslib.as_array(p, shape=s).copy() if int(np.prod(s)) > 0 else None
    buf = ctypes.create_string_buffer(64)
    names = []
    for i in range(d.ng + d.ns):
        assert L.br_host_mech_species(h, i, buf, 64) == 0
        names.append(buf.value.decode())
    out["names"] = names
    th = np.zeros(d.ns)
    assert L.br_host_mech_theta0(h, pkg._lib.dptr(th)) == 0
    out["theta0"] = th
    assert L.br_host_mech_free(h) == 0
    return 0, out


@pytest.mark.parametrize("gas,surf,gasphase", [("grimech.dat", None, None), ("h2o2.dat", None, None),
                                               (None, "ch4ni.xml", "CH4 H2O H2 CO CO2 O2 N2"),
                                               ("grimech.dat", "ch4ni.xml", None)])
def test_native_compiler_tables_bit_identical(pkg, gas, surf, gasphase):
    """br_mech_parse (C++, libbrhip.so) builds the same br_mech_desc tables as the Python host
    compiler, bit for bit (GRI, H2/O2, surface-only, gas + surface), with the same species order."""
    rc, nat = _native(pkg, gas, surf, gasphase)
    assert rc == 0, nat
    m = pkg.Mechanism.from_files(LIB, gas_mech=gas, surface_mech=surf, gasphase=gasphase and gasphase.split())
    assert nat["sizes"] == (m.ng, m.ns, m.nrg, m.nrs)
    assert nat["names"] == m.species
    assert nat["conv"] == m.conv and nat["p_std"] == m.p_std and nat["site_density"] == m.site_density
    py = dict(m.tables, molwt=m.molwt, nasa=m.nasa, sigma=m.sigma)
    for f in _DESC_SHAPES:
        a, b = nat[f], np.asarray(py[f])
        if a is None:
            assert b.size == 0, f
            continue
        assert a.shape == b.shape, f
        if a.dtype.kind == "f":
            assert np.array_equal(a.view(np.uint64), np.ascontiguousarray(b, np.float64).view(np.uint64)), f
        else:
            assert np.array_equal(a, b), f
    np.testing.assert_array_equal(nat["theta0"], m.theta0)


def test_native_compiler_errors(pkg, tmp_path):
    """Bad inputs come back as BR_ERR_INPUT with a message (no exception crosses the C-ABI)."""
    rc, msg = _native(pkg, "nonexistent.dat")
    assert rc == -10 and "cannot open" in msg
    bad = tmp_path / "bad.dat"
    bad.write_text("ELEMENTS H O END\nSPECIES H2 O2 END\nREACTIONS\nH2+XX=2H 1.0 0.0 0.0\nEND\n")
    L = pkg._lib.lib()
    h = ctypes.c_void_p()
    rc = L.br_mech_parse(str(bad).encode(), os.path.join(LIB, "therm.dat").encode(), None, None, 19, ctypes.byref(h))
    assert rc == -10 and "unknown species 'XX'" in L.br_last_error().decode()


@pytest.mark.parametrize("case", ["batch_h2o2", "batch_ch4", "batch_surf", "batch_gas_and_surf", "batch_udf"])
def test_native_batch_xml(pkg, case):
    """br_read_batch_xml reads the five reference scenario inputs as the Python reader does
    (input_data, src/BatchReactor.jl:238-306); a missing <Asv> gives Asv = 1."""
    path = os.path.join(GOLDEN, case, "batch.xml")
    b = pkg._lib.BatchInput()
    assert pkg._lib.lib().br_read_batch_xml(path.encode(), ctypes.byref(b)) == 0
    d = pkg.read_batch_xml(path)
    assert b.gas_mech.decode() == d.get("gas_mech", "") and b.surface_mech.decode() == d.get("surface_mech", "")
    assert b.gasphase.decode().split() == d.get("gasphase", [])
    assert (b.T, b.p, b.time) == (d["T"], d["p"], d["time"])
    assert b.has_Asv == ("Asv" in d) and b.Asv == d.get("Asv", 1.0)
    comp = {b.comp_names[i].value.decode(): b.comp_values[i] for i in range(b.ncomp)}
    assert comp == d["molefractions"] and b.comp_is_mass == 0


@pytest.mark.parametrize("field", ["species", "gas_mech"])
def test_native_batch_xml_overlong_name(pkg, tmp_path, field):
    """A name that does not fit its br_batch_input field is an input error, not a silent
    truncation (a truncated species name would drop its composition entry)."""
    long = "X" * 300
    sp = long if field == "species" else "CH4"
    gm = long if field == "gas_mech" else "grimech.dat"
    p = tmp_path / "batch.xml"
    p.write_text(f"<batch><gas_mech>{gm}</gas_mech><gasphase>CH4 O2 N2</gasphase>"
                 f"<molefractions>{sp}=0.25,O2=0.5,N2=0.25</molefractions>"
                 "<T>1173</T><p>1e5</p><time>10</time></batch>")
    L = pkg._lib.lib()
    b = pkg._lib.BatchInput()
    assert L.br_read_batch_xml(str(p).encode(), ctypes.byref(b)) == -10
    assert "too long" in L.br_last_error().decode()


def test_cli_julia_string_format(pkg):
    """brhip_batch (the C-ABI-only batch_reactor program) formats CSV numbers as Julia's
    string(::Float64): every number token of the reference's own gas+surf CSVs comes back verbatim."""
    import csv
    toks = []
    for name in ("gas_and_surf_golden.csv", "gas_and_surf_covg_golden.csv"):
        for r in list(csv.reader(open(os.path.join(GOLDEN, name))))[1:]:
            toks += r[1:]
    cli = os.path.join(ROOT, "batchreactor.jl_amd", "brhip_batch")
    out = subprocess.run([cli, "--fmt"], input="\n".join(toks), capture_output=True, text=True, check=True).stdout.split()
    assert out == toks


def test_retcode_symbols(pkg):
    """Engine status -> Symbol(sol.retcode) of the reference's CVODE_BDF solve (src/BatchReactor.jl:216),
    one case per status code the engine returns (include/brhip.h), the same table as the Julia host's
    retcode_symbol (checked there by text in test_julia_binding)."""
    from batchreactor_amd import reactor
    want = {0: "Success", -1: "MaxIters", -3: "Unstable", -4: "ConvergenceFailure", -7: "Unstable",
            -10: "Failure", -20: "Failure", -30: "Failure"}
    for status, sym in want.items():
        assert reactor.retcode(status) == sym
        assert reactor.retcode(float(status)) == sym   # stats arrive as doubles
    jl = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "julia",
                           "BatchReactorHIP.jl")).read()
    body = jl[jl.index("function retcode_symbol"):]
    body = body[:body.index("\nend")]
    for status, sym in want.items():
        if sym in ("Success", "MaxIters", "ConvergenceFailure"):
            assert f":{sym}" in body
    assert "s == -4 && return :ConvergenceFailure" in body and "s == -1 && return :MaxIters" in body
    assert "(s == -2 || s == -3 || s == -7) && return :Unstable" in body and "return :Failure" in body


@pytest.mark.parametrize("mech_file,T,x", [("h2o2.dat", 1173.0, {"H2": 0.25, "O2": 0.25, "N2": 0.5}),
                                           ("grimech.dat", 1200.0, {"CH4": 0.25, "O2": 0.5, "N2": 0.25})])
def test_host_cvode_matches_oracle_dq(pkg, orc, mech_file, T, x):
    """br_integrate_host (the udf path's solver: CVODE 5.x on the CPU with a caller's RHS and CVODE's DQ
    Jacobian, src/BatchReactor.jl:204-210) driven by the oracle's own residual! through the ctypes
    callback, against the oracle's integration of the same problem with the DQ Jacobian: the same
    algorithm, so the same accepted steps, counters and end state (to rounding: the two are compiled
    separately). Also the save_data rows: one per accepted step plus t = 0."""
    from batchreactor_amd import _lib
    om = orc.Mech(os.path.join(LIB, mech_file), os.path.join(LIB, "therm.dat"))
    m = pkg.Mechanism.from_files(LIB, gas_mech=mech_file)
    u0 = m.initial_state(T, 1e5, m.mole_fractions(x))
    tf = 1e-2
    rows = []
    status, u, st = _lib.integrate_host(lambda t, u: om.rhs(T, 1.0, u)[0], u0, tf,
                                        on_step=lambda t, u: rows.append((t, u)))
    uo, so, _ = om.integrate(T, 1.0, u0, tf, analytic_jac=False)
    assert status == 0 and so["status"] == 0
    assert int(st[0]) == so["nsteps"] and int(st[2]) == so["nje"] and int(st[3]) == so["nsetups"]
    assert int(st[1]) == so["nfe"] and int(st[4]) == so["nni"] and int(st[19]) == so["nfeDQ"]
    np.testing.assert_allclose(u, uo, rtol=1e-12, atol=1e-22)
    assert len(rows) == so["nsteps"] + 1 and rows[0][0] == 0.0 and rows[-1][0] == tf


def test_host_cvode_status_codes(pkg):
    """br_integrate_host's failure paths and their SciML retcodes: a step limit -> MaxIters, a NaN
    right-hand side -> Unstable-class failure, an exception in the RHS -> re-raised, bad input -> -10."""
    from batchreactor_amd import _lib, reactor
    f = lambda t, u: -1e3 * (u - np.array([1.0, 2.0]))   # noqa: E731  (stiff linear relaxation)
    status, u, st = _lib.integrate_host(f, [0.0, 0.0], 10.0)
    assert status == 0 and np.allclose(u, [1.0, 2.0], rtol=1e-5)
    status, _, st = _lib.integrate_host(f, [0.0, 0.0], 10.0, max_steps=5)
    assert status == -1 and int(st[0]) == 5 and reactor.retcode(status) == "MaxIters"
    status, _, _ = _lib.integrate_host(lambda t, u: np.full(2, np.nan), [1.0, 1.0], 1.0)
    assert status < 0 and reactor.retcode(status) != "Success"

    def boom(t, u):
        raise ValueError("udf failed")
    with pytest.raises(ValueError):
        _lib.integrate_host(boom, [1.0], 1.0)
    assert _lib.integrate_host(f, [0.0, 0.0], -1.0)[0] == -10


def test_host_cvode_robertson_against_scipy(pkg):
    """br_integrate_host on a classic stiff problem that has nothing to do with the oracle (Robertson,
    k1 = 0.04, k2 = 3e7, k3 = 1e4, t = 0..40): against SciPy's Radau at rtol 1e-10, the end state agrees
    to the CVODE tolerance level (rtol 1e-6 / atol 1e-10), mass is conserved, and the DQ Jacobian path
    is used (nje > 0, nfe_dq = n nje)."""
    from scipy.integrate import solve_ivp
    from batchreactor_amd import _lib

    def f(t, y):
        return np.array([-0.04 * y[0] + 1e4 * y[1] * y[2],
                         0.04 * y[0] - 1e4 * y[1] * y[2] - 3e7 * y[1] ** 2,
                         3e7 * y[1] ** 2])
    status, u, st = _lib.integrate_host(f, [1.0, 0.0, 0.0], 40.0)
    assert status == 0 and int(st[2]) > 0 and int(st[19]) == 3 * int(st[2])
    ref = solve_ivp(f, (0.0, 40.0), [1.0, 0.0, 0.0], method="Radau", rtol=1e-10, atol=1e-14).y[:, -1]
    assert np.all(np.abs(u - ref) <= 1e-4 * np.abs(ref) + 1e-9), (u, ref)
    assert abs(u.sum() - 1.0) <= 1e-9
