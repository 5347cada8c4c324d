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
