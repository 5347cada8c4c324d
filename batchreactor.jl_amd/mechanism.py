"""Host-side mechanism compiler: CHEMKIN-II gas mechanisms, NASA-7 ``therm.dat``, the
surface-mechanism XML and the ``batch.xml`` input (the data formats the reference reads).

Mirrors what the reference delegates to its chemistry packages:
  * ``compile_gaschemistry(mech_file)``              src/BatchReactor.jl:251-255
  * ``IdealGas.create_thermo(gasphase, therm.dat)``  src/BatchReactor.jl:265
  * ``SurfaceReactions.compile_mech(file, thermo, gasphase)`` src/BatchReactor.jl:283-287
  * ``input_data(xmlroot, lib_dir, chem)``           src/BatchReactor.jl:238-306
and flattens the result into the structure-of-arrays tables of ``br_mech_desc``
(include/brhip.h). Units are converted to SI here, once, on the host.
"""
from __future__ import annotations

import math
import os
import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

R_GAS = 8.31446261815324  # RxnHelperUtils.R (src/BatchReactor.jl:338)
CAL = 4.184

# Atomic weights [g/mol]. IdealGas's table is not vendored; H/C/O/N are fitted to the
# reference golden (they reproduce rho0 of test/batch_gas_and_surf/gas_profile.csv bit-exactly
# and the diagnosed pressure of every golden row to 3.5e-11). See DESIGN.md.
ATOMIC_WEIGHTS = {
    "H": 1.0078, "C": 12.0107, "O": 15.99977, "N": 14.00643, "AR": 39.948, "HE": 4.002602,
    "NE": 20.1797, "S": 32.065, "CL": 35.453, "F": 18.9984, "E": 5.48579909e-4,
}

# Gas-kinetics convention switches (include/brhip.h BR_CONV_*). 0 = textbook CHEMKIN-II in SI.
# CONV_REFERENCE = what the reference's GasphaseReactions does (identified from its golden output,
# DESIGN.md section 1): rates in mol/cm3 with Kc in mol/m3 (Kc *= 1e6^dnu), falloff rates x [M]
# in mol/cm3, Troe c = -4.0 - 0.67 log10 Fcent. It is the default everywhere.
CONV_KC_UNIT_SLIP = 1
CONV_FALLOFF_XM = 2
CONV_DOC_COVG = 4
CONV_TROE_C4 = 16
CONV_REFERENCE = CONV_KC_UNIT_SLIP | CONV_FALLOFF_XM | CONV_TROE_C4


class MechanismError(ValueError):
    pass


# --------------------------------------------------------------------------------------
# NASA-7 thermo
# --------------------------------------------------------------------------------------
@dataclass
class SpeciesThermo:
    name: str
    elements: dict
    tlow: float
    thigh: float
    tmid: float
    hi: np.ndarray
    lo: np.ndarray

    @property
    def molwt(self) -> float:
        w = 0.0
        for e, c in self.elements.items():
            if e not in ATOMIC_WEIGHTS:
                raise MechanismError(f"unknown element {e} in {self.name}")
            w += c * ATOMIC_WEIGHTS[e]
        return w * 1e-3


def _f(s: str) -> float:
    s = s.strip().replace("D", "E").replace("d", "e")
    return float(s) if s else 0.0


def read_therm(path: str) -> dict:
    """Fixed-column NASA-7 reader (therm.dat, CHEMKIN-II format)."""
    lines = [l.rstrip("\r\n") for l in open(path, encoding="latin-1")]
    out = {}
    i = 0
    while i + 3 < len(lines):
        l1 = lines[i]
        if len(l1) >= 80 and l1[79] == "1" and not l1.startswith("!"):
            l2, l3, l4 = lines[i + 1], lines[i + 2], lines[i + 3]
            name = l1[:18].split()[0].upper()
            el = {}
            for k in range(4):
                sym = l1[24 + 5 * k:26 + 5 * k].strip().upper()
                cnt = l1[26 + 5 * k:29 + 5 * k].strip()
                if sym and sym != "0" and cnt and float(cnt) != 0:
                    el[sym] = el.get(sym, 0) + int(float(cnt))
            tlow, thigh = _f(l1[45:55]), _f(l1[55:65])
            tmid = _f(l1[65:73]) or 1000.0
            c = [_f(l2[15 * k:15 * k + 15]) for k in range(5)]
            c += [_f(l3[15 * k:15 * k + 15]) for k in range(5)]
            c += [_f(l4[15 * k:15 * k + 15]) for k in range(4)]
            out[name] = SpeciesThermo(name, el, tlow, thigh, tmid, np.array(c[:7]), np.array(c[7:14]))
            i += 4
            continue
        i += 1
    return out


# --------------------------------------------------------------------------------------
# CHEMKIN-II gas mechanism
# --------------------------------------------------------------------------------------
@dataclass
class GasReaction:
    equation: str
    reactants: list          # expanded species names
    products: list
    reversible: bool
    third_body: int          # 0 none, 1 +M, 2 (+M) falloff
    A: float                 # SI
    beta: float
    EoR: float               # K
    low: tuple = None        # (A0 SI, beta0, E0/R)
    troe: tuple = None       # (a, T3, T1[, T2])
    efficiencies: dict = field(default_factory=dict)


_EUNITS = {"CAL/MOLE": CAL / R_GAS, "KCAL/MOLE": 1000.0 * CAL / R_GAS, "JOULES/MOLE": 1.0 / R_GAS,
           "KJOULES/MOLE": 1000.0 / R_GAS, "KELVINS": 1.0}


def _side(text: str, species: set):
    out, has_m = [], False
    for term in text.split("+"):
        term = term.strip()
        if not term:
            continue
        m = re.match(r"^(\d+)(.*)$", term)
        coef, name = (int(m.group(1)), m.group(2)) if m else (1, term)
        if name == "M":
            has_m = True
            continue
        if name not in species:
            raise MechanismError(f"unknown species '{name}'")
        out += [name] * coef
    return out, has_m


def read_chemkin(path: str):
    """Returns (species list, [GasReaction])."""
    species, rxns = [], []
    section, efac = None, CAL / R_GAS
    for raw in open(path, encoding="latin-1"):
        line = raw.split("!", 1)[0].strip().upper()
        if not line:
            continue
        word = line.split()[0]
        if word.startswith("ELEM"):
            section = "E"
            continue
        if word.startswith("SPEC"):
            section = "S"
            line = line[len(word):].strip()
            if not line:
                continue
        elif word.startswith("THERMO"):
            section = "T"
            continue
        elif word.startswith("REAC"):
            section = "R"
            for key, f in _EUNITS.items():
                if key in line.split():
                    efac = f
            continue
        if word == "END":
            section = None
            continue
        if section == "S":
            for tok in line.split():
                if tok == "END":
                    section = None
                    break
                if tok not in species:
                    species.append(tok)
        elif section == "R":
            if "=" in line:
                toks = line.split()
                A, b, E = float(toks[-3]), float(toks[-2]), float(toks[-1])
                eq = "".join(toks[:-3])
                falloff = "(+M)" in eq
                eq2 = eq.replace("(+M)", "")
                if "<=>" in eq2:
                    lhs, rhs, rev = *eq2.split("<=>"), True
                elif "=>" in eq2:
                    lhs, rhs, rev = *eq2.split("=>"), False
                else:
                    lhs, rhs, rev = *eq2.split("="), True
                sset = set(species)
                re_, m1 = _side(lhs, sset)
                pr_, m2 = _side(rhs, sset)
                tb = 2 if falloff else (1 if (m1 or m2) else 0)
                order = len(re_) + (1 if tb == 1 else 0)
                rxns.append(GasReaction(eq, re_, pr_, rev, tb, A * 1e-6 ** (order - 1), b, E * efac))
            else:
                if not rxns:
                    continue
                r = rxns[-1]
                if line.startswith("DUP"):
                    continue
                parts = [p.strip() for p in line.split("/")]
                i = 0
                while i + 1 < len(parts):
                    key, val = parts[i], parts[i + 1]
                    if not key:
                        i += 1
                        continue
                    if key == "LOW":
                        a0, b0, e0 = (float(v) for v in val.split())
                        r.low = (a0 * 1e-6 ** len(r.reactants), b0, e0 * efac)
                    elif key == "TROE":
                        r.troe = tuple(float(v) for v in val.split())
                    elif key in ("REV", "SRI", "PLOG", "FORD", "RORD", "HIGH"):
                        raise MechanismError(f"unsupported auxiliary keyword {key}")
                    elif key in species:
                        r.efficiencies[key] = float(val)
                    i += 2
    return species, rxns


# --------------------------------------------------------------------------------------
# surface mechanism XML (ch4ni.xml)
# --------------------------------------------------------------------------------------
@dataclass
class SurfReaction:
    equation: str
    reactants: list          # names (gas or surface), upper case
    products: list
    stick: bool
    A: float                 # SI (arrhenius) or s0
    beta: float
    Ea: float                # J/mol
    coverage: dict = field(default_factory=dict)   # surface species -> eps (J/mol)
    rid: int = -1


def _kv_list(text: str):
    out = {}
    for item in text.split(","):
        if "=" in item:
            k, v = item.split("=", 1)
            out[k.strip().upper()] = float(v)
    return out


def read_surface_xml(path: str, gas_species: list):
    root = ET.parse(path).getroot()
    unit = (root.get("unit") or "kJ/mol").lower()
    efac = {"kj/mol": 1000.0, "j/mol": 1.0, "kcal/mol": 4184.0, "cal/mol": CAL}.get(unit, 1000.0)
    surf = [s.upper() for s in root.findtext("species").split()]
    site = root.find("site")
    sigma = {s: 1.0 for s in surf}
    theta0 = {s: 0.0 for s in surf}
    density = 0.0
    if site is not None:
        if site.findtext("coordination"):
            for k, v in _kv_list(site.findtext("coordination")).items():
                if k in sigma:
                    sigma[k] = v
        density = float(site.findtext("density"))
        if site.findtext("initial"):
            for k, v in _kv_list(site.findtext("initial")).items():
                if k in theta0:
                    theta0[k] = v
    gas_u = [g.upper() for g in gas_species]
    known = set(surf) | set(gas_u)

    def side(text):
        out = []
        for t in text.split("+"):
            t = t.strip().upper()
            if not t:
                continue
            m = re.match(r"^(\d+)\s*(.*)$", t)
            c, nm = (int(m.group(1)), m.group(2).strip()) if m else (1, t)
            if nm not in known:
                raise MechanismError(f"unknown surface-reaction species '{nm}'")
            out += [nm] * c
        return out

    rxns = []
    for kind in ("stick", "arrhenius"):
        blk = root.find(kind)
        if blk is None:
            continue
        for rx in blk.findall("rxn"):
            eq, params = rx.text.split("@")
            lhs, rhs = eq.split("=>")
            re_, pr_ = side(lhs), side(rhs)
            vals = [float(v) for v in params.split()]
            if kind == "stick":
                r = SurfReaction(eq.strip(), re_, pr_, True, vals[0], 0.0, 0.0)
            else:
                ms = sum(1 for s in re_ if s in sigma)
                mg = len(re_) - ms
                r = SurfReaction(eq.strip(), re_, pr_, False, vals[0] * 1e-4 ** (ms - 1) * 1e-6 ** mg,
                                 vals[1], vals[2] * efac)
            r.rid = int(rx.get("id", "-1"))
            rxns.append(r)
    byid = {r.rid: r for r in rxns}
    for cov in root.findall("coverage"):
        for k, v in _kv_list(cov.text).items():
            for rid in cov.get("id").split():
                byid[int(rid)].coverage[k] = v * efac
    return surf, sigma, density, theta0, rxns


# --------------------------------------------------------------------------------------
# batch.xml (input_data, src/BatchReactor.jl:238-306)
# --------------------------------------------------------------------------------------
def read_batch_xml(path: str) -> dict:
    root = ET.parse(path).getroot()
    d = {}
    for tag in ("gas_mech", "surface_mech"):
        if root.findtext(tag):
            d[tag] = root.findtext(tag).strip()
    if root.findtext("gasphase"):
        d["gasphase"] = root.findtext("gasphase").split()
    for tag in ("T", "p", "Asv", "time"):
        if root.findtext(tag) is not None:
            d[tag] = float(root.findtext(tag))
    for tag in ("molefractions", "massfractions"):
        if root.findtext(tag):
            d[tag] = _kv_list(root.findtext(tag))
    return d


def get_path(lib_dir: str, name: str) -> str:
    return os.path.join(lib_dir, name)


# --------------------------------------------------------------------------------------
# compiled mechanism -> br_mech_desc arrays
# --------------------------------------------------------------------------------------
class Mechanism:
    """Gas and/or surface mechanism compiled into the flat SI tables of br_mech_desc."""

    def __init__(self, gas_species, thermo, gas_rxns=(), surf=None, conv=CONV_REFERENCE, p_std=1e5):
        self.gas_species = [g.upper() for g in gas_species]
        self.ng = len(self.gas_species)
        self.thermo = thermo
        self.conv = conv
        self.p_std = p_std
        missing = [s for s in self.gas_species if s not in thermo]
        if missing:
            raise MechanismError(f"species not in therm.dat: {missing}")
        self.molwt = np.array([thermo[s].molwt for s in self.gas_species])
        nasa = np.zeros((self.ng, 15))
        for k, s in enumerate(self.gas_species):
            t = thermo[s]
            nasa[k, 0] = t.tmid
            nasa[k, 1:8] = t.hi
            nasa[k, 8:15] = t.lo
        self.nasa = nasa
        self.gas_rxns = list(gas_rxns)
        if surf is not None:
            self.surf_species, sig, self.site_density, th0, self.surf_rxns = surf
            self.sigma = np.array([sig[s] for s in self.surf_species])
            self.theta0 = np.array([th0[s] for s in self.surf_species])
        else:
            self.surf_species, self.site_density, self.surf_rxns = [], 0.0, []
            self.sigma = np.zeros(0)
            self.theta0 = np.zeros(0)
        self.ns = len(self.surf_species)
        self.n = self.ng + self.ns
        self.species = self.gas_species + self.surf_species
        self._flatten()

    @classmethod
    def from_files(cls, lib_dir, gas_mech=None, surface_mech=None, gasphase=None, conv=CONV_REFERENCE,
                   p_std=1e5):
        thermo = read_therm(get_path(lib_dir, "therm.dat"))
        rxns = []
        if gas_mech:
            species, rxns = read_chemkin(get_path(lib_dir, gas_mech))
        else:
            species = [g.upper() for g in gasphase]
        surf = read_surface_xml(get_path(lib_dir, surface_mech), species) if surface_mech else None
        return cls(species, thermo, rxns, surf, conv, p_std)

    def index(self, name):
        return self.species.index(name.upper())

    def _flatten(self):
        ng, ns = self.ng, self.ns
        gi = {s: k for k, s in enumerate(self.gas_species)}
        ci = {s: k for k, s in enumerate(self.species)}
        nrg, nrs = len(self.gas_rxns), len(self.surf_rxns)
        self.nrg, self.nrs = nrg, nrs
        g_nf = np.zeros(nrg, np.int32); g_nr = np.zeros(nrg, np.int32)
        g_f = -np.ones((nrg, 4), np.int32); g_r = -np.ones((nrg, 4), np.int32)
        g_rev = np.zeros(nrg, np.int32); g_tb = np.zeros(nrg, np.int32)
        g_arr = np.zeros((nrg, 3)); g_low = np.zeros((nrg, 3))
        g_troe_n = np.zeros(nrg, np.int32); g_troe = np.zeros((nrg, 4))
        g_eff = np.ones((nrg, ng))
        for i, r in enumerate(self.gas_rxns):
            if len(r.reactants) > 4 or len(r.products) > 4:
                raise MechanismError(f"reaction {r.equation}: more than 4 entries per side")
            g_nf[i], g_nr[i] = len(r.reactants), len(r.products)
            g_f[i, :g_nf[i]] = [gi[s] for s in r.reactants]
            g_r[i, :g_nr[i]] = [gi[s] for s in r.products]
            g_rev[i] = int(r.reversible)
            g_tb[i] = r.third_body
            g_arr[i] = (r.A, r.beta, r.EoR)
            if r.low is not None:
                g_low[i] = r.low
            if r.troe is not None:
                g_troe_n[i] = len(r.troe)
                g_troe[i, :len(r.troe)] = r.troe
            for s, e in r.efficiencies.items():
                g_eff[i, gi[s]] = e
            if r.third_body == 2 and r.low is None:
                raise MechanismError(f"falloff reaction {r.equation} without LOW")
        s_nf = np.zeros(nrs, np.int32); s_np = np.zeros(nrs, np.int32)
        s_f = -np.ones((nrs, 6), np.int32); s_p = -np.ones((nrs, 6), np.int32)
        s_stick = np.zeros(nrs, np.int32); s_arr = np.zeros((nrs, 3))
        s_ncov = np.zeros(nrs, np.int32); s_cov_sp = np.zeros((nrs, 4), np.int32); s_cov_eps = np.zeros((nrs, 4))
        for i, r in enumerate(self.surf_rxns):
            s_nf[i], s_np[i] = len(r.reactants), len(r.products)
            s_f[i, :s_nf[i]] = [ci[s] for s in r.reactants]
            s_p[i, :s_np[i]] = [ci[s] for s in r.products]
            s_stick[i] = int(r.stick)
            s_arr[i] = (r.A, r.beta, r.Ea)
            s_ncov[i] = len(r.coverage)
            for j, (s, e) in enumerate(r.coverage.items()):
                s_cov_sp[i, j] = ci[s]
                s_cov_eps[i, j] = e
        self.tables = dict(g_nf=g_nf, g_nr=g_nr, g_f=g_f, g_r=g_r, g_rev=g_rev, g_tb=g_tb, g_arr=g_arr,
                           g_low=g_low, g_troe_n=g_troe_n, g_troe=g_troe, g_eff=g_eff, s_nf=s_nf, s_np=s_np,
                           s_f=s_f, s_p=s_p, s_stick=s_stick, s_arr=s_arr, s_ncov=s_ncov, s_cov_sp=s_cov_sp,
                           s_cov_eps=s_cov_eps)

    # ---- composition helpers (IdealGas equivalents) ----
    def mole_fractions(self, comp: dict) -> np.ndarray:
        x = np.zeros(self.ng)
        for k, v in comp.items():
            if k.upper() in self.gas_species:
                x[self.gas_species.index(k.upper())] = v
        return x

    def initial_state(self, T, p, x, theta=None) -> np.ndarray:
        """u0 = [rho*Y_k ; theta] (get_solution_vector, src/BatchReactor.jl:224-232)."""
        x = np.asarray(x, float)
        Mb = float(np.sum(x * self.molwt))
        rho = p * Mb / (R_GAS * T)
        u = np.empty(self.n)
        u[:self.ng] = (x * self.molwt / Mb) * rho
        u[self.ng:] = self.theta0 if theta is None else theta
        return u

    def state_to_molefrac(self, u) -> np.ndarray:
        """Final conversion Y = u/sum(u) -> x (src/BatchReactor.jl:142-144)."""
        u = np.asarray(u, float)
        y = u[..., :self.ng] / np.sum(u[..., :self.ng], axis=-1, keepdims=True)
        t = y / self.molwt
        return t / np.sum(t, axis=-1, keepdims=True)
