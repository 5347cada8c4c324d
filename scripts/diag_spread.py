"""Run-to-run spread of CVODE itself (oracle vs oracle with u0 perturbed by 1e-15 relative), in the
units and bands of tests/test_gpu_parity.py::test_integrate_parity. Usage: diag_spread.py CASE N ANALYTIC(0/1)"""
import sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')]
import _pkgload, oracle as orc
pkg=_pkgload.load()
from batchreactor_amd import ensemble
from parity_bands import OUT_T, band_errors as _band_errors
LIB=os.path.join(ROOT, 'tests', 'golden', 'lib')
case=sys.argv[1]; N=int(sys.argv[2]); aj=int(sys.argv[3])
# ORC_ROP_JITTER=<eps>: the perturbed run also evaluates every rate of progress with a relative +-eps
# (an RHS implementation that rounds differently; what CVODE's DQ Jacobian is most sensitive to)
ROPJ=float(os.environ.get('ORC_ROP_JITTER','0'))
gas={'h2o2':'h2o2.dat','gri':'grimech.dat','gas_surf':'grimech.dat','surf':None}[case]
surf='ch4ni.xml' if case in ('gas_surf','surf') else None
SG="CH4 H2O H2 CO CO2 O2 N2".split()
pm=pkg.Mechanism.from_files(LIB,gas_mech=gas,surface_mech=surf,gasphase=None if gas else SG)
om=orc.Mech(LIB+'/'+gas if gas else None,LIB+'/therm.dat',LIB+'/'+surf if surf else None,gas_species=None if gas else SG)
T,Asv,U0=ensemble.make_inputs(pm,case,0,N)
rng=np.random.default_rng(0)
W=[];S=[];dti=[];nfail=0
for i in range(N):
    ua,sa,Ya=om.integrate_out(T[i],Asv[i],U0[i],10.0,OUT_T,analytic_jac=bool(aj))
    up=U0[i]*(1+1e-15*rng.standard_normal(len(U0[i])))
    orc.lib().orc_set_rop_jitter(ROPJ)
    ub,sb,Yb=om.integrate_out(T[i],Asv[i],up,10.0,OUT_T,analytic_jac=bool(aj))
    orc.lib().orc_set_rop_jitter(0.0)
    if sa['status'] != 0 or sb['status'] != 0:   # a CVODE failure in one run (rounding-chaotic: C5 -3)
        nfail += 1
        continue
    W.append(_band_errors(Yb,Ya,sa['t_ign'])); S.append(sb['nsteps']/sa['nsteps']-1)
    if sa['t_ign']==sa['t_ign']: dti.append(abs(sb['t_ign']-sa['t_ign'])/max(sa['ign_dt'],sb['ign_dt']))
W=np.array(W); S=np.array(S)
print(case,'aj',aj,'band max',W.max(0),'p99',np.percentile(W,99,axis=0),'steps rel max',np.abs(S).max(),'p90',np.percentile(np.abs(S),90),'sum',S.mean(),'tign/dt max',max(dti) if dti else None,'failed pairs',nfail)
import json
print('JSON', json.dumps({'case': case, 'analytic_jac': bool(aj), 'reactors': N, 'rop_jitter': ROPJ, 'dq_inc_jitter': float(os.environ.get('ORC_DQ_JITTER','0')), 'excluded_failed_pairs': nfail,
                          'band_max': W.max(0).tolist(), 'band_p99': np.percentile(W, 99, axis=0).tolist(),
                          'steps_rel_max': float(np.abs(S).max()), 'steps_rel_p90': float(np.percentile(np.abs(S), 90)),
                          'tign_over_dt_max': float(max(dti)) if dti else None}))
# with ORC_DQ_JITTER=<eps> in the environment the perturbed run also perturbs the DQ increments:
#   ORC_DQ_JITTER=1e-15 python scripts/diag_spread.py h2o2 256 0
