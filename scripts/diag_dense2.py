import os, sys, numpy as np
ROOT='/root/repo'; sys.path.insert(0, ROOT)
import _pkgload
pkg = _pkgload.load()
from batchreactor_amd import ensemble
LIB = os.path.join(ROOT, "tests", "golden", "lib")
for gas in ("grimech.dat","h2o2.dat"):
    pm = pkg.Mechanism.from_files(LIB, gas_mech=gas)
    eng = pkg.Engine(pm)
    T, Asv, U0 = ensemble.make_inputs(pm, "gri" if gas=="grimech.dat" else "h2o2", 0, 2)
    tout = np.array([5.0, 9.99, 10.0])
    for ign in (eng.ign1, 0):
        eng.ign1 = ign
        for tf in (10.0, 9.995):
            U, st = eng.integrate(T, Asv, U0, tf, tout=tout)
            print(gas, 'ign', ign, 'tf', tf, 'row sums', np.abs(st['yout']).sum(2).round(4).tolist(), 't_end', st['t_end'], 'nsteps', st['nsteps'])
