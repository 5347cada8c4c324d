"""Lane-level numpy emulation of lu_factor_mf (brhip_device.hpp) + a plain solve, for checking the
index logic of the blocked MFMA LU on the CPU (diagnostic tool; not test infrastructure).
Mirrors the C++ statement by statement: 64-lane vectors, raw-buffer range checks, the
v_mfma_f64_16x16x4f64 operand layouts (A: m = lane & 15, k = lane >> 4; B: k = lane >> 4,
n = lane & 15; C/D: n = lane & 15, m = (lane >> 4) + 4 i)."""
import numpy as np

L = np.arange(64)
OOB = None


def mfma(a, b, c):
    A = np.zeros((16, 4)); B = np.zeros((4, 16))
    A[L & 15, L >> 4] = a
    B[L >> 4, L & 15] = b
    D = np.zeros((16, 16))
    for i in range(4):
        D[(L >> 4) + 4 * i, L & 15] = c[i]
    D = D + A @ B
    return [D[(L >> 4) + 4 * i, L & 15].copy() for i in range(4)]


def bload(mem, lim, off):
    """raw buffer load: off (per lane, doubles) or None (OOB) -> 0 when out of [0, lim)"""
    out = np.zeros(64)
    for l in range(64):
        o = off[l]
        if o is not None and 0 <= o < lim:
            out[l] = mem[o]
    return out


def bstore(mem, lim, off, v):
    for l in range(64):
        o = off[l]
        if o is not None and 0 <= o < lim:
            mem[o] = v[l]


def pivot_lane(a, cand, prow):
    idx = [l for l in range(64) if cand[l]]
    if not idx:
        return 0
    best = max(abs(a[l]) for l in idx)
    c = [l for l in idx if abs(a[l]) == best]
    return min(c, key=lambda l: prow[l])


def lu_factor_mf(J, F, Dv, gamma, n, prow_in, NMAX, PW, stop=1 << 20):
    """J: column-major 64 rows per column (J[col*64 + row]); F: NMAX*NMAX factor matrix (col-major,
    FR = NMAX rows); Dv: 64 doubles. prow_in[lane]: original row of lane. Returns fail, perm."""
    FR = NMAX
    KS = PW // 4
    NRT = (NMAX + 15) // 16
    MAXCT = (NMAX - PW + 15) // 16
    g, m = L >> 4, L & 15
    act = L < n
    prow = prow_in.copy()
    pstep = np.where(act, -1, 1024)
    dinv = np.zeros(64)
    fail = 0
    np_ = (n + PW - 1) // PW
    fo = [l if l < FR else None for l in range(64)]
    Jlim = n * 64
    Flim = NMAX * FR
    Fnlim = n * FR
    scr = np.zeros(256)

    def panel(a, e, piv, c0, nlive, with_e):
        nonlocal fail, pstep, dinv
        for kk in range(PW):
            if kk >= nlive:
                continue
            k = c0 + kk
            cand = pstep < 0
            p = pivot_lane(a[kk], cand, prow)
            piv[kk] = p
            pv = a[kk][p]
            if pv == 0.0 and not fail:
                fail = k + 1
            rinv = 1.0 / pv
            isp = L == p
            rem = cand & ~isp
            l = np.where(rem, a[kk] * rinv, 0.0)
            fv = np.where(rem, l, np.where(cand, 0.0, a[kk] * dinv))
            bstore(F, Flim, [None if fo[x] is None else k * FR + fo[x] for x in range(64)], fv)
            pstep = np.where(isp, k, pstep)
            dinv = np.where(isp, rinv, dinv)
            if with_e:
                for j in range(kk):
                    e[j] = e[j] - e[j][p] * l
                e[kk] = -l
            for j in range(kk + 1, PW):
                if j < nlive:
                    a[j] = a[j] - a[j][p] * l

    for p in range(np_ - 1):
        c0 = PW * p
        live = pstep < 0
        e = [np.zeros(64) for _ in range(PW)]
        piv = [0] * PW
        if p == 0:
            a = [np.where(L < n, (np.arange(64) == 0) * 0.0, 0.0) for _ in range(PW)]
            for j in range(PW):
                jv = bload(J, Jlim, [prow[l] + j * 64 if act[l] else None for l in range(64)])
                a[j] = np.where(j == prow, 1.0, 0.0) - gamma * jv
        else:
            a = [bload(F, Flim, [None if fo[l] is None else (c0 + j) * FR + l for l in range(64)]) for j in range(PW)]
        panel(a, e, piv, c0, PW, True)
        bo = [[None] * KS for _ in range(NRT)]
        for s in range(KS):
            for q in range(4):
                scr[4 * L + q] = e[4 * s + q]
            for t in range(NRT):
                bo[t][s] = scr[4 * (16 * t + m) + g].copy()
        aor = [None] * KS
        ao8 = [None] * KS
        for s in range(KS):
            pr = np.array([piv[4 * s + gg] for gg in g])
            if p == 0:
                aor[s] = prow[pr]
                ao8[s] = aor[s] + m * 64
            else:
                ao8[s] = m * FR + pr
        orow = [None] * NRT
        jt = [None] * NRT
        if p == 0:
            for t in range(NRT):
                orow[t] = np.where(act[16 * t + m], prow[16 * t + m], -1)
                jt[t] = [orow[t][l] + g[l] * 64 if orow[t][l] >= 0 else None for l in range(64)]
        rb = [[(g[l] * FR + 16 * t + m[l]) if 16 * t + m[l] < FR else None for l in range(64)] for t in range(NRT)]
        cs = c0 + PW
        for ct in range(MAXCT):
            cb = cs + 16 * ct
            if cb >= n:
                continue
            ao = [None] * KS
            for s in range(KS):
                if p == 0:
                    jv = bload(J, Jlim, list(ao8[s] + cb * 64))
                    ao[s] = np.where(aor[s] == cb + m, 1.0, 0.0) - gamma * jv
                else:
                    ao[s] = bload(F, Fnlim, list(ao8[s] + cb * FR))
            x = [None] * NRT
            for t in range(NRT):
                if not live[16 * t:16 * t + 16].any():
                    continue
                x[t] = [np.zeros(64) for _ in range(4)]
                for i in range(4):
                    cc = cb + 4 * i
                    if cc < NMAX:
                        if p == 0:
                            jv = bload(J, Jlim, [None if jt[t][l] is None else jt[t][l] + cc * 64 for l in range(64)])
                            x[t][i] = np.where(orow[t] == cc + g, 1.0, 0.0) - gamma * jv
                        else:
                            x[t][i] = bload(F, Flim, [None if rb[t][l] is None else rb[t][l] + cc * FR for l in range(64)])
            for t in range(NRT):
                if x[t] is None:
                    continue
                for s in range(KS):
                    x[t] = mfma(ao[s], bo[t][s], x[t])
                for i in range(4):
                    cc = cb + 4 * i
                    if cc < NMAX:
                        bstore(F, Flim, [None if rb[t][l] is None else rb[t][l] + cc * FR for l in range(64)], x[t][i])
        if p == stop:
            return 0, prow
    c0 = PW * (np_ - 1)
    nlive = n - c0
    e = [np.zeros(64) for _ in range(PW)]
    piv = [0] * PW
    if np_ == 1:
        a = [np.where(j == prow, 1.0, 0.0) - gamma * bload(J, Jlim, [prow[l] + j * 64 if act[l] else None for l in range(64)]) for j in range(PW)]
    else:
        a = [bload(F, Flim, [None if fo[l] is None else (c0 + j) * FR + l for l in range(64)]) if j < nlive else np.zeros(64)
             for j in range(PW)]
    panel(a, e, piv, c0, nlive, False)
    # gather into step order
    if not np.any(act & (pstep != L)):
        perm = prow.copy()
        for c in range(n, NMAX):
            F[c * FR:(c + 1) * FR] = 0.0
        Dv[:] = dinv
    else:
        q = np.array([int(np.where(pstep == s)[0][0]) if s < n else s for s in range(64)])
        perm = prow[q]
        Fc = F.copy()
        for c in range(NMAX):
            for l in range(FR):
                F[c * FR + l] = Fc[min(c, n - 1) * FR + min(q[l], FR - 1)] if c < n else 0.0
        Dv[:] = dinv[q]
    return fail, perm


def solve(F, Dv, n, NMAX, perm, b):
    FR = NMAX
    M = F.reshape(NMAX, FR).T   # M[row][col]
    y = np.zeros(64)
    y[:n] = b[perm[:n]]
    for k in range(n):
        for s in range(k + 1, n):
            y[s] -= M[s, k] * y[k]
    y[:n] *= Dv[:n]
    for k in range(n - 1, -1, -1):
        for s in range(k):
            y[s] -= M[s, k] * y[k]
    x = np.zeros(n)
    x[:n] = y[:n]
    return x


def check(n, NMAX, PW, seed=None, N=4):
    rng = np.random.default_rng(n if seed is None else seed)
    worst = 0.0
    for i in range(N):
        Jm = rng.standard_normal((n, n)) * np.exp(rng.uniform(-8, 8, (n, 1)))
        gamma = np.exp(rng.uniform(-12, -2))
        b = rng.standard_normal(n)
        Jt = np.zeros(NMAX * 64)
        for j in range(n):
            Jt[j * 64:j * 64 + n] = Jm[:, j]
        F = np.full(NMAX * NMAX, np.nan)
        Dv = np.zeros(64)
        prow = L.copy()
        f, perm = lu_factor_mf(Jt, F, Dv, gamma, n, prow, NMAX, PW)
        f2, perm2 = lu_factor_mf(Jt, F, Dv, gamma, n, perm, NMAX, PW)
        x = solve(F, Dv, n, NMAX, perm2, b)
        A = np.eye(n) - gamma * Jm
        res = np.max(np.abs(A @ x - b)) / (np.abs(A).sum(1).max() * np.abs(x).max() + np.abs(b).max())
        worst = max(worst, res)
    return worst


if __name__ == "__main__":
    for n, NMAX in ((53, 56), (40, 56), (64, 64), (33, 56)):
        for PW in (8, 16):
            print(n, NMAX, PW, check(n, NMAX, PW))
