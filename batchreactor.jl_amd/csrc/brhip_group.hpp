// brhip_group.hpp -- GROUP ENGINES: two or four reactors per wave for small mechanisms. A reactor
// occupies a group of GL lanes (GL = 16: one DPP row, n <= 16, "quad", e.g. H2/O2 n = 9, the C2
// ensemble; GL = 32: one half-wave, 16 < n <= 32, "pair", e.g. the surface-only Ni/CH4 case, n = 20,
// C4), lane gl of the group holds component gl. Included by brhip.hip after the controller: the same
// CVODE 5.x restatement (begin_step / ctl_post_rhs / ctl_post_solve, src/BatchReactor.jl:138-141,
// :210) runs with the controller instantiated for GL-lane groups (GW = GL).
//
// Why: one reactor per wave leaves most lanes idle for small n in every per-component operation
// and pays the step controller (~1k instructions) per reactor; one reactor per lane (k_lane) keeps
// a reactor's whole state in one lane's registers (436 registers, 1 wave/SIMD, spills, 2.6 MB of
// memory traffic per H2/O2 reactor) and runs every controller branch of 64 diverging reactors. Here
// the controller serves 2 or 4 reactors per instruction (2- or 4-way divergence at most), group
// reductions are DPP row butterflies (plus one permlane16 swap for 32-lane groups), the LU factors
// live in registers (one row per lane) and the solve needs no memory.
//
// Per reactor (LDS): [Ctl | V: NVEC x GL doubles | species block (GLay) | kd: {kf, kr} per gas
// reaction | fod: {k0/kinf, log10 Fcent, c, n} per falloff reaction | skd: k(T) per surface
// reaction]. Global: the saved Jacobian, GL x GL column-major per group slot. Mechanism tables as for
// the wavefront engine (LDS image, records with the pad species 64 = conc 1.0).
// kd lives in the group's global slot after its saved Jacobian (L2-resident: a few hundred bytes per
// group), and a gas-only 16-lane species block drops its surface sums (66 doubles instead of 82):
// 2.38 instead of 2.83 KB of LDS per H2/O2 reactor, so four 16-reactor workgroups (16 waves) fit a
// CU's 160 KB instead of three (round 5: C2 +11 %; kd in LDS was the round-4 layout).
#pragma once

namespace grp {
// species block of a group (doubles): conc[CONC + k], gas production sums ACCW, surface production
// sums ACCS, third-body sums MC (<= 32 efficiency sets), conc[ONE] = 1.0 (the records' pad species
// Lay<1>::ONE = 64, so conc + 64 must land on it)
template <int GL>
struct GLay {
    static constexpr int CONC = 0, ACCW = GL, ONE = 64, ACCS = 66;
    static constexpr int MC = GL == 16 ? 32 : 98;
    static constexpr int DOUBLES = GL == 16 ? 82 : 130;
    static_assert(GL == 16 || GL == 32, "group width");
    static_assert(ONE == Lay<1>::ONE, "pad species");
};
constexpr int MAX_SETS = 32;
// (Nordsieck / work vectors NM wide instead of GL measured 1.078M vs 1.096M reactors/s, round 5,
// profiles/r05_h2o2_quad_wpe_ab.json; not kept)
__host__ __device__ constexpr int vstride(int gl, int nm) { return nm > 0 ? gl : gl; }
__host__ __device__ inline int vbytes(int gl, int nm) { return NVEC * vstride(gl, nm) * 8; }
__host__ __device__ inline int sp_off(int gl, int nm) { return CTL_BYTES + vbytes(gl, nm); }
// species-block doubles: gas-only 16-lane groups need no surface sums (ACCS) past ONE = 64
__host__ __device__ inline int sp_doubles(int gl, int nrs) {
    return gl == 16 ? (nrs == 0 ? 66 : GLay<16>::DOUBLES) : GLay<32>::DOUBLES;
}
__host__ __device__ inline int fod_off(int gl, int nm, int nrg, int nrs) { (void)nrg; return sp_off(gl, nm) + sp_doubles(gl, nrs) * 8; }
__host__ __device__ inline int block_bytes(int gl, int nm, int nrg, int nfo, int nrs) {
    const int b = fod_off(gl, nm, nrg, nrs) + 32 * nfo + 8 * nrs;
    return (b + 15) / 16 * 16;
}
// global doubles per group slot: the saved Jacobian (GL x GL), then kd (64-B aligned; at least 8: the
// RHS prefetches the pair of reaction 0 even when there are no gas reactions)
__host__ __device__ inline int slot_doubles(int gl, int nrg) { return gl * gl + ((2 * nrg + 7) / 8 * 8 > 8 ? (2 * nrg + 7) / 8 * 8 : 8); }
}  // namespace grp
typedef BR_GLOBAL double QKd;   // {kf, kr} pairs: the group slot in global memory

// max of a 32-bit value over each 16-lane DPP row (every lane gets its row's max)
__device__ __forceinline__ unsigned row_umax(unsigned x) {
    unsigned r;
    asm volatile(
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_max_u32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1"
        : "=&v"(r)
        : "v"(x));
    return r;
}
// ... over each group (32-lane groups: the two row maxima exchanged by a permlane16 swap)
template <int GL>
__device__ __forceinline__ unsigned group_umax(unsigned x) {
    const unsigned m = row_umax(x);
    if constexpr (GL == 16) return m;
    else {
        const auto p = __builtin_amdgcn_permlane16_swap(m, m, false, false);
        return max((unsigned)p[0], (unsigned)p[1]);
    }
}

// compile-time loop: f(std::integral_constant<int, K>) for K = B .. E-1
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}
// value of lane K of this lane's 16-lane row (DPP row_newbcast: a VALU move, no LDS crossbar)
template <int K>
__device__ __forceinline__ double row_bcast(double v) { return dppd<0x150 + K>(v); }
// value of lane K (compile time) of this lane's group: the row broadcast, and for 32-lane groups the
// row holding lane K through a permlane16 swap
template <int GL, int K>
__device__ __forceinline__ double group_bcast(double v) {
    const double r = row_bcast<K & 15>(v);
    if constexpr (GL == 16) return r;
    else {
        const RowPair p = row_pair(r);
        return K < 16 ? p.even : p.odd;
    }
}

// T-only constants of one group's reactor (init_tconst for the group layout): {kf, kr} per gas
// reaction into kd, falloff constants into fod, k(T) per surface reaction into skd; g/RT per gas
// species in the ACCW slots (scratch)
template <int GL>
__device__ __forceinline__ void g_init_tconst(const Tab& tb, double* sp, QKd* kd, double* fod, double* skd, double T,
                                              int gl) {
    typedef grp::GLay<GL> L;
    const double lT = log(T);
    double* grt = sp + L::ACCW;
    const int ng = MF(ng), nrg = MF(nrg), nrs = MF(nrs);
    if (gl == 0) sp[L::ONE] = 1.0;
    if (gl < ng) {
        const double* c = MF(nasa) + 15 * gl;
        const double* a = (T < c[0]) ? c + 8 : c + 1;
        const double h = a[0] + a[1] * T / 2 + a[2] * T * T / 3 + a[3] * T * T * T / 4 + a[4] * T * T * T * T / 5 + a[5] / T;
        const double s = a[0] * lT + a[1] * T + a[2] * T * T / 2 + a[3] * T * T * T / 3 + a[4] * T * T * T * T / 4 + a[6];
        grt[gl] = h - s;
    }
    wave_sync();
    const double RT = R_GAS * T;
#pragma unroll 1
    for (int r = gl; r < nrg; r += GL) {
        const auto rec = rx_rec(tb.rx, r);
        const uint32_t info = rec[2];
        const double* gp = MF(g_par) + 4 * r;
        const double kf = gp[0] * exp(gp[1] * lT - gp[2] / T);
        double kr = 0.0;
        if (gi_rev(info)) {
            double dg = 0.0;
            const int nf = gi_nf(info), nr = gi_nr(info);
            for (int e = 0; e < 4; ++e) if (e < nr) dg += grt[sp8(rec[1], e)];
            for (int e = 0; e < 4; ++e) if (e < nf) dg -= grt[sp8(rec[0], e)];
            double Kc = exp(-dg) * pow(MF(p_std) / RT, (double)MF(g_dnu)[r]);
            Kc *= gp[3];
            kr = kf / Kc;
        }
        kd[2 * r] = kf;
        kd[2 * r + 1] = kr;
        if (gi_tb(info) == 2) {
            const int fi = gi_foidx(info);
            const double* fp = MF(fo_par) + 8 * fi;
            double* fo = fod + 4 * fi;
            fo[0] = fp[0] * exp(fp[1] * lT - fp[2] / T) / kf;
            double fcv = 1.0;
            if (gi_troe(info)) {
                fcv = (1 - fp[3]) * exp(-T / fp[4]) + fp[3] * exp(-T / fp[5]);
                if (gi_troe(info) == 4) fcv += exp(-fp[6] / T);
            }
            const double lfc = log10(fcv);
            fo[1] = lfc;
            fo[2] = ((MF(conv) & BR_CONV_TROE_C4) ? -4.0 : -0.4) - 0.67 * lfc;
            fo[3] = 0.75 - 1.27 * lfc;
        }
    }
#pragma unroll 1
    for (int r = gl; r < nrs; r += GL) {                               // as init_tconst
        const uint32_t info = tb.sx[SX_WORDS * r + 4];
        const double* spr = MF(s_par) + 4 * r;
        double k;
        if (si_stick(info)) k = spr[0] * sqrt(RT / (2 * M_PI * spr[3]));
        else k = spr[0] * pow(T, spr[1]) * exp(-spr[2] / RT);
        skd[r] = k;
    }
    // the kd stores reach L2 and this CU's L1 is invalidated before any lane reads the slot (it held
    // the previous reactor's constants), as init_tconst's RXD
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    wave_sync();
}

// the mass-action part kf prod(c_f) - kr prod(c_b) of gas reaction r of a group (products in the
// wavefront engine's order; pad slots read conc[ONE] = 1), the reactant / product concentrations
// kept for the Jacobian
template <int GL>
__device__ __forceinline__ double g_mass_action_k(const double* sp, double2 k, uint32_t w0, uint32_t w1,
                                                  double (&cf)[4], double (&cb)[4]) {
    typedef grp::GLay<GL> L;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        cf[e] = sp[L::CONC + sp8(w0, e)];
        cb[e] = sp[L::CONC + sp8(w1, e)];
    }
    double Pf = (cf[0] * cf[1]) * cf[2], Pb = (cb[0] * cb[1]) * cb[2];
    if (MF(nu4)) { Pf *= cf[3]; Pb *= cb[3]; }
    return k.x * Pf - k.y * Pb;
}
// {kf, kr} of gas reaction r: one 16-byte load
__device__ __forceinline__ double2 g_kpair(const QKd* kd, int r) {
    return make_double2(kd[2 * r], kd[2 * r + 1]);   // (16-B aligned: one dwordx4 load)
}
template <int GL>
__device__ __forceinline__ double g_mass_action(const double* sp, const QKd* kd, uint32_t w0, uint32_t w1, int r,
                                                double (&cf)[4], double (&cb)[4]) {
    return g_mass_action_k<GL>(sp, g_kpair(kd, r), w0, w1, cf, cb);
}

// residual! (src/BatchReactor.jl:312-376) of a group's reactor: du of component gl (gas rates
// :355, surface rates :344, du assembly with the Asv quirk :345,:363-373); the pressure of this
// evaluation to *p_out (save_data semantics). Same arithmetic order as the wavefront engine's rhs()
// (concentrations, third-body pairing, rate products, falloff, surface coverage factor).
template <int GL>
__device__ __forceinline__ double g_rhs(const Tab& tb, double* sp, const QKd* kd, const double* fod, const double* skd,
                                        double T, double Asv, double Asv_th, double u, int gl, double* p_out) {
    typedef grp::GLay<GL> L;
    const int n = MF(n), ng = MF(ng), nrg = MF(nrg), nrs = MF(nrs), nset = MF(nset);
    const bool gas = gl < ng;
    // the {kf, kr} pairs of this lane's first two gas reactions, issued before the concentration and
    // third-body setup so their latency overlaps it (kd is in global memory)
    const double2 kz = make_double2(0.0, 0.0);
    const double2 kp0 = nrg > 0 ? g_kpair(kd, gl < nrg ? gl : 0) : kz;
    const double2 kp1 = nrg > GL ? g_kpair(kd, gl + GL < nrg ? gl + GL : 0) : kz;
    const double Mk = tb.molwt[gl];
    const double c = gl < n ? (gas ? u / Mk : u) : 0.0;              // c_k = u_k / M_k; coverages as is
    sp[L::CONC + gl] = c;
    sp[L::ACCW + gl] = 0.0;
    if (nrs) sp[L::ACCS + gl] = 0.0;
    const double Ctot = gsum<GL>(gas ? c : 0.0);
    const double p = R_GAS * T * Ctot;
    wave_sync();
    const double* conc = sp + L::CONC;
#pragma unroll 1
    for (int t = gl; t < nset; t += GL) {                              // third-body sums per efficiency set
        const uint32_t w = tb.tbs[t];                                  // (pairing as third_body_sets)
        const int b = w & 0xFFFFF, e = b + (int)(w >> 20);
        double s0 = Ctot, s1 = 0.0;
        int i = b;
#pragma unroll 1
        for (; i + 1 < e; i += 2) {
            const double2 e0 = *reinterpret_cast<const double2*>(tb.tbe + 16 * i);
            const double2 e1 = *reinterpret_cast<const double2*>(tb.tbe + 16 * (i + 1));
            s0 = fma(e0.y, conc[__double_as_longlong(e0.x) & 0xFFFF], s0);
            s1 = fma(e1.y, conc[__double_as_longlong(e1.x) & 0xFFFF], s1);
        }
        if (i < e) {
            const double2 e0 = *reinterpret_cast<const double2*>(tb.tbe + 16 * i);
            s0 = fma(e0.y, conc[__double_as_longlong(e0.x) & 0xFFFF], s0);
        }
        sp[L::MC + t] = s0 + s1;
    }
    wave_sync();
    double* accw = sp + L::ACCW;
    double* accs = sp + L::ACCS;
    const bool xm = (MF(conv) & 2) != 0;
    int it = 0;   // (uniform: the pass index)
#pragma unroll 1
    for (int r = gl; r < nrg; r += GL, ++it) {                         // gas reaction r on lane r mod GL
        const auto rr = rx_rec(tb.rx, r);
        const uint4 ra = *reinterpret_cast<const uint4*>(rr.a);
        const uint4 rb = *reinterpret_cast<const uint4*>(rr.b);
        double cf[4], cb[4];
        double2 kp;
        if (it == 0) kp = kp0;
        else if (it == 1) kp = kp1;
        else kp = g_kpair(kd, r);
        double D = g_mass_action_k<GL>(sp, kp, ra.x, ra.y, cf, cb);
        const int tbk = gi_tb(ra.z);
        if (tbk) {                                                     // as production()'s rate
            const double Mc = sp[L::MC + gi_tbidx(ra.z)];
            if (tbk == 1) D *= Mc;
            else {
                double fac, dfac;
                falloff<false>(fod + 4 * gi_foidx(ra.z), gi_troe(ra.z) != 0, Mc, fac, dfac);
                D *= fac;
                if (xm) D *= Mc * 1e-6;                                // [M] in mol/cm3
            }
        }
        scatter(accw, rb.x, rb.y, rb.z, rb.w, D);
    }
    const double RT = R_GAS * T;
#pragma unroll 1
    for (int r = gl; r < nrs; r += GL) {                               // surface reactions (production())
        const uint32_t* rec = tb.sx + SX_WORDS * r;
        const int nc = si_ncov(rec[4]);
        const double* xe = tb.sxe + SXE_DOUBLES * r;
        double k = skd[r] * xe[4];
        if (nc) {
            double s = 0.0;
            for (int j = 0; j < 4; ++j) if (j < nc) s += xe[j] * conc[sp8(rec[5], j)];
            k *= exp(-s / RT);
        }
        const double P = ((conc[sp8(rec[0], 0)] * conc[sp8(rec[0], 1)]) * (conc[sp8(rec[0], 2)] * conc[sp8(rec[0], 3)])) *
                         (conc[sp8(rec[1], 0)] * conc[sp8(rec[1], 1)]);
        scatter(accs, rec[6], rec[7], rec[8], rec[9], k * P);
    }
    wave_sync();
    const double w = gl < n ? accw[gl] : 0.0;
    if (nrs == 0) {                                                    // gas only (:363-370)
        wave_sync();
        if (gl == 0) *p_out = p;
        return gl < n ? w * Mk : 0.0;
    }
    const double sf = gl < n ? accs[gl] : 0.0;
    wave_sync();
    if (gl == 0) *p_out = p;
    if (gas) return (sf * Asv + w) * Mk;                               // :345, :363-370
    if (gl < n) return sf * Asv_th * tb.sigma[gl] / MF(G);             // :367 / :370
    return 0.0;
}

// (A register-row gas Jacobian -- every group evaluates every reaction, the sparse partials reach
// their column by scalar compares -- measured 902.2k vs 980.6k reactors/s for the column passes below,
// 78.8k vs 40.3k cycles per Jacobian: round 4. Removed in round 6.)

// Analytic Jacobian of a group's reactor with surface chemistry, in column passes as the wavefront
// engine's general jacobian() (brhip_device.hpp; oracle jac_tc): for each component j, the reactions
// whose rate depends on j (host column lists) spread over the group's lanes compute dq_r/du_j and
// scatter nu_kr dq_r/du_j into the production sums (gas reactions: d/dc_j, M_k / M_j applied per
// row; surface reactions: reactant partials with dc/du = 1/M, 1 (sticking) or Gamma/sigma and the
// coverage-dependent activation term -eps/RT q), then lane k writes J[k][j] = M_k w / M_j + M_k Asv
// s (gas rows) or Asv_th sigma_k / Gamma s (surface rows) to the saved-J slot through `jst`. No
// register tile: the state it needs is the species block of the RHS just evaluated.
template <int GL, class JST>
__device__ __forceinline__ void g_jac_cols(const Tab& tb, double* sp, const QKd* kd, const double* fod, const double* skd,
                                           double T, double Asv, double Asv_th, int gl, JST&& jst) {
    typedef grp::GLay<GL> L;
    const int n = MF(n), ng = MF(ng), nrg = MF(nrg), nrs = MF(nrs);
    const bool xm = (MF(conv) & 2) != 0;
    const double RT = R_GAS * T, Gs = MF(G);
    const double* conc = sp + L::CONC;
    double* accw = sp + L::ACCW;
    double* accs = sp + L::ACCS;
    const double Mk = tb.molwt[gl];
    const int* cp = MF(col_ptr);
    const int* cr = MF(col_rx);
#pragma unroll 1
    for (int j = 0; j < n; ++j) {
        accw[gl] = 0.0;
        if (nrs) accs[gl] = 0.0;   // (gas-only 16-lane blocks have no surface sums)
        wave_sync();
        const int cb = cp[j], ce = cp[j + 1];
#pragma unroll 1
        for (int i = cb + gl; i < ce; i += GL) {
            const int rr = cr[i];
            if (rr < nrg) {                                              // gas reaction: dq/dc_j
                const int r = rr;
                const auto rec = rx_rec(tb.rx, r);
                const uint32_t info = rec[2];
                const int nf = gi_nf(info), nr = gi_nr(info), tbk = gi_tb(info);
                double cf[4], cb4[4];
                const double D = g_mass_action<GL>(sp, kd, rec[0], rec[1], r, cf, cb4);
                double pre = 1.0, coefM = 0.0;
                if (tbk) {
                    const double Mc = sp[L::MC + gi_tbidx(info)];
                    if (tbk == 1) { pre = Mc; coefM = 1.0; }
                    else {
                        double fac, dfac;
                        falloff<true>(fod + 4 * gi_foidx(info), gi_troe(info) != 0, Mc, fac, dfac);
                        pre = fac * (xm ? Mc * 1e-6 : 1.0);
                        coefM = dfac * (xm ? Mc * 1e-6 : 1.0) + (xm ? fac * 1e-6 : 0.0);
                    }
                }
                double d = 0.0;
#pragma unroll
                for (int e = 0; e < 4; ++e) if (e < nf && sp8(rec[0], e) == j) {
                    double pr = kd[2 * r];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nf) pr *= conc[sp8(rec[0], e2)];
                    d += pre * pr;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) if (e < nr && sp8(rec[1], e) == j) {
                    double pr = kd[2 * r + 1];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) if (e2 != e && e2 < nr) pr *= conc[sp8(rec[1], e2)];
                    d -= pre * pr;
                }
                if (tbk && j < ng) d += (D * coefM) * MF(tb_eff)[gi_tbidx(info) * n + j];
                scatter(accw, rec[4], rec[5], rec[6], rec[7], d);
            } else {                                                     // surface reaction: dq/du_j
                const int r = rr - nrg;
                const uint32_t* rec = tb.sx + SX_WORDS * r;
                const uint32_t info = rec[4];
                const int nf = si_nf(info), nc = si_ncov(info);
                const bool stick = si_stick(info);
                const double* eps = tb.sxe + SXE_DOUBLES * r;
                double k = skd[r];
                if (nc) {
                    double s = 0.0;
                    for (int jj = 0; jj < 4; ++jj) if (jj < nc) s += eps[jj] * conc[sp8(rec[5], jj)];
                    k *= exp(-s / RT);
                }
                double cv[6], dc[6];
                int spe[6];
#pragma unroll
                for (int e = 0; e < 6; ++e) {
                    spe[e] = e < nf ? (e < 4 ? sp8(rec[0], e) : sp8(rec[1], e - 4)) : -1;
                    cv[e] = 1.0; dc[e] = 0.0;
                    if (e < nf) {
                        const int s = spe[e];
                        if (s < ng) { cv[e] = conc[s]; dc[e] = 1.0 / tb.molwt[s]; }
                        else if (stick) { cv[e] = conc[s]; dc[e] = 1.0; }
                        else { cv[e] = conc[s] * Gs / tb.sigma[s]; dc[e] = Gs / tb.sigma[s]; }
                    }
                }
                double d = 0.0;
#pragma unroll
                for (int e = 0; e < 6; ++e) if (spe[e] == j) {
                    double pr = k;
#pragma unroll
                    for (int e2 = 0; e2 < 6; ++e2) if (e2 != e && e2 < nf) pr *= cv[e2];
                    d += pr * dc[e];
                }
                if (nc) {
                    double P = 1.0;
#pragma unroll
                    for (int e = 0; e < 6; ++e) if (e < nf) P *= cv[e];
                    const double q = k * P;
                    for (int jj = 0; jj < 4; ++jj) if (jj < nc && (int)sp8(rec[5], jj) == j) d += q * (-eps[jj] / RT);
                }
                scatter(accs, rec[6], rec[7], rec[8], rec[9], d);
            }
        }
        wave_sync();
        const bool act = gl < n;
        const double w = act ? accw[gl] : 0.0;
        const double sf = (act && nrs) ? accs[gl] : 0.0;
        double v;
        if (gl < ng) v = (j < ng ? Mk * w / tb.molwt[j] : 0.0) + Mk * Asv * sf;
        else v = Asv_th * tb.sigma[gl] / Gs * sf;
        jst(j, act ? v : 0.0);
        wave_sync();
    }
}

// group pivot of step k: the first max |a| (bit patterns: a 32-bit max over the high words, then
// over the low words, then the lowest lane) among candidate lanes of the group; returns that lane
// within the group. SUNDIALS denseGETRF takes the first row of largest |a_ik| in the current
// (already interchanged) row order -- the lane order here.
template <int GL>
__device__ __forceinline__ int g_pivot(double a, bool cand, int gl) {
    const unsigned long long bits = (unsigned long long)__double_as_longlong(a) & 0x7fffffffffffffffull;
    const unsigned hi = cand ? (unsigned)(bits >> 32) : 0u;
    const unsigned mh = group_umax<GL>(hi);
    const bool top = cand && hi == mh;
    // usual case: one lane of each (active) group holds the largest high word -- it is the pivot,
    // and the low-word and lowest-lane rounds are skipped (wave-uniform test; C2 +0.5 %)
    const unsigned long long tb = __ballot(top);
    const unsigned gm = (unsigned)(tb >> (threadIdx.x & (64 - GL))) & (GL == 32 ? 0xffffffffu : 0xffffu);
    if (__ballot(__builtin_popcount(gm) != 1) == 0) return __builtin_ctz(gm);
    const unsigned lo = top ? (unsigned)bits : 0u;
    const unsigned ml = group_umax<GL>(lo);
    const bool top2 = top && lo == ml;
    const unsigned key = top2 ? ~(unsigned)gl : 0u;
    return (int)(~group_umax<GL>(key));
}

// LU of A = I - gamma J with partial pivoting as SUNDIALS denseGETRF (src/BatchReactor.jl:204-210:
// CVODE's dense linear solver), one row per lane in registers, rows interchanged physically (lane
// = current row position): after the factorization lane s holds row s of the factors (L's
// multipliers in a[k < s], U in a[k >= s]), dinv = 1 / u_ss, and orig = the original row now at
// lane s (the accumulated interchanges, applied to b by g_solve). Interchanges are bpermutes of the
// two rows' registers, issued only when some group of the wave needs one; the pivot row's values
// reach the group by DPP broadcasts from the compile-time lane k. Returns 0 or k+1 (zero pivot at
// step k, as denseGETRF).
template <int GL, int NM>
__device__ __forceinline__ int g_lu(const double (&jr)[NM], double gamma, int n, int gl, double (&a)[NM], int& orig,
                                    double& dinv) {
    const int gb = (int)(threadIdx.x & (64 - GL));
#pragma unroll
    for (int j = 0; j < NM; ++j) a[j] = ((j == gl && gl < n) ? 1.0 : 0.0) - gamma * jr[j];
    orig = gl;
    dinv = 0.0;
    int fail = 0;
    sfor<0, NM>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if (k < n) {
            const int p = g_pivot<GL>(a[k], gl >= k && gl < n, gl);
            if (__ballot(p != k) != 0) {                                 // interchange rows k and p
                const int src = gb + (gl == k ? p : (gl == p ? k : gl));
#pragma unroll
                for (int j = 0; j < NM; ++j) a[j] = lane_pull(a[j], src);
                orig = __builtin_amdgcn_ds_bpermute(src * 4, orig);
            }
            const double pv = group_bcast<GL, k>(a[k]);
            if (pv == 0.0 && fail == 0) fail = k + 1;
            const double rinv = 1.0 / pv;
            const bool below = gl > k;
            const double l = below ? a[k] * rinv : 0.0;                  // denseGETRF: a_ik *= 1 / a_kk
            if (below) a[k] = l;
            if (gl == k) dinv = rinv;
            // 16-lane groups: the pivot-row value enters the FMA as its DPP operand (v_fmac_f64_dpp
            // row_newbcast:k, the rows of all groups at once): one VALU op per element instead of two
            // DPP moves and an FMA; fma(u_kj, -l, a_ij) is fma(-u_kj, l, a_ij) exactly
#pragma unroll
            for (int j = k + 1; j < NM; ++j)
                if (j < n) {
                    if constexpr (GL == 16) dpp_fnma_self<k, 0xF>(a[j], l);
                    else a[j] = fma(-group_bcast<GL, k>(a[j]), l, a[j]);
                }
        }
    });
    return fail;
}

// solve (I - gamma J) x = b with g_lu's factors (denseGETRS): b interchanged (P b: one bpermute),
// forward with the unit L, backward with U; each step's pivot value reaches the group by a DPP
// broadcast from the compile-time lane k. b and x in component order (lane gl).
template <int GL, int NM>
__device__ __forceinline__ double g_solve(const double (&a)[NM], int orig, double dinv, int n, int gl, double b) {
    const int gb = (int)(threadIdx.x & (64 - GL));
    double y = lane_pull(gl < n ? b : 0.0, gb + orig);
    sfor<0, NM>([&](auto kc) {                                          // L y = P b
        constexpr int k = decltype(kc)::value;
        if (k + 1 < n) {
            if constexpr (GL == 16) {
                dpp_fnma_self<k, 0xF>(y, (gl > k) ? a[k] : 0.0);   // y += -l_sk y_k, y_k as the DPP operand
            } else {
                const double yk = group_bcast<GL, k>(y);
                y = fma(-((gl > k) ? a[k] : 0.0), yk, y);
            }
        }
    });
    double x = 0.0;
    sfor<0, NM>([&](auto kc) {                                          // U x = y, k = n-1 .. 0
        constexpr int k = NM - 1 - decltype(kc)::value;
        if (k < n) {
            if (gl == k) x = y * dinv;
            if constexpr (GL == 16) {
                dpp_fnma<k, 0xF, true>(y, x, (gl < k) ? a[k] : 0.0);   // y += -u_sk x_k
            } else {
                const double xk = group_bcast<GL, k>(x);
                y = fma(-((gl < k) ? a[k] : 0.0), xk, y);
            }
        }
    });
    return gl < n ? x : 0.0;
}

// the controller entry points for GL-lane groups (inline: out of line measured more VGPRs)
template <int GL, int VS>
__device__ __forceinline__ int g_post_rhs(LCtl* C, VA<1, GL, VS>& V, int gl, const double (&f)[1], double (&b)[1]) {
    return ctl_post_rhs<1, GL>(C, V, gl, f, b);
}
template <int GL, int VS>
__device__ __forceinline__ int g_post_solve(LCtl* C, VA<1, GL, VS>& V, int gl, double (&delta)[1], int lu_fail) {
    return ctl_post_solve<1, GL>(C, V, gl, delta, lu_fail);
}

#ifndef BR_GPRIO
// issue priority (s_setprio) of a wave while one of its groups runs its Jacobian / LU (the wave's other
// groups idle meanwhile): C2 993.8k vs 986.7k reactors/s at 2 (mean of two alternations, round 4)
#define BR_GPRIO 2
#endif
#ifndef BR_QWPB
#define BR_QWPB 4   // waves per workgroup (16 quad / 8 pair reactors); tables staged once per workgroup
#endif
#ifndef BR_QWPE
#define BR_QWPE 4   // waves per SIMD the register allocation targets for 16-lane groups (<= 128 VGPRs,
                    // ~128 B/lane spilled). Quad H2/O2: with the LDS block cut to 2.38 KB (kd global),
                    // four workgroups fit a CU: 1.100M reactors/s at 4 vs 981k at 3 (round 5); with the
                    // 2.83 KB block LDS capped it at 12 waves/CU (882k at 3 vs 693k at 2, round 4)
#endif
#ifndef BR_QWPE32
#define BR_QWPE32 3 // ... for 32-lane groups (surface-only Ni/CH4, n = 20: 194.8k reactors/s at 3 (228 B/lane
                    // spilled) vs 159.1k at 2; the wavefront engine does 217.7k, round 4)
#endif

// the group integrator kernel: persistent grid, every group takes reactor indices from o.work
template <int GL, int NM>
__global__ __launch_bounds__(64 * BR_QWPB) __attribute__((amdgpu_waves_per_eu(GL == 16 ? BR_QWPE : BR_QWPE32))) void k_group(
    DevMech M, int N, const double* __restrict__ Tv, const double* __restrict__ Asvv, double* __restrict__ U,
    const double* __restrict__ tfv, KOpts o, double* __restrict__ stats, double* __restrict__ Jws) {
    static_assert(NM <= GL, "register tile wider than the group");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    stage_tables(M, smem_raw);
    const Tab tb = tab_view<1>(smem_raw, M);
    constexpr int GPW = 64 / GL;                                        // groups per wave
    const int lane = threadIdx.x & 63, gl = lane & (GL - 1);
    const int grp = (int)(threadIdx.x / GL);                            // group within the workgroup
    const int slot = blockIdx.x * (BR_QWPB * GPW) + grp;                // workspace slot of this group
    const int RB = grp::block_bytes(GL, NM, MF(nrg), MF(nfo), MF(nrs));
    char* rbase = smem_raw + M.img_bytes + (size_t)grp * RB;
    LCtl* C = (LCtl*)rbase;
    VA<1, GL, grp::vstride(GL, NM)> V{(LDbl*)(rbase + CTL_BYTES), gl};
    double* sp = reinterpret_cast<double*>(rbase + grp::sp_off(GL, NM));
    double* fod = reinterpret_cast<double*>(rbase + grp::fod_off(GL, NM, MF(nrg), MF(nrs)));
    double* skd = fod + 4 * MF(nfo);
    const int SD = grp::slot_doubles(GL, MF(nrg));                      // global doubles per group slot
    QKd* kd = launder(Jws) + (size_t)slot * SD + GL * GL;
    // the group's saved-J slot through a buffer resource: lane offset in a VGPR, the column offset
    // j GL 8 as the instruction's scalar offset (as 64-bit addresses, the columns past 4 KB of a 32-lane
    // slot were materialised per column, hoisted out of the loop and spilled)
    const __amdgpu_buffer_rsrc_t jrs = __builtin_amdgcn_make_buffer_rsrc((void*)launder(Jws), (short)0, 0x7fffffff, 0x00020000);
    const unsigned jvo = (unsigned)(slot * SD + gl) * 8u;
    auto jst = [&](int j, double v) { __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), jrs, jvo, j * (GL * 8), 0); };
    auto jld = [&](int j) { return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(jrs, jvo, j * (GL * 8), 0)); };
    const int n = MF(n);
    const bool asv_fixed = (MF(conv) & 4) != 0;
    double* p_last = reinterpret_cast<double*>(rbase);                  // Ctl::p_last is the first field
    // this group's reactor: the first one from the work counter
    auto take = [&]() -> int {
        int v = 0;
        if (gl == 0) v = atomicAdd(o.work, 1);
        return __builtin_amdgcn_ds_bpermute((int)(threadIdx.x & (64 - GL)) * 4, v);
    };
    int rid = take();
    double T = 0.0, Asv = 1.0, Asv_th = 1.0;
    bool fresh = true;
    int dqj = -1;   // >= 0: building column dqj of the DQ Jacobian
    double a[NM];
    int orig = gl;
    double dinv = 0.0;
#pragma unroll
    for (int j = 0; j < NM; ++j) a[j] = 0.0;
    unsigned long long cyc0 = 0;
#if BR_PHASE_CLOCKS   // diagnostic build: this group's shader clocks per phase (br_stats cyc_*)
    unsigned long long q_rhs_c = 0, q_jac_c = 0, q_lu_c = 0, q_sol_c = 0, q_ctl_c = 0, q_all = 0;
#define QCLK(v) const unsigned long long v = clock64()
#define QACC(acc, v) acc += clock64() - v
#else
#define QCLK(v)
#define QACC(acc, v)
#endif
    for (;;) {
        if (__ballot(rid < N) == 0) break;
        if (rid < N) {
            if (fresh) {                                                // ---- CVodeInit for reactor rid
                fresh = false;
                cyc0 = wall_clock64();
#if BR_PHASE_CLOCKS
                q_rhs_c = q_jac_c = q_lu_c = q_sol_c = q_ctl_c = 0;
                q_all = clock64();
#endif
                T = Tv[rid];
                Asv = Asvv ? Asvv[rid] : 1.0;
                Asv_th = asv_fixed ? 1.0 : Asv;
                C->a_rtol = o.rtol; C->a_atol = o.atol; C->a_hmax_inv = o.hmax_inv; C->a_ufac = o.ufac;
                C->a_max_steps = o.max_steps; C->a_trace_cap = 0; C->a_trace = nullptr; C->a_rid = rid; C->a_n = n;
                C->a_ign = o.ign; C->a_nout = o.nout; C->a_tout = o.tout; C->a_yout = o.yout;
                g_init_tconst<GL>(tb, sp, kd, fod, skd, T, gl);
                const bool act = gl < n;
                const double u0 = act ? U[(size_t)rid * n + gl] : 0.0;
#pragma unroll
                for (int j = 0; j < NVEC; ++j) V.at(j, 0) = 0.0;
                V.at(0, 0) = u0;
                V.at(V_Y, 0) = u0;
                V.at(V_EWT, 0) = act ? 1.0 / (o.rtol * fabs(u0) + o.atol) : 1.0;
                const double su = gsum<GL>(act ? fabs(u0) : 0.0);
#pragma unroll
                for (int i = 0; i < QMAX + 2; ++i) C->tau[i] = 0.0;
#pragma unroll
                for (int i = 0; i < 6; ++i) C->tq[i] = 0.0;
#pragma unroll
                for (int i = 0; i <= QMAX; ++i) C->l[i] = 0.0;
                C->tn = 0.0; C->h = 0.0; C->rl1 = 0.0; C->gamma = 0.0; C->gamrat = 1.0; C->gammap = 0.0; C->crate = 1.0;
                C->delp = 0.0; C->hprime = 0.0; C->hscale = 0.0; C->eta = 1.0; C->etamax = ETAMX1; C->acnrm = 0.0;
                C->saved_tq5 = 0.0; C->saved_t = 0.0; C->tol = 0.0; C->hg = 0.0; C->hub = 0.0; C->hlb = 0.0; C->hnew = 0.0;
                C->tstop = tfv[rid];
                C->ulimit = o.ufac > 0.0 ? o.ufac * su : INFINITY;
                C->q = 1; C->qprime = 1; C->L = 2; C->qwait = 2;
                C->nst = 0; C->nfe = 0; C->nsetups = 0; C->nje = 0; C->nni = 0; C->ncfn = 0; C->netf = 0; C->nstlp = 0;
                C->nstlj = 0; C->ncf = 0; C->nef = 0; C->nstloc = 0; C->status = 0; C->m_it = 0; C->convfail = 0;
                C->count1 = 0; C->phase = PH_F0; C->callSetup = 0; C->jbad = 0; C->jcur_nls = 0; C->hnewOK = 0;
                C->newj = 0; C->p_last = 0.0;
                C->iout = 0; C->ign_t = 0.0; C->ign_rate = -INFINITY; C->t_ign = NAN; C->ign_x = 0.0; C->ign_dt = NAN;
                C->dq_mininc = 1.0; C->nfe_dq = 0;
                if (o.ign >= 0) {
                    double uv[1] = {u0};
                    C->ign_x = mole_frac_of<1, GL>(uv, gl, o.ign);
                }
                if (o.nout) {                                           // outputs at t <= 0: the initial state
                    int io = 0;
                    while (io < o.nout && !(o.tout[io] > 0.0)) {
                        if (act) o.yout[((size_t)rid * o.nout + io) * n + gl] = u0;
                        ++io;
                    }
                    C->iout = io;
                }
                wave_sync();
            }
            // ---- one RHS for this group's reactor, then its controller. dqj >= 0: this RHS is at
            // y + inc_dqj e_dqj, column dqj of CVODE's DQ Jacobian (cvLsDenseDQJac, k_integrate's
            // dq_* steps with GL-lane groups)
            double yv = V.at(V_Y, 0);
            if (dqj >= 0) {
                double inc[1];
                dq_incs<1, GL>(C, V, gl, inc);
                if (gl == dqj) yv += inc[0];
            }
            QCLK(c_r);
            const double fv = g_rhs<GL>(tb, sp, kd, fod, skd, T, Asv, Asv_th, yv, gl, p_last);
            BR_XG_AFTER_RHS();
            QACC(q_rhs_c, c_r);
            double f[1] = {fv}, b[1];
            int act_code;
            bool jac_ready = false;
            QCLK(c_c);
            if (dqj >= 0) {
                double inc[1];
                dq_incs<1, GL>(C, V, gl, inc);
                const double ii = 1.0 / gbcast<GL>(inc[0], dqj);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, ii * fv - ii * V.at(V_TEMP, 0)), jrs,
                                                      jvo + (unsigned)dqj * (GL * 8u), 0, 0);
                C->nfe_dq = C->nfe_dq + 1;
                if (++dqj < n) {
                    act_code = A_RHS;
                } else {
                    dqj = -1;
                    dq_newton_rhs<1, GL>(C, V, gl, b);
                    act_code = A_SETUP;
                    jac_ready = true;
                }
            } else {
                BR_SUB_T(pr0);
                act_code = g_post_rhs<GL>(C, V, gl, f, b);
                BR_SUB_ADD(3, pr0);
                if (act_code == A_SETUP && o.dq_jac && C->newj) {
                    dq_begin<1, GL>(C, V, gl, f);
                    dqj = 0;
                    act_code = A_RHS;
                }
            }
            QACC(q_ctl_c, c_c);
            int lu_fail = 0;
            if (act_code == A_SETUP) {
#if BR_GPRIO   // a wave with a group in its setup (the others idle) issues first
                __builtin_amdgcn_s_setprio(BR_GPRIO);
#endif
                if (!jac_ready && C->newj) {                            // analytic Jacobian at y, saved
                    QCLK(c_j);
                    g_jac_cols<GL>(tb, sp, kd, fod, skd, T, Asv, Asv_th, gl, jst);   // column passes
#pragma unroll 1
                    for (int j = n; j < NM; ++j) jst(j, 0.0);                 // padding columns
                    BR_XG_AFTER_JAC();
                    QACC(q_jac_c, c_j);
                }
                QCLK(c_l);
                double jr[NM];
#pragma unroll
                for (int j = 0; j < NM; ++j) jr[j] = jld(j);
                lu_fail = g_lu<GL, NM>(jr, C->gamma, n, gl, a, orig, dinv);
                BR_XG_AFTER_LU();
                QACC(q_lu_c, c_l);
#if BR_GPRIO
                __builtin_amdgcn_s_setprio(0);
#endif
            }
            if (act_code == A_SOLVE || act_code == A_SETUP) {
                QCLK(c_s);
                double delta[1] = {0.0};
                if (!lu_fail) {
                    delta[0] = g_solve<GL, NM>(a, orig, dinv, n, gl, b[0]);
                    BR_XG_AFTER_SOLVE();
                }
                QACC(q_sol_c, c_s);
                QCLK(c_p);
                BR_SUB_T(ps_all);
                act_code = g_post_solve<GL>(C, V, gl, delta, lu_fail);
                BR_SUB_ADD(13, ps_all);
                QACC(q_ctl_c, c_p);
            }
            if (act_code == A_DONE) {                                   // ---- results, next reactor
                const int status = C->status;
                const double u_out = status ? V.at(0, 0) : V.at(V_Y, 0);
                if (gl < n) U[(size_t)rid * n + gl] = u_out;
                if (stats && gl == 0) {
                    double* st = stats + (size_t)rid * BR_NSTAT;
                    st[0] = C->nst; st[1] = C->nfe; st[2] = C->nje; st[3] = C->nsetups; st[4] = C->nni;
                    st[5] = C->ncfn; st[6] = C->netf; st[7] = (double)status;
                    st[8] = (double)(wall_clock64() - cyc0);
#if BR_PHASE_CLOCKS
                    st[9] = (double)q_rhs_c; st[10] = (double)q_jac_c; st[11] = (double)q_lu_c; st[12] = (double)q_sol_c;
                    st[14] = (double)q_ctl_c; st[15] = (double)(clock64() - q_all);
#else
                    st[9] = st[10] = st[11] = st[12] = st[14] = st[15] = 0.0;
#endif
                    st[13] = C->tn;
                    st[16] = o.ign >= 0 ? (double)C->t_ign : NAN; st[17] = o.ign >= 0 ? (double)C->ign_rate : NAN;
                    st[18] = o.ign >= 0 ? (double)C->ign_dt : NAN; st[19] = C->nfe_dq;
                }
                rid = take();
                fresh = true;
            }
        }
    }
#undef QCLK
#undef QACC
}
