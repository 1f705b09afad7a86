// shud_ele_packed.hip — production element kernel on the packed class layout (shud_dev.h DevPacked).
//
// Same physics, same fp64 operation order as shud_ele_kernel (shud_kernels.hip) — which restates
// f_etFlux (MD_ET.cpp:343-404), updateElement/Flux_Infiltration/Flux_Recharge (Element.cpp:271-384),
// fun_Ele_surface/fun_Ele_sub (MD_ElementFlux.cpp:35-156), fun_Seg_surface/fun_Seg_sub
// (MD_RiverFlux.cpp:100-126), PassValue's Qe2r sums (MD_f.cpp:228-235) and f_applyDY (MD_f.cpp:65-156).
// What differs is only how the operands reach the registers:
//   * loads are unconditional (neighbour indices clamped to the element itself on a boundary edge), so
//     they never queue behind branches; the element's own records are issued up front, each edge's
//     neighbour data at the top of its (rolled) iteration — at 96 VGPRs five waves per SIMD hide the
//     latency that three waves holding everything up front could not;
//   * the element's own streams arrive as 16-byte records (global_load_dwordx4), per-element hydraulic
//     parameters through a class id into a table that stays in L1/L2;
//   * single-use streams are loaded/stored non-temporally and workgroups are dealt to XCDs in
//     contiguous chunks so the neighbour rows an element block gathers are in its own XCD's L2.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "shud_dev.h"
#include "shud_physics.h"

namespace shud {

typedef double v2d __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
template <class T>
__device__ __forceinline__ T ldnt(const T *p) { return __builtin_nontemporal_load(p); }
// one 16-byte non-temporal load (global_load_dwordx4 nt)
__device__ __forceinline__ double2 ldnt2(const double2 *p) {
    const v2d v = __builtin_nontemporal_load((const v2d *)p);
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ int4 ldnt4(const int4 *p) {
    const v4i v = __builtin_nontemporal_load((const v4i *)p);
    return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stnt2(double2 *p, double a, double b) {
    v2d v;
    v.x = a;
    v.y = b;
    __builtin_nontemporal_store(v, (v2d *)p);
}

__device__ __forceinline__ int pk_flags(double2 a) { return (int)(unsigned)(__double_as_longlong(a.y) & 0xffffffffLL); }
__device__ __forceinline__ int pk_class(double2 a) { return (int)((unsigned long long)__double_as_longlong(a.y) >> 32); }

// uYgw of element j from its packed flags (MD_update.cpp:114-125 / MD_f_omp.cpp:119-128)
template <int MODE>
__device__ __forceinline__ double ugw_pk(const DevMesh &m, double ygw_raw, int flags, int j) {
    const int ibc = (int)(int16_t)(flags & 0xffff);
    if (ibc == 0) return MODE == 0 ? ygw_raw : rmax(0.0, ygw_raw);
    if (ibc > 0) return m.eybc[ibc];
    return m.ugw_stale[j];
}

// HOIST: where the neighbour / edge-geometry loads are issued — 0: with the element's own loads at the
// top (maximum latency cover, most live registers), 1: after the vertical phase, 2: after f_etFlux,
// 3: per edge inside a rolled edge loop (fewest live registers; production).
template <int MODE, bool OPEN, bool DIAG, bool FU1, int LBW = 1, int HOIST = 0>
__global__ void __launch_bounds__(256, LBW)
shud_ele_kernel_packed(DevMesh m, DevPacked p, YView Y, double *__restrict__ dy, int n_compute, int cur,
                       DevDiag dg) {
    const int i = block_id<1>() * blockDim.x + threadIdx.x;
    if (i >= n_compute) return;
    const int NEl = m.num_ele;
    const int nown = Y.n_own;

    // ---------------- issue every load first ----------------
    const double2 zz = p.zz[i];
    const double2 aqk = p.aqk[i];
    const int4 mt = ldnt4(&p.meta[i]);
    const double2 snp = ldnt2(&p.s_np[i]), stl = ldnt2(&p.s_tl[i]);
    const double etp = ldnt(&m.etp[i]);
    double2 fu;
    if (FU1) { fu.x = 1.0; fu.y = 1.0; } else fu = ldnt2(&p.s_fu[i]);
    const double2 csv = ldnt2(&p.cs[cur][i]);
    const double ysf_raw = Y.sf(i), yus_raw = Y.us(i), ygw_raw = Y.gw(i);
    int nbv[3] = {mt.x, mt.y, mt.z};
    double2 nzz[3], naq[3], e01, e2a, d01;
    double nsf_raw[3], ngw_raw[3], d2;
    auto load_lateral = [&]() {
        e01 = ldnt2(&p.ge01[i]);
        e2a = ldnt2(&p.ge2a[i]);
        d01 = ldnt2(&p.gd01[i]);
        d2 = ldnt(&p.gd2[i]);
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int nc = nbv[j] >= 0 ? nbv[j] : i;     // boundary edge: a harmless in-bounds load
            nzz[j] = p.zz[nc];
            naq[j] = p.aqk[nc];
            nsf_raw[j] = Y.sf(nc);
            ngw_raw[j] = Y.gw(nc);
        }
    };
    if (HOIST == 0) load_lateral();
    (void)nbv;
    const int flags = pk_flags(aqk);
    const int cid = pk_class(aqk);
#define CL(f) p.ctab[CF_##f * p.ncls + cid]
    const int ibc = (int)(int16_t)(flags & 0xffff);
    const int iss = (flags >> 16) & 3;
    const int nseg = (flags >> 18) & 63;

    // ---- f_update ----
    double usf = ysf_raw, uus = yus_raw;
    if (MODE == 1) { usf = (usf >= 0.) ? usf : 0.; uus = (uus >= 0.) ? uus : 0.; }
    const double ugw = ugw_pk<MODE>(m, ygw_raw, flags, i);
    const double aq = aqk.x, infD = CL(infD), ThS = CL(ThetaS), ThR = CL(ThetaR);
    const double infK = CL(infKsatV), hA = CL(hAreaF), macKV = CL(macKsatV);
    const double fu_surf = fu.x, fu_sub = fu.y;

    // ---- f_etFlux (MD_ET.cpp:343-404), serial semantics only ----
    double Es = 0., Eu = 0., Eg = 0., Tu = 0., Tg = 0., eic = csv.y, ibeta = 0.;
    if (MODE == 0) {
        const double satn_prev = csv.x;
        const double vf = CL(VegFrac), va = vf, vb = 1. - vf, pj = 1. - CL(ImpAF);
        const double pet = snp.y, ptr = stl.x;
        {
            double fc = ThS * K_FC_RATIO;
            double b = (satn_prev * (ThS - ThR) - ThR) / (fc - ThR);
            b = rmin(rmax(0., b), 1.);
            ibeta = 0.5 * (1 - cos(K_PI * b));
        }
        Es = rmin(rmax(0., usf), pet) * vb;
        if (Es < pet) {
            if (ugw > aq - infD) { Eg = rmin(rmax(0., ugw), pet - Es) * pj * vb; Eu = 0.; }
            else { Eg = 0.; Eu = rmin(rmax(0., uus), ibeta * (pet - Es)) * pj * vb; }
        }
        if (stl.y > K_ZERO) {
            if (eic >= ptr) { Tg = Tu = 0.; eic = ptr * pj * va; }
            else if (ugw > aq - CL(RzD)) { Tg = rmin(rmax(0., ugw), (ptr - eic)) * pj * va; Tu = 0.; }
            else { Tg = 0.; Tu = rmin(rmax(0., uus), ibeta * (ptr - eic)) * pj * va; }
        } else { Tg = Tu = eic = 0.; }
        const double trans = Tg + Tu, evapo = Eu + Eg + Es, eta = eic + evapo + trans;
        if (eta > etp * 2.) { atomicAdd(&m.err->n_warn, 1ULL); report(m.err, 0x10u, 4, i); }
        bool neg = false;
        neg |= (Es < 0.0 || isnan(Es) || isinf(Es) || fabs(Es - K_NA_VALUE) < K_ZERO);
        neg |= (Eu < 0.0 || isnan(Eu) || isinf(Eu) || fabs(Eu - K_NA_VALUE) < K_ZERO);
        neg |= (Eg < 0.0 || isnan(Eg) || isinf(Eg) || fabs(Eg - K_NA_VALUE) < K_ZERO);
        neg |= (Tu < 0.0 || isnan(Tu) || isinf(Tu) || fabs(Tu - K_NA_VALUE) < K_ZERO);
        neg |= (Tg < 0.0 || isnan(Tg) || isinf(Tg) || fabs(Tg - K_NA_VALUE) < K_ZERO);
        if (neg) report(m.err, 0x04u, 2, i);
        else if (isnan(eta) || isinf(eta) || isnan(evapo) || isinf(evapo) || isnan(trans) || isinf(trans))
            report(m.err, 0x08u, 3, i);
        if (DIAG) { dg.q_es[i] = Es; dg.q_eu[i] = Eu; dg.q_eg[i] = Eg; dg.q_tu[i] = Tu; dg.q_tg[i] = Tg;
                    dg.q_eta[i] = eta; dg.i_beta[i] = ibeta; }
    }

    if (HOIST == 2) {
        __builtin_amdgcn_sched_barrier(0);
        load_lateral();
    }
    // ---- updateElement (Element.cpp:347-384) ----
    const double ekh = eff_kh(ugw, aq, CL(macD), CL(macKsatH), CL(vAreaF), CL(KsatH));
    if (ekh < 0. || ekh > 1e9) report(m.err, 0x02u, 1, i);
    double deficit = aq - ugw;
    const double kmax = infK * (1. - hA) + macKV * hA;
    double theta, satn, satkr;
    if (deficit <= 0.) { deficit = 0.; satn = 1.; theta = ThS; }
    else { theta = uus / deficit * ThS; satn = (theta - ThR) / (ThS - ThR); }
    if (satn > 0.99) { satn = 1.0; satkr = 1.0; theta = ThS; }
    else if (satn <= K_ZERO) { satn = 0.; satkr = 0.; theta = ThR; }
    else {
        const double n = CL(Beta);
        const double tmp = -1. + pow(1. - pow(satn, n / (n - 1.)), (n - 1.) / n);
        satkr = sqrt(satn) * tmp * tmp;
    }
    stnt2(&p.cs[cur ^ 1][i], satn, eic);

    // ---- Flux_Infiltration (Element.cpp:271-303) ----
    double qi = 0., qex = 0.;
    {
        const double av = usf + snp.x;
        if (ugw + uus > aq || deficit < uus) {
            qex = fabs(ugw + uus - aq) / aq * kmax;
        } else if (av > 0. && deficit > infD) {
            const double grad = 1. + av / infD;
            double ek;
            if (av > kmax) ek = infK * (1 - hA) + hA * macKV * satn;
            else if (av > infK) ek = satkr * infK * (1 - hA) + hA * macKV * satn;
            else ek = satkr * infK * (1 - hA);
            qi = rmin(av, rmax(0., grad * ek));
        }
    }
    const double q_infil = qi * fu_surf, q_exfil = qex * fu_surf;
    // ---- Flux_Recharge (Element.cpp:304-335) ----
    double qr = 0.;
    {
        const double KV = CL(KsatV);
        if (!(ugw > aq - infD && uus < deficit)) {
            double grad = 0.;
            if (theta > ThR && !(uus <= K_EPSILON)) {
                grad = (theta - ThR) / (ThS * K_FC_RATIO - ThR);
                grad = rmax(grad, 0.);
            }
            if (!(infK <= 0. || KV <= 0.)) {
                const double ku = infK * satkr;
                qr = grad * ((ku * KV) * (deficit + ugw) / (deficit * KV + ugw * ku));
            }
        }
    }
    const double q_rech = qr * fu_sub;

    // DY terms that do not depend on the lateral fluxes, in the reference's left-to-right order
    // (MD_f.cpp:88-90): dsf = ((net_prep - infil) + exfil) - Qsurf/area - Es,  dus complete,
    // dgw = (recharge - exfil) - Qsub/area - Eg - Tg.  Computing them here ends the live ranges of the
    // individual ET/vertical terms before the register-heavy lateral loop.
    const double dsf_head = snp.x - q_infil + q_exfil;
    const double dgw_head = q_rech - q_exfil;
    const double sy = CL(Sy);
    if (i < nown) {
        const double dus = (q_infil - q_rech - Eu - Tu) / sy;
        __builtin_nontemporal_store(dus, &dy[nown + i]);
    }
    if (HOIST == 1) {
        __builtin_amdgcn_sched_barrier(0);     // keep the lateral loads (and their registers) out of phase 1
        load_lateral();
    }
    // ---- own river segments (fun_Seg_surface / fun_Seg_sub) and Qe2r (PassValue) ----
    const double zs = zz.x, zb = zz.y, dep = CL(depression), rgh = CL(rough);
    double qe2r_surf = 0., qe2r_sub = 0.;
    if (nseg) {
        const double isf_seg = rmax(0., usf - q_infil + q_exfil);
        for (int k = mt.w, k1 = mt.w + nseg; k < k1; k++) {
            const int r = m.seg_riv[k];
            double yraw;
            const double yr = uriv_of<MODE>(m, Y, r, &yraw);
            const double rdep = m.riv_depth[r];
            const double L = m.seg_len[k];
            const double qs = weir_jtoi(zs, isf_seg, zs - rdep, yr, zs + 0.0, m.seg_cwr[k], L, dep);
            const double qg = r2e_gw(yr, zs - rdep, ugw, zb, ekh, m.riv_ksath[r], L, m.riv_bedthick[r]) * fu_sub;
            m.qseg_surf[k] = qs;
            m.qseg_sub[k] = qg;
            qe2r_surf += -qs;
            qe2r_sub += -qg;
        }
    }
    if (DIAG) {
        dg.q_infil[i] = q_infil; dg.q_exfil[i] = q_exfil; dg.q_recharge[i] = q_rech;
        dg.e_ic[i] = eic; dg.u_satn[i] = satn; dg.eff_kh[i] = ekh;
        dg.qe2r_surf[i] = qe2r_surf; dg.qe2r_sub[i] = qe2r_sub;
    }
    if (i >= nown) return;    // ghost element of a partition: vertical + segments only

    // ---- fun_Ele_surface / fun_Ele_sub over 3 edges (MD_ElementFlux.cpp:35-156) ----
    double sumsurf = qe2r_surf, sumsub = qe2r_sub;
    bool nan_q = false;
    const double isf = usf < 0. ? 0. : usf;
    if (HOIST == 3) {
        e01 = ldnt2(&p.ge01[i]);
        e2a = ldnt2(&p.ge2a[i]);
        d01 = ldnt2(&p.gd01[i]);
        d2 = ldnt(&p.gd2[i]);
    }
#pragma unroll
    for (int j0 = 0; j0 < 3; j0 += (HOIST == 3 ? 3 : 1)) {
#pragma unroll 1
    for (int j = j0; j < (HOIST == 3 ? 3 : j0 + 1); j++) {
        const int nb = j == 0 ? nbv[0] : j == 1 ? nbv[1] : nbv[2];
        const double B = j == 0 ? e01.x : j == 1 ? e01.y : e2a.x;
        const double Dj = j == 0 ? d01.x : j == 1 ? d01.y : d2;
        double2 nzzj, naqj;
        double nsfj, ngwj;
        if (HOIST == 3) {                          // this edge's neighbour data, loaded in the iteration
            const int ncl = nb >= 0 ? nb : i;
            nzzj = p.zz[ncl];
            naqj = p.aqk[ncl];
            nsfj = Y.sf(ncl);
            ngwj = Y.gw(ncl);
        } else {
            nzzj = nzz[j]; naqj = naq[j]; nsfj = nsf_raw[j]; ngwj = ngw_raw[j];
        }
        double qsf = 0., qsb = 0.;
        if (nb >= 0) {
            const int cn = pk_class(naqj);
#define CN(f) p.ctab[CF_##f * p.ncls + cn]
            double nsf = nsfj;
            if (MODE == 1) nsf = (nsf >= 0.) ? nsf : 0.;
            nsf = nsf < 0. ? 0. : nsf;
            const double zsn = nzzj.x;
            const double d2n = Dj;
            const double dh = (isf + zs) - (nsf + zsn);
            double ym = ((isf + zs) > (nsf + zsn)) ? ((isf > dep) ? isf : 0.) : ((nsf > dep) ? nsf : 0.);
            ym = rmin(ym, K_MAXYSURF);
            if (ym > 0.) {
                const double s = dh / d2n;
                if (s > 0 && isf <= 0) qsf = 0.;
                else if (s < 0 && nsf <= 0) qsf = 0.;
                else qsf = manning(ym * B, 0.5 * (rgh + CN(rough)), ym, s);   // avgRough, Element.cpp:253
            }
            const double ugn = ugw_pk<MODE>(m, ngwj, pk_flags(naqj), nb);
            const double zbn = nzzj.y;
            const double dhg = (ugw + zb) - (ugn + zbn);
            double q = 0.;
            if (dhg > 0. && ugw <= 0.02) q = 0.;
            else if (dhg < 0. && ugn <= 0.02) q = 0.;
            else {
                const double ekn = eff_kh(ugn, naqj.x, CN(macD), CN(macKsatH), CN(vAreaF), CN(KsatH));
#undef CN
                const double ymg = (rmax(ugw, 0.) + rmax(ugn, 0.)) * .5;
                const double grad = dhg / d2n;
                const double kmean = 0.5 * (ekh + ekn);
                q = kmean * grad * ymg * B;
            }
            qsb = q * fu_sub;
        } else if (!OPEN) {
            qsb = 0. * fu_sub;
        } else {
            const double d2e = m.dist2edge[j * NEl + i];
            if (isf > dep) {
                const double s = isf / d2e * 0.5;
                if (s > 0.) qsf = sqrt(s) * cbrt(isf * isf * isf * isf * isf) * B / rgh;
            }
            double q = 0.;
            if (ugw > dep * 10.) {
                const double grad = ugw / d2e * 0.5;
                if (grad > 0.) q = ekh * grad;
            }
            qsb = q * fu_sub;
        }
        if (MODE == 0) nan_q |= (isnan(qsf) || isinf(qsf) || isnan(qsb) || isinf(qsb));
        sumsurf += qsf;
        sumsub += qsb;
        if (DIAG) { dg.qele_surf[j * NEl + i] = qsf; dg.qele_sub[j * NEl + i] = qsb; }
    }
    }
    if (MODE == 0 && nan_q) report(m.err, 0x01u, 0, i);

    // ---- f_applyDY element part (MD_f.cpp:88-131 / MD_f_omp.cpp:26-46) ----
    const double area = e2a.y;
    double dsf = dsf_head - sumsurf / area - Es;
    double dgw = dgw_head - sumsub / area - Eg - Tg;
    if (ibc > 0) dgw = 0;
    else if (ibc < 0) dgw += m.eqbc[-ibc] / area;
    if (iss == 1) dsf += 0.0 / area;
    else if (iss == 2) dgw += 0.0 / area;
#undef CL
    dgw /= sy;
    __builtin_nontemporal_store(dsf, &dy[i]);
    __builtin_nontemporal_store(dgw, &dy[2 * nown + i]);
    if (DIAG) { dg.qele_surf_tot[i] = sumsurf; dg.qele_sub_tot[i] = sumsub; }
}

// step inputs (SoA staging in DevMesh) -> packed records; `what` bits: 1 np, 2 tl, 4 fu, 8 u_satn, 16 e_ic
__global__ void __launch_bounds__(256)
shud_pack_step_kernel(DevMesh m, DevPacked p, int n, int cur, unsigned what) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (what & 1) p.s_np[i] = make_double2(m.net_prep[i], m.pot_evap[i]);
    if (what & 2) p.s_tl[i] = make_double2(m.pot_tran[i], m.lai[i]);
    if (what & 4) p.s_fu[i] = make_double2(m.fu_surf[i], m.fu_sub[i]);
    if (what & 8) p.cs[cur][i].x = m.u_satn[0][i];
    if (what & 16) p.cs[cur][i].y = m.e_ic[0][i];
}

// pk_waves (SHUD_RHS_PK_WAVES, A/B only): minimum waves per SIMD, 0 = compiler's choice
template <int MODE, bool OPEN, bool DIAG, bool FU1>
static void launch_p(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int n, int cur,
                     const DevDiag &dg, hipStream_t s, int pk_waves) {
    int nb = (n + 255) / 256;
    nb = (nb + 7) / 8 * 8;                  // block_id<1> deals blocks to XCDs in contiguous chunks
#define KP(W, H) hipLaunchKernelGGL((shud_ele_kernel_packed<MODE, OPEN, DIAG, FU1, W, H>), dim3(nb), dim3(256), 0, s, \
                                    m, p, Y, dy, n, cur, dg)
    if (MODE == 0 && !OPEN && !DIAG) {       // A/B builds: pk_waves = W + 10 * HOIST
        switch (pk_waves) {
            case 4: KP(4, 0); return;
            case 10: KP(1, 1); return;
            case 14: KP(4, 1); return;
            case 20: KP(1, 2); return;
            case 24: KP(4, 2); return;
            case 30: KP(1, 3); return;
            case 34: KP(4, 3); return;
            case 35: KP(5, 3); return;
            case 36: KP(6, 3); return;
            case 38: KP(8, 3); return;
            default: break;
        }
    }
    // production build: neighbour data loaded inside a rolled edge loop (HOIST 3) at >= 5 waves/SIMD —
    // 96 VGPRs, no spills; 0.78 ms vs 0.87 ms for all-loads-up-front at 145 VGPRs / 3 waves (syn-10M A/B)
    KP(5, 3);
#undef KP
}

void launch_element_kernel_packed(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int n_compute,
                                  int cur, int mode, bool open, bool diag, bool fu_unit, const DevDiag &dg,
                                  hipStream_t s, int pk_waves) {
    if (n_compute <= 0) return;
#define LP(MO, OP, DI, FU) launch_p<MO, OP, DI, FU>(m, p, Y, dy, n_compute, cur, dg, s, pk_waves)
#define LFU(MO, OP, DI) do { if (fu_unit) LP(MO, OP, DI, true); else LP(MO, OP, DI, false); } while (0)
#define LDI(MO, OP) do { if (diag) LFU(MO, OP, true); else LFU(MO, OP, false); } while (0)
#define LOP(MO) do { if (open) LDI(MO, true); else LDI(MO, false); } while (0)
    if (mode == 0) LOP(0); else LOP(1);
#undef LOP
#undef LDI
#undef LFU
#undef LP
}

void launch_pack_step_kernel(const DevMesh &m, const DevPacked &p, int n, int cur, unsigned what, hipStream_t s) {
    if (n <= 0 || !what) return;
    hipLaunchKernelGGL(shud_pack_step_kernel, dim3((n + 255) / 256), dim3(256), 0, s, m, p, n, cur, what);
}

}  // namespace shud
