// shud_kernels.hip — gfx950 kernels for the SHUD RHS (DankerMu/SHUD-up src/Model/f.cpp:2-32).
//
// Two launches per RHS evaluation (both owner-computes, no atomics on fp64 sums):
//   shud_ele_kernel : one lane per element.  Fuses loop A (f_etFlux MD_ET.cpp:343-404,
//                     updateElement Element.cpp:347-384, infiltration/recharge :271-335), loop B
//                     (fun_Ele_surface/fun_Ele_sub MD_ElementFlux.cpp:35-156, neighbour effKH
//                     recomputed on the fly from the neighbour's state), the element's own river
//                     segments (loop C, MD_RiverFlux.cpp:100-126) gathered through an element-sorted
//                     CSR, the Qe2r part of PassValue (MD_f.cpp:228-235) and the element half of
//                     f_applyDY (MD_f.cpp:65-156).  Writes DY[sf,us,gw], carried qEleE_IC/u_satn and
//                     the per-segment fluxes the river kernel reduces.
//   shud_riv_kernel : one lane per reach.  Flux_RiverDown (MD_RiverFlux.cpp:5-63) for itself and for
//                     its upstream reaches (the junction sum of PassValue MD_f.cpp:236-240 in ascending
//                     reach order), segment sums in ascending segment order, river DY (MD_f.cpp:157-179).
// Every reduction is evaluated in the reference's order, so results are deterministic and equal to
// the serial reference up to libm (OCML vs glibc pow/cbrt/cos) rounding.  Same leaf functions as the packed kernel
// (shud_physics.h: pow_tab for satKfun, OCML's cos on [0, pi] = cos_small), so both layouts give the same bits.
// Compiled with -ffp-contract=off (the reference x86-64 -O3 build has no FMA).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "shud_dev.h"
#include "shud_physics.h"

namespace shud {

// ===================================================================================
// element kernel
// ===================================================================================
template <int MODE, bool OPEN, bool DIAG>
__global__ void __launch_bounds__(256)
shud_ele_kernel(DevMesh m, YView Y, double *__restrict__ dy, int n_compute, int cur, int cur_e, DevDiag dg) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_compute) return;
    const int NEl = m.num_ele;        // local element count (stride of per-edge arrays)
    const int nown = Y.n_own;
    const int flags = m.eflags[i];
    const int ibc = (int)(int16_t)(flags & 0xffff);
    const int iss = (flags >> 16) & 3;            // 0 none, 1 >0, 2 <0

    // ---- f_update (MD_update.cpp:102-189 / MD_f_omp.cpp:104-170) ----
    double usf = Y.sf(i), uus = Y.us(i);
    if (MODE == 1) { usf = (usf >= 0.) ? usf : 0.; uus = (uus >= 0.) ? uus : 0.; }
    const double ugw = ugw_of<MODE>(m, Y, i, ibc);

    const double aq = m.aq[i], infD = m.infD[i], ThS = m.ThetaS[i], ThR = m.ThetaR[i];
    const double infK = m.infKsatV[i], hA = m.hAreaF[i], macKV = m.macKsatV[i];
    const double fu_surf = m.fu_surf[i], fu_sub = m.fu_sub[i];

    // ---- f_etFlux (MD_ET.cpp:343-404), serial semantics only ----
    double Es = 0., Eu = 0., Eg = 0., Tu = 0., Tg = 0., eic = 0., ibeta = 0.;
    if (MODE == 0) {
        const double satn_prev = m.u_satn[cur][i];
        const double vf = m.VegFrac[i], va = vf, vb = 1. - vf, pj = 1. - m.ImpAF[i];
        const double pet = m.pot_evap[i], ptr = m.pot_tran[i];
        eic = m.e_ic[cur_e][i];
        {   // SoilMoistureStress is_sm_et.cpp:131-140
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
        if (m.lai[i] > K_ZERO) {
            if (eic >= ptr) { Tg = Tu = 0.; eic = ptr * pj * va; }
            else if (ugw > aq - m.RzD[i]) { Tg = rmin(rmax(0., ugw), (ptr - eic)) * pj * va; Tu = 0.; }
            else { Tg = 0.; Tu = rmin(rmax(0., uus), ibeta * (ptr - eic)) * pj * va; }
        } else { Tg = Tu = eic = 0.; }
        const double trans = Tg + Tu, evapo = Eu + Eg + Es, eta = eic + evapo + trans;
        report_w(m.err, eta > m.etp[i] * 2., 0x10u, 4, i, true);
        bool neg = false;
        neg |= (Es < 0.0 || isnan(Es) || isinf(Es) || fabs(Es - K_NA_VALUE) < K_ZERO);
        neg |= (Eu < 0.0 || isnan(Eu) || isinf(Eu) || fabs(Eu - K_NA_VALUE) < K_ZERO);
        neg |= (Eg < 0.0 || isnan(Eg) || isinf(Eg) || fabs(Eg - K_NA_VALUE) < K_ZERO);
        neg |= (Tu < 0.0 || isnan(Tu) || isinf(Tu) || fabs(Tu - K_NA_VALUE) < K_ZERO);
        neg |= (Tg < 0.0 || isnan(Tg) || isinf(Tg) || fabs(Tg - K_NA_VALUE) < K_ZERO);
        report_w(m.err, neg, 0x04u, 2, i);
        report_w(m.err, !neg && (isnan(eta) || isinf(eta) || isnan(evapo) || isinf(evapo) || isnan(trans) || isinf(trans)),
                 0x08u, 3, i);
        m.e_ic[cur_e ^ 1][i] = eic;
        if (DIAG) { dg.q_es[i] = Es; dg.q_eu[i] = Eu; dg.q_eg[i] = Eg; dg.q_tu[i] = Tu; dg.q_tg[i] = Tg;
                    dg.q_eta[i] = eta; dg.i_beta[i] = ibeta; }
    }

    // ---- updateElement (Element.cpp:347-384) ----
    const double ekh = eff_kh(ugw, aq, m.macD[i], m.macKsatH[i], m.vAreaF[i], m.KsatH[i]);
    report_w(m.err, ekh < 0. || ekh > 1e9, 0x02u, 1, i);
    double deficit = aq - ugw;
    const double kmax = infK * (1. - hA) + macKV * hA;
    double theta, satn, satkr;
    if (deficit <= 0.) { deficit = 0.; satn = 1.; theta = ThS; }
    else { theta = uus / deficit * ThS; satn = (theta - ThR) / (ThS - ThR); }
    if (satn > 0.99) { satn = 1.0; satkr = 1.0; theta = ThS; }
    else if (satn <= K_ZERO) { satn = 0.; satkr = 0.; theta = ThR; }
    else {   // satKfun Equations.cpp:136-141
        // Beta > 1 (every class the packed layout admits): the packed kernel's pow_tab, so both layouts give the same
        // bits (shud_physics.h sat_kfun, tables from __constant__ memory); any other Beta: the full pow
        const double n = m.Beta[i];
        const double ex1 = n / (n - 1.), ex2 = (n - 1.) / n;
        if (n > 1. && __builtin_isfinite(ex1) && __builtin_isfinite(ex2)) {
            satkr = sat_kfun(satn, ex1, ex2);
        } else {
            const double tmp = -1. + pow(1. - pow(satn, ex1), ex2);
            satkr = sqrt(satn) * tmp * tmp;
        }
    }
    m.u_satn[cur ^ 1][i] = satn;

    // ---- Flux_Infiltration (Element.cpp:271-303) ----
    double qi = 0., qex = 0.;
    {
        const double av = usf + m.net_prep[i];
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
        const double KV = m.KsatV[i];
        if (!(ugw > aq - infD && uus < deficit)) {
            double grad = 0.;
            if (theta > ThR && !(uus <= K_EPSILON)) {
                grad = (theta - ThR) / (ThS * K_FC_RATIO - ThR);
                grad = rmax(grad, 0.);
            }
            if (!(infK <= 0. || KV <= 0.)) {
                const double ku = infK * satkr;
                qr = grad * ((ku * KV) * (deficit + ugw) / (deficit * KV + ugw * ku));  // meanHarmonic
            }
        }
    }
    const double q_rech = qr * fu_sub;

    // ---- own river segments (fun_Seg_surface/fun_Seg_sub) and Qe2r (PassValue) ----
    const double zs = m.z_surf[i], zb = m.z_bottom[i], dep = m.depression[i];
    double qe2r_surf = 0., qe2r_sub = 0.;
    {
        const int k0 = m.seg_off[i], k1 = m.seg_off[i + 1];
        double isf_seg = rmax(0., usf - q_infil + q_exfil);
        for (int k = k0; k < k1; k++) {
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
        dg.e_ic[i] = (MODE == 0) ? eic : m.e_ic[cur_e][i]; dg.u_satn[i] = satn; dg.eff_kh[i] = ekh;
        dg.qe2r_surf[i] = qe2r_surf; dg.qe2r_sub[i] = qe2r_sub;
    }
    if (i >= nown) return;    // seg-ghost element of a partition: vertical + segments only

    // ---- fun_Ele_surface / fun_Ele_sub over 3 edges (MD_ElementFlux.cpp:35-156) ----
    double sumsurf = qe2r_surf, sumsub = qe2r_sub;     // QeleSurfTot = Qe2r_Surf + sum_j (MD_f.cpp:68-72)
    bool nan_q = false;
    const double isf = usf < 0. ? 0. : usf;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const int nb = m.nabr[j * NEl + i];
        const double B = m.edge[j * NEl + i];
        double qsf = 0., qsb = 0.;
        if (nb >= 0) {
            // surface (Manning)
            double nsf = Y.sf(nb);
            if (MODE == 1) nsf = (nsf >= 0.) ? nsf : 0.;
            nsf = nsf < 0. ? 0. : nsf;
            const double zsn = m.z_surf[nb];
            const double d2n = m.dist2nabor[j * NEl + i];
            const double dh = (isf + zs) - (nsf + zsn);
            double ym = ((isf + zs) > (nsf + zsn)) ? ((isf > dep) ? isf : 0.) : ((nsf > dep) ? nsf : 0.);
            ym = rmin(ym, K_MAXYSURF);
            if (ym > 0.) {
                const double s = dh / d2n;
                if (s > 0 && isf <= 0) qsf = 0.;
                else if (s < 0 && nsf <= 0) qsf = 0.;
                else qsf = manning(ym * B, m.avg_rough[j * NEl + i], ym, s);
            }
            // subsurface (Darcy); neighbour effKH recomputed from its own state (loop A value)
            const int fn = m.eflags[nb];
            const double ugn = ugw_of<MODE>(m, Y, nb, (int)(int16_t)(fn & 0xffff));
            const double zbn = m.z_bottom[nb];
            const double dhg = (ugw + zb) - (ugn + zbn);
            double q = 0.;
            if (dhg > 0. && ugw <= 0.02) q = 0.;
            else if (dhg < 0. && ugn <= 0.02) q = 0.;
            else {
                const double ekn = eff_kh(ugn, m.aq[nb], m.macD[nb], m.macKsatH[nb], m.vAreaF[nb], m.KsatH[nb]);
                const double ymg = (rmax(ugw, 0.) + rmax(ugn, 0.)) * .5;
                const double grad = dhg / d2n;
                const double kmean = 0.5 * (ekh + ekn);
                q = kmean * grad * ymg * B;
            }
            qsb = q * fu_sub;
        } else if (!OPEN) {
            qsb = 0. * fu_sub;                     // Q = 0 for a closed boundary, times fu_Sub
        } else {
            if (isf > dep) {
                const double s = isf / m.dist2edge[j * NEl + i] * 0.5;
                if (s > 0.) qsf = sqrt(s) * cbrt(isf * isf * isf * isf * isf) * B / m.rough[i];
            }
            double q = 0.;
            if (ugw > dep * 10.) {
                const double grad = ugw / m.dist2edge[j * NEl + i] * 0.5;
                if (grad > 0.) q = ekh * grad;
            }
            qsb = q * fu_sub;
        }
        if (MODE == 0) nan_q |= (isnan(qsf) || isinf(qsf) || isnan(qsb) || isinf(qsb));
        sumsurf += qsf;
        sumsub += qsb;
        if (DIAG) { dg.qele_surf[j * NEl + i] = qsf; dg.qele_sub[j * NEl + i] = qsb; }
    }
    if (MODE == 0) report_w(m.err, nan_q, 0x01u, 0, i);

    // ---- f_applyDY element part (MD_f.cpp:88-131 / MD_f_omp.cpp:26-46) ----
    const double area = m.area[i];
    double dsf = m.net_prep[i] - q_infil + q_exfil - sumsurf / area - Es;
    double dus = q_infil - q_rech - Eu - Tu;
    double dgw = q_rech - q_exfil - sumsub / area - Eg - Tg;
    if (ibc > 0) dgw = 0;
    else if (ibc < 0) dgw += m.eqbc[-ibc] / area;
    if (iss == 1) dsf += 0.0 / area;          // QSS is never assigned (always 0)
    else if (iss == 2) dgw += 0.0 / area;
    const double sy = m.Sy[i];
    dus /= sy;
    dgw /= sy;
    dy[i] = dsf;
    dy[nown + i] = dus;
    dy[2 * nown + i] = dgw;
    if (DIAG) { dg.qele_surf_tot[i] = sumsurf; dg.qele_sub_tot[i] = sumsub; }
}

// ===================================================================================
// river kernel
// ===================================================================================

// River.cpp:49-62 updateRiver + River.hpp:115-127
__device__ __forceinline__ RivGeom riv_geom(const DevMesh &m, int r, double y) {
    const double w0 = m.riv_bw[r], s = m.riv_bankslope[r];
    RivGeom g;
    const double topw = y * s * 2.0 + w0;
    const double a = y * (w0 + y * s);
    const double ys = y * s;
    const double p = 2.0 * sqrt(y * y + ys * ys) + w0;
    const double eqw = 0.5 * ((y * s * 2.0 + w0) + w0);
    const double ta = eqw * m.riv_len[r];
    g.topw = (topw < 0.) ? 0. : topw;
    g.csarea = (a < 0.) ? 0. : a;
    g.csperem = (p < 0.) ? 0. : p;
    g.toparea = (ta < 0.) ? 0. : ta;
    return g;
}

// MD_RiverFlux.cpp:5-63 for reach r (non-lake); needs r's pre-BC geometry and post-BC stages
template <int MODE>
__device__ __forceinline__ double riv_down_flux(const DevMesh &m, const YView &Y, int r, double ur,
                                                const RivGeom &g) {
    const int d = m.riv_down[r];
    const double n = m.riv_avg_rough[r];
    if (d >= 0) {
        double ydraw;
        const double ud = uriv_of<MODE>(m, Y, d, &ydraw);
        const double smean = (m.riv_slope[r] + m.riv_slope[d]) * 0.5;
        const double s = ((ur - m.riv_depth[r]) - (ud - m.riv_depth[d])) / m.riv_d2down[r] + smean;
        const double R = (g.csperem <= K_ZERO) ? 0. : (g.csarea / g.csperem);
        return manning(g.csarea, n, R, s);
    } else if (d >= -3) {
        const double s = m.riv_slope[r] + ur * 2. / m.riv_len[r];
        const double R = (g.csperem <= 0.) ? 0. : (g.csarea / g.csperem);
        return manning(g.csarea, n, R, s);
    }
    return g.csarea * sqrt(K_GRAV * ur) * 60.;     // -4: critical depth
}

template <int MODE, bool DIAG>
__global__ void __launch_bounds__(256)
shud_riv_kernel(DevMesh m, YView Y, double *__restrict__ dy, DevDiag dg) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= Y.n_own_riv) return;
    double yg;
    const double ur = uriv_of<MODE>(m, Y, r, &yg);
    const RivGeom g = riv_geom(m, r, yg);
    const double qdown = riv_down_flux<MODE>(m, Y, r, ur, g);
    // junction: QrivUp[down] += -QrivDown[i], i ascending (MD_f.cpp:236-240)
    double qup = 0.;
    for (int k = m.up_off[r], k1 = m.up_off[r + 1]; k < k1; k++) {
        const int u = m.up_idx[k];
        double yu;
        const double uu = uriv_of<MODE>(m, Y, u, &yu);
        const RivGeom gu = riv_geom(m, u, yu);
        qup += -riv_down_flux<MODE>(m, Y, u, uu, gu);
    }
    // segment sums, ascending reference segment order (MD_f.cpp:228-235)
    double qsurf = 0., qsub = 0.;
    for (int k = m.rseg_off[r], k1 = m.rseg_off[r + 1]; k < k1; k++) {
        const int p = m.rseg_pos[k];
        qsurf += m.qseg_surf[p];
        qsub += m.qseg_sub[p];
    }
    const int bc = m.riv_bc[r];
    const double qbc = (bc < 0) ? m.rqbc[-bc] : 0.0;
    double d;
    if (bc > 0) d = 0.;
    else if (MODE == 0) {   // MD_f.cpp:162-166
        d = (-qup - qsurf - qsub - qdown + qbc) / m.riv_len[r];
        if (d < -1. * g.csarea) d = -1. * g.csarea;
        if (d == 0.) d = 0.;                                         // fun_dAtodY functions.hpp:141-153
        else {
            const double s = m.riv_bankslope[r];
            if (fabs(s) < K_EPS_SLOPE) d = d / g.topw;
            else {                                                   // Quadratic functions.hpp:125-139
                const double sa = fabs(s);
                const double cc = g.topw * g.topw + 4 * sa * d;
                d = (cc < K_ZERO) ? -1. * g.topw / (2. * sa) : (-g.topw + sqrt(cc)) / (2 * sa);
            }
        }
    } else {                // MD_f_omp.cpp:59
        d = (-qup - qsurf - qsub - qdown + qbc) / g.toparea;
    }
    dy[3 * Y.n_own + r] = d;
    if (DIAG) { dg.qriv_down[r] = qdown; dg.qriv_up[r] = qup; dg.qriv_surf[r] = qsurf; dg.qriv_sub[r] = qsub; }
}

// gather owned states that peers hold as ghosts: ele AoS [sf,us,gw] records, then reaches
__global__ void __launch_bounds__(256)
shud_pack_kernel(const double *__restrict__ y, int n_own, int n_own_riv, const int *__restrict__ eidx,
                 int ne, const int *__restrict__ ridx, int nr, double *__restrict__ ebuf,
                 double *__restrict__ rbuf) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ne) {
        const int i = eidx[t];
        ebuf[3 * t] = y[i];
        ebuf[3 * t + 1] = y[n_own + i];
        ebuf[3 * t + 2] = y[2 * n_own + i];
    } else if (t < ne + nr) {
        const int k = t - ne;
        rbuf[k] = y[3 * n_own + ridx[k]];
    }
}

// ---- launchers ----
template <int MODE, bool OPEN, bool DIAG>
static void launch_ele(const DevMesh &m, const YView &Y, double *dy, int n_compute, int cur, int cur_e,
                       const DevDiag &dg, hipStream_t s) {
    const int bs = 256;
    if (n_compute <= 0) return;
    hipLaunchKernelGGL((shud_ele_kernel<MODE, OPEN, DIAG>), dim3((n_compute + bs - 1) / bs), dim3(bs), 0, s,
                       m, Y, dy, n_compute, cur, cur_e, dg);
}
template <int MODE, bool DIAG>
static void launch_riv(const DevMesh &m, const YView &Y, double *dy, const DevDiag &dg, hipStream_t s) {
    const int bs = 256;
    if (Y.n_own_riv <= 0) return;
    hipLaunchKernelGGL((shud_riv_kernel<MODE, DIAG>), dim3((Y.n_own_riv + bs - 1) / bs), dim3(bs), 0, s,
                       m, Y, dy, dg);
}

void launch_element_kernel(const DevMesh &m, const YView &Y, double *dy, int n_compute, int cur, int cur_e,
                           int mode, bool open, bool diag, const DevDiag &dg, hipStream_t s) {
#define L(MO, OP, DI) launch_ele<MO, OP, DI>(m, Y, dy, n_compute, cur, cur_e, dg, s)
    if (mode == 0) {
        if (open) { if (diag) L(0, true, true); else L(0, true, false); }
        else { if (diag) L(0, false, true); else L(0, false, false); }
    } else {
        if (open) { if (diag) L(1, true, true); else L(1, true, false); }
        else { if (diag) L(1, false, true); else L(1, false, false); }
    }
#undef L
}
void launch_river_kernel(const DevMesh &m, const YView &Y, double *dy, int mode, bool diag,
                         const DevDiag &dg, hipStream_t s) {
    if (mode == 0) { if (diag) launch_riv<0, true>(m, Y, dy, dg, s); else launch_riv<0, false>(m, Y, dy, dg, s); }
    else { if (diag) launch_riv<1, true>(m, Y, dy, dg, s); else launch_riv<1, false>(m, Y, dy, dg, s); }
}
void launch_pack_kernel(const double *y, int n_own, int n_own_riv, const int *eidx, int ne, const int *ridx,
                        int nr, double *ebuf, double *rbuf, hipStream_t s) {
    const int n = ne + nr;
    if (n <= 0) return;
    hipLaunchKernelGGL(shud_pack_kernel, dim3((n + 255) / 256), dim3(256), 0, s, y, n_own, n_own_riv, eidx, ne,
                       ridx, nr, ebuf, rbuf);
}

}  // namespace shud
