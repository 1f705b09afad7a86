// shud_et.hip — ET-step prelude on the device (C-ABI include/shud_et.h).
//
// One thread per element: tReadForcing (src/ModelData/MD_ET.cpp:21-281) then ET() (:282-341) fused, writing
// the RHS handle's step inputs in place (SoA staging + the packed records when the handle is packed).  The
// leaf equations restate src/Equations/is_sm_et.hpp / is_sm_et.cpp / Equations.hpp / functions.hpp, cited
// inline; operation order as in the reference (-ffp-contract=off), the reference's own min/max.
// Once per ET step, ~200 B/element: HBM-bound, no LDS needed (the per-step station/LAI/MF rows and the
// TSR solar samples are a few KB, read through the scalar cache).
#include <hip/hip_runtime.h>

#include "shud_et_dev.h"
#include "shud_physics.h"

namespace shud {

// ---- leaf equations ----
#define ET_NA_VALUE (-9999.0)
__device__ __forceinline__ bool ifequal(double x, double y) { return fabs(x - y) < K_ZERO; }   // functions.hpp:155-161
// Equations.hpp:65-72 (dTdZ = 0.0065, Macros.hpp:50)
__device__ __forceinline__ double temperature_on_elevation(double t, double zi, double zt) {
    if (ifequal(zi, ET_NA_VALUE) || ifequal(zt, ET_NA_VALUE)) return t;
    return t + (zt - zi) * 0.0065;
}
// functions.hpp:191-201
__device__ __forceinline__ double frozen_fraction(double T, double high, double low) {
    if (T > high) return 0;
    if (T < low) return 1;
    const double x = (high - T) / (high - low);
    return rmin(1.0, rmax(x, 0.0));
}
// is_sm_et.cpp:56-62 (SecADay = 86400, Macros.hpp:43)
__device__ __forceinline__ double pet_pm_openwater(double Delta, double Gamma, double lambda, double Rad, double ed,
                                                   double U2) {
    double ETp = (Delta * Rad * 86400. + Gamma * 6.43 * (1.0 + 0.536 * U2) * ed) / (Delta + Gamma);
    ETp = ETp / lambda;
    ETp = ETp * 0.001 / 86400.;
    return ETp;
}
// is_sm_et.cpp:31-55 (Cp = 1.013e-3, Macros.hpp:72)
__device__ __forceinline__ double pet_penman_monteith(double Rad, double rho, double ed, double Delta, double r_a,
                                                      double r_s, double Gamma, double lambda) {
    const double E_rad = Delta * Rad;
    const double E_air = rho * 1.013e-3 * ed / r_a;
    const double r_sa = r_s / r_a;
    double ETp = (E_rad + E_air) / (Delta + Gamma * (1 + r_sa));
    ETp = ETp / lambda;
    ETp = ETp * 0.001;
    return ETp;
}
// is_sm_et.hpp:119-140 (VON_KARMAN = 0.4, Macros.hpp:70)
__device__ __forceinline__ double aerodynamic_resistance(double Uz, double hc, double Z_u, double Z_e) {
    const double d = 0.67 * hc;
    const double Z_om = 0.123 * hc;
    const double Z_ov = 0.0123 * hc;
    return log(fabs(Z_u - d) / Z_om) * log(fabs(Z_e - d) / (Z_ov)) / (0.4 * 0.4 * Uz);
}

// ---- the fused prelude kernel ----
__global__ void __launch_bounds__(256) shud_et_kernel(DevEt e, EtStepDev s, DevErr *err) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.ne) return;
    const int idx = e.iforc[i];
    const double *st = s.station + 6 * idx;

    // ---- tReadForcing (MD_ET.cpp:21-281) ----
    double prcp = st[1] * s.cPrep;                                            // :52
    const double t0 = st[2];
    const double temp = temperature_on_elevation(t0, e.z_surf[i], s.station_z[idx]) + s.cTemp;   // :54
    const double lai = s.lai_row[e.ilc[i]] * s.cLAItsd;                       // :55
    const double mf = s.mf_row[e.imf[i]] * s.cMF / 1440.;                     // :57
    const double dswrf_h = st[5];                                             // :61
    double dswrf_t = dswrf_h, factor = 1.0;
    if (s.terrain) {                                                          // :64-200
        if (s.tsr_mode == 1) {
            factor = 0.0;
        } else {
            if (s.tsr_mode == 3) {                                            // :140-196 (new forcing interval)
                double num = 0.0;
                const double cap = s.rad_factor_cap, cosz_min = s.rad_cosz_min;
                if (s.tsr_den > 0.0 && s.tsr_n > 0) {
                    const double nx = e.nx[i], ny = e.ny[i], nz = e.nz[i];
                    for (int k = 0; k < s.tsr_n; k++) {
                        const double wdt = s.tsr_wdt[k];
                        if (!(wdt > 0.0)) continue;
                        const double sx = s.tsr_sx[k], sy = s.tsr_sy[k], sz = s.tsr_sz[k];
                        const double cosi = nx * sx + ny * sy + nz * sz;
                        if (!(cosi > 0.0) || !isfinite(cosi)) continue;
                        double denom = sz;
                        if (denom < cosz_min) denom = cosz_min;
                        if (!(denom > 0.0) || !isfinite(denom)) continue;
                        double fk = cosi / denom;
                        if (!isfinite(fk) || !(fk > 0.0)) continue;
                        if (fk > cap) fk = cap;
                        num += wdt * fk;
                    }
                }
                double feff = 0.0;
                if (s.tsr_den > 0.0) {
                    feff = num / s.tsr_den;
                    if (!isfinite(feff) || !(feff > 0.0)) feff = 0.0;
                    if (feff > s.rad_factor_cap) feff = s.rad_factor_cap;
                }
                e.tsr_factor[i] = feff;
            }
            factor = e.tsr_factor[i];
        }
        dswrf_t = dswrf_h * factor;
    }
    double rn = (s.radiation_input_mode == 1) ? dswrf_t : dswrf_t * (1 - e.albedo[i]);   // :208-214
    const double wind = fabs(st[4]) + 0.001;                                  // :215
    double rh = st[3];
    prcp = prcp * 0.001 / 1440.;                                              // :221
    rn = rn * 1.0e-6;                                                         // :223
    rh = rmin(rmax(rh, 0.01), 1.0);                                           // :229 (CONST_RH)
    const double P = e.fixp[i];
    const double lambda = 2.501 - 0.002361 * temp;                            // LatentHeat, is_sm_et.hpp:70-75
    const double Gamma = 0.0016286 * P / lambda;                              // is_sm_et.hpp:97-102
    const double es = 0.6108 * exp(17.27 * temp / (temp + 237.3));            // is_sm_et.hpp:103-106
    const double ea = es * rh;
    const double ed = es - ea;
    const double tt = (temp + 237.3);                                         // is_sm_et.hpp:163-167
    const double Delta = 4098. * es / (tt * tt);
    const double rho = 3.486 * P / (275. + temp);                             // is_sm_et.hpp:154-162
    double G;                                                                 // :238-247
    if (e.ilake[i] > 0) G = 0.;
    else if (lai > 0) G = 0.4 * exp(-0.5 * lai) * rn;
    else G = 0.1 * rn;
    const double RG = rn - G;
    // WindProfile(2.0, wind, windH, 0., ROUGHNESS_WATER = 0.00137), is_sm_et.hpp:149-152
    const double U2 = wind * log((2.0 - 0.) / 0.00137) / log((e.windh[i] - 0.) / 0.00137);
    const double qpet = s.cETP * pet_pm_openwater(Delta, Gamma, lambda, RG, ed, U2) * 60.;   // :251
    double qptr, etp;
    if (e.ilake[i] > 0 || lai <= 0.) {                                        // :252-258
        qptr = s.cETP * 0.;
        etp = qpet;
    } else {                                                                  // :259-279
        const double hc = lai * 0.5;
        const double Zm = hc * 1.3333;
        const double ra = aerodynamic_resistance(wind, hc, Zm, Zm);
        // CheckNonZero (functions.cpp:155-161) -> myexit(ERRNAN = 10)
        report_w(err, ra <= 0.0 || isnan(ra) || isinf(ra) || fabs(ra - ET_NA_VALUE) < K_ZERO, 0x20u, 5, i);
        const double rs = 200. / lai;                                         // BulkSurfaceResistance(lai)
        qptr = s.cETP * pet_penman_monteith(RG, rho, ed, Delta, ra, rs, Gamma, lambda) * 60.;
        const double vf = e.vegf[i];
        etp = qptr * vf + qpet * (1. - vf);
        report_w(err, isnan(qptr) || isinf(qptr), 0x40u, 6, i);              // CheckNANi(qPotTran)
    }

    // ---- ET() (MD_ET.cpp:282-341) ----
    const double DT = s.t_next - s.t;
    const double T = temp;
    double snStg = e.y_snow[i];
    const double snFrac = frozen_fraction(T, 1.0, -3.0);                      // Train, Tsnow (Macros.hpp:59-60)
    double fu_sub = 1., fu_surf = 1.;
    if (s.cryosphere) {                                                       // :301-311, AccTemperature.hpp
        const int ne = e.ne;
        // surface accumulator
        double ta = e.tacc_surf[i] + T;
        double acc = e.acc_surf[i];
        if (s.push_day) {
            const double v = ta / (double)s.n_of_day;
            e.ring_surf[(size_t)s.surf_tail * ne + i] = v;
            acc += v;
            if (s.surf_pop) acc -= e.ring_surf[(size_t)s.surf_head * ne + i];
            ta = 0.;
        }
        e.tacc_surf[i] = ta;
        e.acc_surf[i] = acc;
        const double ta_surf = acc / (double)s.surf_size;
        ta = e.tacc_sub[i] + T;
        acc = e.acc_sub[i];
        if (s.push_day) {
            const double v = ta / (double)s.n_of_day;
            e.ring_sub[(size_t)s.sub_tail * ne + i] = v;
            acc += v;
            if (s.sub_pop) acc -= e.ring_sub[(size_t)s.sub_head * ne + i];
            ta = 0.;
        }
        e.tacc_sub[i] = ta;
        e.acc_sub[i] = acc;
        const double ta_sub = acc / (double)s.sub_size;
        fu_sub = 1. - frozen_fraction(ta_sub, s.ft_sub_max, s.ft_sub_min);
        fu_surf = 1. - frozen_fraction(ta_surf, s.ft_surf_max, s.ft_surf_min);
    }
    const double snAcc = snFrac * prcp;
    double snMelt = (T > 0.0 ? (T - 0.0) * mf : 0.);                          // To = 0 (Macros.hpp:61)
    snMelt = rmin(rmax(0., snStg / DT), rmax(0., snMelt));
    snStg += (snAcc - snMelt) * DT;
    const double vgFrac = e.vegf[i];
    double icStg = (vgFrac > K_ZERO) ? (e.y_is[i] / vgFrac) : 0.0;
    double icAcc, icEvap;
    if (lai > K_ZERO) {
        const double icMax = s.cISmax * 0.0002 * lai;                         // IC_MAX (Macros.hpp:64)
        icAcc = rmin(prcp - snAcc, rmax(0., (icMax - icStg) / DT));
        icEvap = rmin(rmax(0., icStg / DT), qpet);
    } else {
        icAcc = 0.;
        icEvap = 0.;
    }
    icStg += (icAcc - icEvap) * DT;
    const double eic = icEvap * vgFrac;
    const double netp = (1. - snFrac) * prcp + snMelt - icAcc * vgFrac;
    e.y_is[i] = icStg * vgFrac;
    e.y_snow[i] = snStg;

    // ---- outputs: diagnostics + the RHS step inputs (single-use streams: non-temporal stores) ----
#define STN(p, v) __builtin_nontemporal_store((double)(v), &(p)[i])
    STN(e.t_prcp, prcp); STN(e.t_temp, temp); STN(e.t_lai, lai); STN(e.t_mf, mf); STN(e.t_rn, rn);
    STN(e.t_wind, wind); STN(e.t_rh, rh); STN(e.rn_factor, factor);
    STN(e.rn_h, dswrf_h); STN(e.rn_t, dswrf_t);
    STN(e.q_prep, prcp); STN(e.q_pet, qpet); STN(e.q_ptr, qptr); STN(e.q_etp, etp); STN(e.q_netp, netp);
    STN(e.q_eic, eic); STN(e.fu_surf, fu_surf); STN(e.fu_sub, fu_sub);
#undef STN
    if (s.packed) {                                   // the element kernel's records (shud_dev.h DevPacked)
        s.s_np[i] = make_double2(netp, qpet);
        s.s_tl[i] = make_double2(qptr, etp);
        s.sfl[i] = (s.sfl[i] & 0x7fffffff) | (lai > K_ZERO ? (int)0x80000000u : 0);   // f_etFlux's LAI test
        if (s.cryosphere) s.s_fu[i] = make_double2(fu_surf, fu_sub);
        s.cs_cur[i].y = eic;
    }
}

void launch_et_kernel(const DevEt &e, const EtStepDev &s, DevErr *err, hipStream_t st) {
    if (e.ne <= 0) return;
    hipLaunchKernelGGL(shud_et_kernel, dim3((e.ne + 255) / 256), dim3(256), 0, st, e, s, err);
}

}  // namespace shud
