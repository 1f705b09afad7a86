/* shud_oracle_et.c — CPU restatement of SHUD's ET-step prelude (TEST INFRASTRUCTURE ONLY: the checker
 * for shud_et_step, include/shud_et.h; never linked into the product library).
 *
 * Restates, loop by loop, src/ModelData/MD_ET.cpp:
 *   tReadForcing(t, i)   :21-281  (forcing rows, TSR factor cache per element, PET)
 *   ET(t, tnext)         :282-341 (snow, interception, cryosphere accumulators)
 * with the leaf equations of src/Equations/is_sm_et.hpp/.cpp, Equations.hpp:65-72, functions.hpp:191-201 and
 * the per-element _AccTemp queues of src/classes/AccTemperature.hpp (each element keeps its own queue here,
 * as the reference does; the device keeps the shared bookkeeping once).  glibc libm, -ffp-contract=off.
 * Parity unpinned (no reference build): see DESIGN.md §2.
 * Deviation, flagged: _AccTemp::ACC is never initialised by the reference's constructor
 * (AccTemperature.hpp:27,41-45); it starts at 0.0 here and on the device. */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "shud_et.h"

#define NA_VALUE (-9999.0)
#define ZERO 1.0e-10
#define CONST_RH 0.01
#define ROUGHNESS_WATER 0.00137
#define IC_MAX 0.0002
#define Train 1.0
#define Tsnow (-3.0)
#define To 0.0
#define dTdZ 0.0065
#define SecADay 86400
#define VON_KARMAN 0.4
#define Cp 1.013e-3
#define SWNET 1

static inline double rmin(double a, double b) { return (a > b ? b : a); }   /* functions.hpp:117-123 */
static inline double rmax(double a, double b) { return (a < b ? b : a); }
static int ifequal(double x, double y) { return fabs(x - y) < ZERO; }      /* functions.hpp:155-161 */

/* Equations.hpp:65-72 */
static double TemperatureOnElevation(double t, double Zi, double Zt) {
    if (ifequal(Zi, NA_VALUE) || ifequal(Zt, NA_VALUE)) return t;
    return t + (Zt - Zi) * dTdZ;
}
/* functions.hpp:191-201 */
static double FrozenFraction(double T, double high, double low) {
    double x;
    if (T > high) return 0;
    else if (T < low) return 1;
    x = (high - T) / (high - low);
    return rmin(1.0, rmax(x, 0.0));
}
/* is_sm_et.hpp */
static double LatentHeat(double Temp) { return 2.501 - 0.002361 * Temp; }
static double PsychrometricConstant(double Pressure, double lambda) { return 0.0016286 * Pressure / lambda; }
static double VaporPressure_Sat(double T) { return 0.6108 * exp(17.27 * T / (T + 237.3)); }
static double SlopeSatVaporPressure(double Temp, double ES) { double tt = (Temp + 237.3); return 4098. * ES / (tt * tt); }
static double AirDensity(double P, double Temp) { return 3.486 * P / (275. + Temp); }
static double WindProfile(double Zx, double Um, double Zm, double d, double Z0) {
    return Um * log((Zx - d) / Z0) / log((Zm - d) / Z0);
}
static double AerodynamicResistance(double Uz, double hc, double Z_u, double Z_e) {
    double r_a, d, Z_om, Z_ov;
    d = 0.67 * hc;
    Z_om = 0.123 * hc;
    Z_ov = 0.0123 * hc;
    r_a = log(fabs(Z_u - d) / Z_om) * log(fabs(Z_e - d) / (Z_ov)) / (VON_KARMAN * VON_KARMAN * Uz);
    return r_a;
}
static double BulkSurfaceResistance(double lai) { return 200. / lai; }
/* is_sm_et.cpp:31-62 */
static double PET_Penman_Monteith(double Rad, double rho, double ed, double Delta, double r_a, double r_s,
                                  double Gamma, double lambda) {
    double E_rad, E_air, r_sa;
    E_rad = Delta * Rad;
    E_air = rho * Cp * ed / r_a;
    r_sa = r_s / r_a;
    double ETp = (E_rad + E_air) / (Delta + Gamma * (1 + r_sa));
    ETp = ETp / lambda;
    ETp = ETp * 0.001;
    return ETp;
}
static double PET_PM_openwater(double Delta, double Gamma, double lambda, double Rad, double ed, double U2) {
    double ETp = (Delta * Rad * SecADay + Gamma * 6.43 * (1.0 + 0.536 * U2) * ed) / (Delta + Gamma);
    ETp = ETp / lambda;
    ETp = ETp * 0.001 / SecADay;
    return ETp;
}

/* AccTemperature.hpp: one queue per element */
typedef struct {
    double Time_start, T_AccDay, ACC;
    int N_of_day, MaxLen;
    double *q;          /* ring of MaxLen + 1 */
    int head, size, cap;
} AccTemp;
static void acc_init(AccTemp *a, int maxlen) {
    a->Time_start = -9999.; a->T_AccDay = 0.; a->ACC = 0.; a->N_of_day = 0; a->MaxLen = maxlen;
    a->cap = maxlen + 1; a->q = (double *)calloc(a->cap, sizeof(double)); a->head = 0; a->size = 0;
}
static void acc_push_value(AccTemp *a, double x) {                       /* AccTemperature.hpp:27-36 */
    a->q[(a->head + a->size) % a->cap] = x; a->size++;
    a->ACC += x;
    if (a->size > a->MaxLen) {
        a->ACC -= a->q[a->head];
        a->head = (a->head + 1) % a->cap; a->size--;
    }
}
static void acc_push(AccTemp *a, double x, double tnow) {               /* AccTemperature.hpp:48-58 */
    a->T_AccDay += x;
    a->N_of_day++;
    if ((tnow - a->Time_start) >= 1440.) {
        acc_push_value(a, a->T_AccDay / a->N_of_day);
        a->T_AccDay = 0.;
        a->N_of_day = 0;
        a->Time_start = tnow;
    }
}
static double acc_get(const AccTemp *a) { return a->ACC / a->size; }

typedef struct OracleEt {
    int NE;
    int *iforc, *ilc, *imf, *ilake;
    double *z_surf, *albedo, *fixp, *windh, *vegf, *nx, *ny, *nz;
    ShudEtParams par;
    double *t_prcp, *t_temp, *t_lai, *t_mf, *t_rn, *t_wind, *t_rh, *qElePrep, *qPotEvap, *qPotTran, *qEleETP;
    double *qEleNetPrep, *qEleE_IC, *yEleIS, *yEleSnow, *fu_Surf, *fu_Sub, *rn_factor, *tsr_factor;
    int *tsr_has;     /* tsr_factor_bucket[i] == current bucket */
    AccTemp *acc_surf, *acc_sub;
    int exit_code, exit_index;
} OracleEt;

static double *dupd(const double *p, int n) {
    double *q = (double *)calloc(n ? n : 1, sizeof(double));
    if (p) memcpy(q, p, sizeof(double) * n);
    return q;
}
static int *dupi(const int32_t *p, int n, int fill) {
    int *q = (int *)malloc(sizeof(int) * (n ? n : 1));
    for (int i = 0; i < n; i++) q[i] = p ? p[i] : fill;
    return q;
}

OracleEt *oracle_et_create(const ShudEtMeshSoA *m, const ShudEtParams *p) {
    OracleEt *E = (OracleEt *)calloc(1, sizeof(OracleEt));
    int n = m->num_ele;
    E->NE = n;
    E->par = *p;
    E->iforc = dupi(m->iforc, n, 0); E->ilc = dupi(m->ilc, n, 1); E->imf = dupi(m->imf, n, 1);
    E->ilake = dupi(m->ilake, n, 0);
    E->z_surf = dupd(m->z_surf, n); E->albedo = dupd(m->albedo, n); E->fixp = dupd(m->fix_pressure, n);
    E->windh = dupd(m->wind_h, n); E->vegf = dupd(m->veg_frac, n);
    E->nx = dupd(m->nx, n); E->ny = dupd(m->ny, n); E->nz = dupd(m->nz, n);
    double **arrs[] = {&E->t_prcp, &E->t_temp, &E->t_lai, &E->t_mf, &E->t_rn, &E->t_wind, &E->t_rh, &E->qElePrep,
                       &E->qPotEvap, &E->qPotTran, &E->qEleETP, &E->qEleNetPrep, &E->qEleE_IC, &E->yEleIS,
                       &E->yEleSnow, &E->fu_Surf, &E->fu_Sub, &E->rn_factor, &E->tsr_factor};
    for (size_t k = 0; k < sizeof(arrs) / sizeof(arrs[0]); k++) *arrs[k] = dupd(NULL, n);
    E->tsr_has = (int *)calloc(n ? n : 1, sizeof(int));
    E->acc_surf = (AccTemp *)calloc(n ? n : 1, sizeof(AccTemp));
    E->acc_sub = (AccTemp *)calloc(n ? n : 1, sizeof(AccTemp));
    for (int i = 0; i < n; i++) {
        acc_init(&E->acc_surf[i], p->ft_surf_day);
        acc_init(&E->acc_sub[i], p->ft_sub_day);
    }
    return E;
}

void oracle_et_set_state(OracleEt *E, const double *y_is, const double *y_snow) {
    if (y_is) memcpy(E->yEleIS, y_is, sizeof(double) * E->NE);
    if (y_snow) memcpy(E->yEleSnow, y_snow, sizeof(double) * E->NE);
}

/* MD_ET.cpp:21-281 for element i; returns 10 on myexit(ERRNAN) */
static int tReadForcing(OracleEt *E, const ShudEtForcing *f, int i) {
    const ShudEtParams *gc = &E->par;
    int idx = E->iforc[i];
    const double *row = f->station + 6 * idx;
    double etp, ra, rs, t0, hc, U2, Uz, Zmeasure, lai, GroundHeatFlux, RG;
    E->t_prcp[i] = row[1] * gc->cPrep;
    t0 = row[2];
    E->t_temp[i] = TemperatureOnElevation(t0, E->z_surf[i], f->station_z[idx]) + gc->cTemp;
    E->t_lai[i] = f->lai_row[E->ilc[i]] * gc->cLAItsd;
    lai = E->t_lai[i];
    E->t_mf[i] = f->mf_row[E->imf[i]] * gc->cMF / 1440.;
    const double dswrf_h = row[5];
    double dswrf_t = dswrf_h, factor = 1.0;
    if (gc->terrain_radiation) {
        if (f->tsr_mode == SHUD_TSR_NO_TIME) {
            factor = 0.0;
        } else {
            if (f->tsr_mode == SHUD_TSR_RECOMPUTE) E->tsr_has[i] = 0;     /* new bucket (:60-136) */
            if (!E->tsr_has[i]) {                                         /* :140-196 */
                double num = 0.0;
                const double cap = gc->rad_factor_cap, cosz_min = gc->rad_cosz_min;
                if (f->tsr_den > 0.0 && f->tsr_n > 0) {
                    const int n = f->tsr_n;
                    const double nx = E->nx[i], ny = E->ny[i], nz = E->nz[i];
                    for (int k = 0; k < n; k++) {
                        const double wdt = f->tsr_wdt[k];
                        if (!(wdt > 0.0)) continue;
                        const double sx = f->tsr_sx[k], sy = f->tsr_sy[k], sz = f->tsr_sz[k];
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
                if (f->tsr_den > 0.0) {
                    feff = num / f->tsr_den;
                    if (!isfinite(feff) || !(feff > 0.0)) feff = 0.0;
                    if (feff > gc->rad_factor_cap) feff = gc->rad_factor_cap;
                }
                E->tsr_factor[i] = feff;
                E->tsr_has[i] = 1;
            }
            factor = E->tsr_factor[i];
        }
        dswrf_t = dswrf_h * factor;
    }
    E->rn_factor[i] = factor;
    if (gc->radiation_input_mode == SWNET) E->t_rn[i] = dswrf_t;
    else E->t_rn[i] = dswrf_t * (1 - E->albedo[i]);
    Uz = E->t_wind[i] = (fabs(row[4]) + 0.001);
    E->t_rh[i] = row[3];
    E->t_prcp[i] = E->t_prcp[i] * 0.001 / 1440.;
    E->t_rn[i] = E->t_rn[i] * 1.0e-6;
    E->t_rh[i] = rmin(rmax(E->t_rh[i], CONST_RH), 1.0);
    E->qElePrep[i] = E->t_prcp[i];
    double lambda = LatentHeat(E->t_temp[i]);
    double Gamma = PsychrometricConstant(E->fixp[i], lambda);
    double es = VaporPressure_Sat(E->t_temp[i]);
    double ea = es * E->t_rh[i];
    double ed = es - ea;
    double Delta = SlopeSatVaporPressure(E->t_temp[i], es);
    double rho = AirDensity(E->fixp[i], E->t_temp[i]);
    if (E->ilake[i] > 0) {
        GroundHeatFlux = 0.;
        RG = E->t_rn[i];
    } else {
        if (lai > 0) GroundHeatFlux = 0.4 * exp(-0.5 * lai) * E->t_rn[i];
        else GroundHeatFlux = 0.1 * E->t_rn[i];
    }
    RG = E->t_rn[i] - GroundHeatFlux;
    U2 = WindProfile(2.0, E->t_wind[i], E->windh[i], 0., ROUGHNESS_WATER);
    E->qPotEvap[i] = gc->cETP * PET_PM_openwater(Delta, Gamma, lambda, RG, ed, U2) * 60.;
    if (E->ilake[i] > 0) {
        E->qPotTran[i] = gc->cETP * 0.;
        etp = E->qPotEvap[i];
    } else if (lai <= 0.) {
        E->qPotTran[i] = gc->cETP * 0.;
        etp = E->qPotEvap[i];
    } else {
        hc = lai * 0.5;
        Zmeasure = hc * 1.3333;
        ra = AerodynamicResistance(Uz, hc, Zmeasure, Zmeasure);
        if (ra <= 0.0 || isnan(ra) || isinf(ra) || fabs(ra - NA_VALUE) < ZERO) return 10;   /* CheckNonZero */
        rs = BulkSurfaceResistance(lai);
        E->qPotTran[i] = gc->cETP * PET_Penman_Monteith(RG, rho, ed, Delta, ra, rs, Gamma, lambda) * 60.;
        etp = E->qPotTran[i] * E->vegf[i] + E->qPotEvap[i] * (1. - E->vegf[i]);
        if (isnan(E->qPotTran[i]) || isinf(E->qPotTran[i])) return 11;          /* CheckNANi -> 10 */
    }
    E->qEleETP[i] = etp;
    return 0;
}

/* updateforcing's tReadForcing loop (MD_ET.cpp:14-20) then ET() (:282-341); returns the exit code */
int oracle_et_step(OracleEt *E, const ShudEtForcing *f) {
    E->exit_code = 0; E->exit_index = -1;
    for (int i = 0; i < E->NE; i++) {
        int c = tReadForcing(E, f, i);
        if (c) { E->exit_code = 10; E->exit_index = i; return 10; }
    }
    const ShudEtParams *gc = &E->par;
    double T, LAI, MF, prcp, snFrac, snAcc, snMelt, snStg, icAcc, icEvap, icStg, icMax, vgFrac;
    double DT_min = f->t_next - f->t, ta_surf, ta_sub;
    for (int i = 0; i < E->NE; i++) {
        T = E->t_temp[i];
        prcp = E->t_prcp[i];
        MF = E->t_mf[i];
        snStg = E->yEleSnow[i];
        snFrac = FrozenFraction(T, Train, Tsnow);
        if (gc->cryosphere) {
            acc_push(&E->acc_surf[i], T, f->t);
            acc_push(&E->acc_sub[i], T, f->t);
            ta_surf = acc_get(&E->acc_surf[i]);
            ta_sub = acc_get(&E->acc_sub[i]);
            E->fu_Sub[i] = 1. - FrozenFraction(ta_sub, gc->ft_sub_max, gc->ft_sub_min);
            E->fu_Surf[i] = 1. - FrozenFraction(ta_surf, gc->ft_surf_max, gc->ft_surf_min);
        } else {
            E->fu_Sub[i] = 1.;
            E->fu_Surf[i] = 1.;
        }
        snAcc = snFrac * prcp;
        snMelt = (T > To ? (T - To) * MF : 0.);
        snMelt = rmin(rmax(0., snStg / DT_min), rmax(0., snMelt));
        snStg += (snAcc - snMelt) * DT_min;
        LAI = E->t_lai[i];
        vgFrac = E->vegf[i];
        icStg = (vgFrac > ZERO) ? (E->yEleIS[i] / vgFrac) : 0.0;
        if (LAI > ZERO) {
            icMax = gc->cISmax * IC_MAX * LAI;
            icAcc = rmin(prcp - snAcc, rmax(0., (icMax - icStg) / DT_min));
            icEvap = rmin(rmax(0., icStg / DT_min), E->qPotEvap[i]);
        } else {
            icAcc = 0.;
            icEvap = 0.;
        }
        icStg += (icAcc - icEvap) * DT_min;
        E->yEleIS[i] = icStg * vgFrac;
        E->yEleSnow[i] = snStg;
        E->qEleE_IC[i] = icEvap * vgFrac;
        E->qEleNetPrep[i] = (1. - snFrac) * prcp + snMelt - icAcc * vgFrac;
    }
    return 0;
}

int oracle_et_exit_index(OracleEt *E) { return E->exit_index; }

static void cpo(double *dst, const double *src, int n) { if (dst) memcpy(dst, src, sizeof(double) * n); }
void oracle_et_get(OracleEt *E, ShudEtOut *o) {
    int n = E->NE;
    cpo(o->t_prcp, E->t_prcp, n); cpo(o->t_temp, E->t_temp, n); cpo(o->t_lai, E->t_lai, n);
    cpo(o->t_mf, E->t_mf, n); cpo(o->t_rn, E->t_rn, n); cpo(o->t_wind, E->t_wind, n); cpo(o->t_rh, E->t_rh, n);
    cpo(o->qEleprep, E->qElePrep, n); cpo(o->qPotEvap, E->qPotEvap, n); cpo(o->qPotTran, E->qPotTran, n);
    cpo(o->qEleETP, E->qEleETP, n); cpo(o->qEleNetPrep, E->qEleNetPrep, n); cpo(o->qEleE_IC, E->qEleE_IC, n);
    cpo(o->yEleIS, E->yEleIS, n); cpo(o->yEleSnow, E->yEleSnow, n); cpo(o->fu_surf, E->fu_Surf, n);
    cpo(o->fu_sub, E->fu_Sub, n); cpo(o->rn_factor, E->rn_factor, n);
}

void oracle_et_destroy(OracleEt *E) {
    if (!E) return;
    for (int i = 0; i < E->NE; i++) { free(E->acc_surf[i].q); free(E->acc_sub[i].q); }
    void *ps[] = {E->iforc, E->ilc, E->imf, E->ilake, E->z_surf, E->albedo, E->fixp, E->windh, E->vegf, E->nx, E->ny,
                  E->nz, E->t_prcp, E->t_temp, E->t_lai, E->t_mf, E->t_rn, E->t_wind, E->t_rh, E->qElePrep,
                  E->qPotEvap, E->qPotTran, E->qEleETP, E->qEleNetPrep, E->qEleE_IC, E->yEleIS, E->yEleSnow,
                  E->fu_Surf, E->fu_Sub, E->rn_factor, E->tsr_factor, E->tsr_has, E->acc_surf, E->acc_sub};
    for (size_t k = 0; k < sizeof(ps) / sizeof(ps[0]); k++) free(ps[k]);
    free(E);
}
