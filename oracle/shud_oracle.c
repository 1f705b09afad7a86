/*
 * shud_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the SHUD RHS (DankerMu/SHUD-up).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / CPU baseline — never as the product path (which is the HIP library under
 * shud-up_amd/).
 *
 * PARITY STATUS: "parity unpinned".  The reference ships no tests, fixtures or golden vectors for
 * this path, and its RHS cannot be compiled here without SUNDIALS' nvector headers
 * (src/Model/Macros.hpp:163,166 include them unconditionally; SUNDIALS is not installed and writing
 * stand-in headers for it is not allowed).  This file is therefore a line-by-line restatement of the
 * reference algorithm, cited file:line below, cross-checked by an independent numpy restatement
 * (oracle/numpy_oracle.py) and by conservation identities (tests/test_oracle.py).
 *
 * Structure follows the reference exactly: f_update -> f_loop (loops A,B,C,D + PassValue) ->
 * f_applyDY, with the same fp64 operation order, the reference's own min/max (functions.hpp:117-123,
 * NaN-propagation differs from fmin/fmax) and glibc libm (the same libm the reference links).
 * Loops A-D and applyDY run OpenMP-parallel over independent entities (as MD_f_omp.cpp does);
 * every reduction (PassValue, QeleSurfTot) runs in the reference's index order, so the result does
 * not depend on the thread count.  Build with -ffp-contract=off (x86-64 g++ -O3 emits no FMA).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "shud_rhs.h"

/* ---- constants: src/Model/Macros.hpp:46-77 ---- */
#define EPSILON 0.005
#define ZERO 1.0e-10
#define EPS_SLOPE 0.05e-6
#define MINPSI -1000000
#define FieldCapacityRatio 0.75
#define PI 3.1415926
#define GRAV 9.8
#define MAXYSURF 0.5
#define NA_VALUE -9999

/* functions.hpp:117-123 */
static inline double rmin(double a, double b) { return (a > b ? b : a); }
static inline double rmax(double a, double b) { return (a < b ? b : a); }

typedef struct OracleModel {
    int NE, NR, NS, mode, close_boundary;
    int NL, lakeon;                              /* lakes (MD_Lake.cpp; Model_Data.hpp:182-191) */
    /* static mesh (owned copies) */
    int *nabr;                                   /* [NE*3] element-major, 0-based / -1 */
    double *area, *z_surf, *z_bottom, *depression, *edge, *dist2nabor, *dist2edge, *avg_rough, *rough;
    int *ibc, *iss;
    int *riv_down, *riv_bc;
    double *riv_length, *riv_bed_slope, *riv_dist2down, *riv_avg_rough, *riv_depth, *riv_bw,
           *riv_bankslope, *riv_ksath, *riv_bedthick;
    int *seg_ele, *seg_riv;
    double *seg_length, *seg_cwr;
    /* lakes: ids, _Element::lakenabr (MD_Lake.cpp:131-143), _River::toLake (:44-52), bathymetry, state */
    int *ilake, *lakenabr, *NumEleLake, *toLake, *lake_off;
    double *lake_y, *lake_a, *qElePrep, *yLakeStg, *y2LakeArea, *QLakeSurf, *QLakeSub, *QLakeRivIn, *QLakeRivOut,
           *qLakeEvap, *qLakePrcp, *lakeQsub;
    /* element params */
    double *AquiferDepth, *macD, *macKsatH, *geo_vAreaF, *KsatH, *KsatV, *infKsatV, *hAreaF,
           *macKsatV, *ThetaS, *ThetaR, *Beta, *infD, *Sy, *RzD, *VegFrac, *ImpAF;
    /* step inputs */
    double *qEleNetPrep, *qPotEvap, *qPotTran, *qEleETP, *t_lai, *fu_Surf, *fu_Sub;
    double *eyBC, *eqBC, *ryBC, *rqBC;
    /* Model_Data scratch / state (Model_Data.cpp:90-167) */
    double *uYsf, *uYus, *uYgw, *uYriv;
    double *QeleSurf, *QeleSub;                  /* [NE*3] like double** rows */
    double *QeleSurfTot, *QeleSubTot, *Qe2r_Surf, *Qe2r_Sub;
    double *qEleInfil, *qEleExfil, *qEleRecharge;
    double *qEs, *qEu, *qEg, *qTu, *qTg, *qEleTrans, *qEleEvapo, *qEleETA, *iBeta, *qEleE_IC;
    double *QBC, *yBC;
    /* _Element u_* scratch (Element.hpp:101-116) */
    double *u_effKH, *u_satn, *u_deficit, *u_theta, *u_satKr, *u_phius, *u_effkInfi, *Kmax, *u_qi, *u_qex, *u_qr;
    /* _River u_* (River.hpp:75-80) */
    double *r_topWidth, *r_CSarea, *r_CSperem, *r_eqWidth, *r_TopArea, *r_qBC, *r_yBC;
    double *QrivSurf, *QrivSub, *QrivDown, *QrivUp, *QsegSurf, *QsegSub;
    int n_eyBC, n_eqBC, n_ryBC, n_rqBC;
    long long nFCall;
    /* first fatal error of the last call, as myexit() would have seen it */
    int exit_code, exit_index, exit_kind;
    long long n_aet_warn;
    int quiet;
} OracleModel;

static double *dup_d(const double *p, size_t n, double fill) {
    double *q = (double *)malloc(sizeof(double) * (n ? n : 1));
    if (p) memcpy(q, p, sizeof(double) * n);
    else for (size_t i = 0; i < n; i++) q[i] = fill;
    return q;
}
static int *dup_i(const int32_t *p, size_t n, int fill) {
    int *q = (int *)malloc(sizeof(int) * (n ? n : 1));
    for (size_t i = 0; i < n; i++) q[i] = p ? p[i] : fill;
    return q;
}
static double *zeros(size_t n) { return (double *)calloc(n ? n : 1, sizeof(double)); }

static int g_threads = 0;
void oracle_set_threads(int n) { g_threads = n; }
int oracle_get_threads(void) {
#ifdef _OPENMP
    return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
    return 1;
#endif
}
#ifdef _OPENMP
#define NT (g_threads > 0 ? g_threads : omp_get_max_threads())
#endif

void oracle_destroy(OracleModel *M);
OracleModel *oracle_create(const ShudMeshSoA *m, const ShudParamsSoA *p, int mode) {
    OracleModel *M = (OracleModel *)calloc(1, sizeof(OracleModel));
    int NE = m->num_ele, NR = m->num_riv, NS = m->num_seg;
    M->NE = NE; M->NR = NR; M->NS = NS; M->mode = mode; M->close_boundary = m->close_boundary;
    M->nabr = (int *)malloc(sizeof(int) * 3 * (NE ? NE : 1));
    M->edge = zeros(3 * NE); M->dist2nabor = zeros(3 * NE); M->dist2edge = zeros(3 * NE); M->avg_rough = zeros(3 * NE);
    for (int i = 0; i < NE; i++)
        for (int j = 0; j < 3; j++) {       /* edge-major SoA -> element-major rows */
            M->nabr[i * 3 + j] = m->nabr[j * NE + i];
            M->edge[i * 3 + j] = m->edge[j * NE + i];
            M->dist2nabor[i * 3 + j] = m->dist2nabor[j * NE + i];
            M->dist2edge[i * 3 + j] = m->dist2edge ? m->dist2edge[j * NE + i] : 0.;
            M->avg_rough[i * 3 + j] = m->avg_rough[j * NE + i];
        }
    M->area = dup_d(m->area, NE, 0); M->z_surf = dup_d(m->z_surf, NE, 0); M->z_bottom = dup_d(m->z_bottom, NE, 0);
    M->depression = dup_d(m->depression, NE, 0.0002); M->rough = dup_d(m->rough, NE, 0);
    M->ibc = dup_i(m->ibc, NE, 0); M->iss = dup_i(m->iss, NE, 0);
    M->riv_down = dup_i(m->riv_down, NR, -3); M->riv_bc = dup_i(m->riv_bc, NR, 0);
    M->riv_length = dup_d(m->riv_length, NR, 0); M->riv_bed_slope = dup_d(m->riv_bed_slope, NR, 0);
    M->riv_dist2down = dup_d(m->riv_dist2down, NR, 0); M->riv_avg_rough = dup_d(m->riv_avg_rough, NR, 0);
    M->riv_depth = dup_d(m->riv_depth, NR, 0); M->riv_bw = dup_d(m->riv_bottom_width, NR, 0);
    M->riv_bankslope = dup_d(m->riv_bankslope, NR, 0); M->riv_ksath = dup_d(m->riv_ksath, NR, 0);
    M->riv_bedthick = dup_d(m->riv_bedthick, NR, 0);
    M->seg_ele = dup_i(m->seg_ele, NS, 0); M->seg_riv = dup_i(m->seg_riv, NS, 0);
    M->seg_length = dup_d(m->seg_length, NS, 0); M->seg_cwr = dup_d(m->seg_cwr, NS, 0);
#define CP(f) M->f = dup_d(p->f, NE, 0)
    M->AquiferDepth = dup_d(p->aquifer_depth, NE, 0);
    CP(macD); CP(macKsatH); CP(geo_vAreaF); CP(KsatH); CP(KsatV); CP(infKsatV); CP(hAreaF);
    CP(macKsatV); CP(ThetaS); CP(ThetaR); CP(Beta); CP(infD); CP(Sy); CP(RzD); CP(VegFrac); CP(ImpAF);
#undef CP
    M->qEleNetPrep = zeros(NE); M->qPotEvap = zeros(NE); M->qPotTran = zeros(NE); M->qEleETP = zeros(NE);
    M->t_lai = zeros(NE); M->fu_Surf = dup_d(NULL, NE, 1.0); M->fu_Sub = dup_d(NULL, NE, 1.0);
    M->eyBC = zeros(1); M->eqBC = zeros(1); M->ryBC = zeros(1); M->rqBC = zeros(1);
    M->uYsf = zeros(NE); M->uYus = zeros(NE); M->uYgw = zeros(NE); M->uYriv = zeros(NR);
    M->QeleSurf = zeros(3 * NE); M->QeleSub = zeros(3 * NE);
    M->QeleSurfTot = zeros(NE); M->QeleSubTot = zeros(NE); M->Qe2r_Surf = zeros(NE); M->Qe2r_Sub = zeros(NE);
    M->qEleInfil = zeros(NE); M->qEleExfil = zeros(NE); M->qEleRecharge = zeros(NE);
    /* qEs..qTg are `new double[]` (uninitialised) in the reference (Model_Data.cpp:115-119); the
       OMP path never writes them, we pin them to 0 */
    M->qEs = zeros(NE); M->qEu = zeros(NE); M->qEg = zeros(NE); M->qTu = zeros(NE); M->qTg = zeros(NE);
    M->qEleTrans = zeros(NE); M->qEleEvapo = zeros(NE); M->qEleETA = zeros(NE); M->iBeta = zeros(NE);
    M->qEleE_IC = zeros(NE); M->QBC = zeros(NE); M->yBC = zeros(NE);
    M->u_effKH = zeros(NE); M->u_satn = zeros(NE); M->u_deficit = zeros(NE); M->u_theta = zeros(NE);
    M->u_satKr = zeros(NE); M->u_phius = zeros(NE); M->u_effkInfi = zeros(NE); M->Kmax = zeros(NE);
    M->u_qi = zeros(NE); M->u_qex = zeros(NE); M->u_qr = zeros(NE);
    M->r_topWidth = zeros(NR); M->r_CSarea = zeros(NR); M->r_CSperem = zeros(NR); M->r_eqWidth = zeros(NR);
    M->r_TopArea = zeros(NR); M->r_qBC = zeros(NR); M->r_yBC = zeros(NR);
    M->QrivSurf = zeros(NR); M->QrivSub = zeros(NR); M->QrivDown = zeros(NR); M->QrivUp = zeros(NR);
    M->QsegSurf = zeros(NS); M->QsegSub = zeros(NS);
    /* lakes: lakeon when any iLake > 0 (MD_readin.cpp:262-263), NumLake = LakeUniqueID (MD_Lake.cpp:12-29) */
    int NL = m->num_lake > 0 ? m->num_lake : 0;
    M->NL = NL;
    M->ilake = dup_i(m->ilake, NE, 0);
    for (int i = 0; i < NE; i++) if (M->ilake[i] > 0) M->lakeon = 1;
    M->lakenabr = (int *)calloc(3 * (NE ? NE : 1), sizeof(int));
    M->NumEleLake = (int *)calloc(NL ? NL : 1, sizeof(int));
    M->toLake = (int *)malloc(sizeof(int) * (NR ? NR : 1));
    M->lake_off = dup_i(m->lake_bathy_off, NL + 1, 0);
    int nb = NL ? M->lake_off[NL] : 0;
    M->lake_y = dup_d(m->lake_bathy_y, nb, 0); M->lake_a = dup_d(m->lake_bathy_a, nb, 0);
    M->qElePrep = zeros(NE); M->lakeQsub = zeros(3 * NE);
    M->yLakeStg = zeros(NL); M->y2LakeArea = zeros(NL); M->QLakeSurf = zeros(NL); M->QLakeSub = zeros(NL);
    M->QLakeRivIn = zeros(NL); M->QLakeRivOut = zeros(NL); M->qLakeEvap = zeros(NL); M->qLakePrcp = zeros(NL);
    for (int i = 0; i < NR; i++)                                   /* MD_Lake.cpp:44-52 */
        M->toLake[i] = (M->lakeon && M->riv_down[i] <= -4) ? (-3 - M->riv_down[i]) - 1 : NA_VALUE;
    if (M->lakeon) {
        for (int i = 0; i < NE; i++) if (M->ilake[i] > 0 && M->ilake[i] <= NL) M->NumEleLake[M->ilake[i] - 1]++;
        for (int i = 0; i < NE; i++)                               /* MD_Lake.cpp:131-143 */
            if (M->ilake[i] <= 0)
                for (int j = 0; j < 3; j++) {
                    int inabr = M->nabr[i * 3 + j];
                    if (inabr >= 0 && M->ilake[inabr] > 0) M->lakenabr[i * 3 + j] = M->ilake[inabr];
                }
    }
    M->quiet = 1;
    if (M->lakeon && mode == SHUD_MODE_OMP) {   /* the OMP path has no lake physics: not restated */
        oracle_destroy(M);
        return NULL;
    }
    return M;
}

static void set_arr(double *dst, const double *src, int n) { if (src) memcpy(dst, src, sizeof(double) * n); }
static double *set_tab(double *old, const double *src, int n, int *nstore) {
    if (!src) return old;
    free(old);
    double *q = (double *)malloc(sizeof(double) * (n + 1));
    memcpy(q, src, sizeof(double) * (n + 1));
    *nstore = n;
    return q;
}

void oracle_set_step_inputs(OracleModel *M, const ShudStepInputs *in) {
    int NE = M->NE;
    set_arr(M->qEleNetPrep, in->net_prep, NE); set_arr(M->qPotEvap, in->pot_evap, NE);
    set_arr(M->qPotTran, in->pot_tran, NE); set_arr(M->qEleETP, in->etp, NE);
    set_arr(M->t_lai, in->lai, NE); set_arr(M->fu_Surf, in->fu_surf, NE); set_arr(M->fu_Sub, in->fu_sub, NE);
    set_arr(M->qEleE_IC, in->e_ic, NE); set_arr(M->u_satn, in->u_satn, NE);
    set_arr(M->qElePrep, in->prcp, NE);
    /* uYgw of iBC<0 elements is never refreshed by f_update (MD_update.cpp:123-125) */
    if (in->ugw_stale)
        for (int i = 0; i < NE; i++) if (M->ibc[i] < 0) M->uYgw[i] = in->ugw_stale[i];
    M->eyBC = set_tab(M->eyBC, in->ele_ybc, in->n_ele_ybc, &M->n_eyBC);
    M->eqBC = set_tab(M->eqBC, in->ele_qbc, in->n_ele_qbc, &M->n_eqBC);
    M->ryBC = set_tab(M->ryBC, in->riv_ybc, in->n_riv_ybc, &M->n_ryBC);
    M->rqBC = set_tab(M->rqBC, in->riv_qbc, in->n_riv_qbc, &M->n_rqBC);
}

/* ===================== leaf equations (src/Equations) ===================== */
/* Equations.hpp:36-39 */
static inline double pow23(double x) { double t = cbrt(x); return t * t; }
/* Equations.hpp:41-43 */
static inline double sqpow2(double x, double y) { return sqrt(x * x + y * y); }
/* Equations.hpp:45-48 */
static inline double meanHarmonic(double k1, double k2, double d1, double d2) {
    return (k1 * k2) * (d1 + d2) / (d1 * k2 + d2 * k1);
}
/* Equations.hpp:50-52 */
static inline double meanArithmetic(double k1, double k2, double d1, double d2) {
    return (k1 * d1 + k2 * d2) / (d1 + d2);
}
/* Equations.hpp:54-63 */
static inline double ManningEquation(double Area, double rough, double R, double S) {
    if (S > 0) return sqrt(S) * Area * pow23(R) / rough;
    else return -1.0 * sqrt(-S) * Area * pow23(R) / rough;
}
/* Equations.hpp:31-33 (dead for DY; kept so u_phius matches) */
static inline double sat2psi(double elemSatn, double alpha, double n) {
    return -(pow(pow(elemSatn, n / (1 - n)) - 1, 1 / n) / alpha);
}
/* Equations.cpp:8-51 */
static double avgY_sf(double z1, double y1, double z2, double y2, double threshold) {
    double h1 = z1 + y1, h2 = z2 + y2;
    if (h1 > h2) return (y1 > threshold) ? y1 : 0.;
    else return (y2 > threshold) ? y2 : 0.;
}
/* Equations.cpp:52-70 */
static double avgY_gw(double z1, double y1, double z2, double y2, double threshold) {
    (void)z1; (void)z2; (void)threshold;
    y1 = rmax(y1, 0.);
    y2 = rmax(y2, 0.);
    return (y1 + y2) * .5;
}
/* Equations.cpp:116-134; returns error flag via *bad (myexit(ERRDATAIN)=13) */
static double effKH(double Ygw, double aqDepth, double MacD, double Kmac, double AF, double Kmx, int *bad) {
    double effk = 0;
    if (MacD <= ZERO || Ygw < aqDepth - MacD) {
        effk = Kmx;
    } else {
        if (Ygw > aqDepth) {
            effk = (Kmac * MacD * AF + Kmx * (aqDepth - MacD * AF)) / aqDepth;
        } else {
            effk = (Kmac * (Ygw - (aqDepth - MacD)) * AF +
                    Kmx * (aqDepth - MacD + (Ygw - (aqDepth - MacD)) * (1 - AF))) / Ygw;
        }
    }
    if (effk < 0. || effk > 1e9) *bad = 1;
    return effk;
}
/* Equations.cpp:136-141 */
static double satKfun(double elemSatn, double n) {
    double temp = -1. + pow(1. - pow(elemSatn, n / (n - 1.)), (n - 1.) / n);
    return sqrt(elemSatn) * temp * temp;
}
/* is_sm_et.cpp:131-140 (truncated PI) */
static double SoilMoistureStress(double ThetaS, double ThetaR, double SatRatio) {
    double fc, beta_s;
    fc = ThetaS * FieldCapacityRatio;
    beta_s = (SatRatio * (ThetaS - ThetaR) - ThetaR) / (fc - ThetaR);
    beta_s = rmin(rmax(0., beta_s), 1.);
    beta_s = 0.5 * (1 - cos(PI * beta_s));
    return beta_s;
}
/* Flux_RiverElement.cpp:11-55 */
static double flux_R2E_GW(double yr, double zr, double ye, double ze, double Kele, double Kriv,
                          double L, double D_riv) {
    double dh, A, g, K, he, hr, Q = 0.0;
    if (Kele < ZERO || Kriv < ZERO) return 0.;
    K = meanArithmetic(Kele, Kriv, 1., 1.);
    he = ye + ze;
    hr = yr + zr;
    dh = hr - he;
    if (dh > ZERO) {
        if (he > zr) A = (yr + (he - zr)) * .5 * L;
        else A = yr * L;
        if (yr < EPSILON) Q = 0.;
        else { g = dh / D_riv; Q = A * K * g; }
    } else if (dh < -ZERO) {
        if (ye > ZERO) {
            A = (yr + (he - zr)) * .5 * L;
            g = dh / D_riv;
            Q = A * K * g;
        } else Q = 0.;
    } else Q = 0.;
    return Q;
}
/* functions.hpp:125-139 */
static inline double Quadratic(double s, double w, double dA) {
    double ret = 0., cc;
    s = fabs(s);
    cc = w * w + 4 * s * dA;
    if (cc < ZERO) ret = -1. * w / (2. * s);     /* stderr "Error in Quadratic" when cc < -ZERO */
    else ret = (-w + sqrt(cc)) / (2 * s);
    return ret;
}
/* functions.hpp:141-153 */
static inline double fun_dAtodY(double dA, double w_top, double s) {
    double dy = 0.;
    if (dA == 0.) return 0.;
    if (fabs(s) < EPS_SLOPE) dy = dA / w_top;
    else dy = Quadratic(s, w_top, dA);
    return dy;
}
/* functions.hpp:183-189 */
static inline double fixMaxValue(double x, double defVal) { return (x < defVal) ? defVal : x; }
/* River.hpp:115-127 */
static inline double fun_CrossArea(double y, double w0, double s) { return y * (w0 + y * s); }
static inline double fun_CrossPerem(double y, double w0, double s) { return 2.0 * sqpow2(y, y * s) + w0; }
static inline double fun_TopWidth(double y, double w0, double s) { return y * s * 2.0 + w0; }
static inline double fun_EqWidth(double y, double w0, double s) { double w1 = fun_TopWidth(y, w0, s); return 0.5 * (w1 + w0); }

/* ===================== domain objects ===================== */
/* River.cpp:49-62 _River::updateRiver */
static void updateRiver(OracleModel *M, int i, double newY) {
    double w0 = M->riv_bw[i], s = M->riv_bankslope[i];
    double topw = fun_TopWidth(newY, w0, s), csa = fun_CrossArea(newY, w0, s), per = fun_CrossPerem(newY, w0, s);
    double eqw = fun_EqWidth(newY, w0, s), ta = eqw * M->riv_length[i];
    M->r_topWidth[i] = fixMaxValue(topw, 0.);
    M->r_CSarea[i] = fixMaxValue(csa, 0.);
    M->r_CSperem[i] = fixMaxValue(per, 0.);
    M->r_eqWidth[i] = fixMaxValue(eqw, 0.);
    M->r_TopArea[i] = fixMaxValue(ta, 0.);
}

/* Element.cpp:347-384 _Element::updateElement (bad -> effKH myexit) */
static void updateElement(OracleModel *M, int i, double Ysurf, double Yunsat, double Ygw, int *bad) {
    (void)Ysurf;
    M->u_effKH[i] = effKH(Ygw, M->AquiferDepth[i], M->macD[i], M->macKsatH[i], M->geo_vAreaF[i], M->KsatH[i], bad);
    M->u_deficit[i] = M->AquiferDepth[i] - Ygw;
    M->Kmax[i] = M->infKsatV[i] * (1. - M->hAreaF[i]) + M->macKsatV[i] * M->hAreaF[i];
    if (M->u_deficit[i] <= 0.) {
        M->u_deficit[i] = 0.;
        M->u_satn[i] = 1.;
        M->u_theta[i] = M->ThetaS[i];
    } else {
        M->u_theta[i] = Yunsat / M->u_deficit[i] * M->ThetaS[i];
        M->u_satn[i] = (M->u_theta[i] - M->ThetaR[i]) / (M->ThetaS[i] - M->ThetaR[i]);
    }
    if (M->u_satn[i] > 0.99) {
        M->u_satn[i] = 1.0; M->u_satKr[i] = 1.0; M->u_phius[i] = 0.; M->u_theta[i] = M->ThetaS[i];
    } else if (M->u_satn[i] <= ZERO) {
        M->u_satn[i] = 0.; M->u_satKr[i] = 0.; M->u_phius[i] = MINPSI; M->u_theta[i] = M->ThetaR[i];
    } else {
        M->u_satKr[i] = satKfun(M->u_satn[i], M->Beta[i]);
        /* sat2psi (Element.cpp:376-377) is dead for DY (u_phius is never read by a flux): skipped */
    }
    M->u_effkInfi[i] = M->infKsatV[i] * (1 - M->hAreaF[i]) + M->u_satn[i] * M->macKsatV[i] * M->hAreaF[i];
}

/* Element.cpp:271-303 _Element::Flux_Infiltration */
static void Flux_Infiltration(OracleModel *M, int i, double Ysurf, double Yunsat, double Ygw, double netprcp) {
    double av = Ysurf + netprcp, grad = 0;
    double Aq = M->AquiferDepth[i], infD = M->infD[i], Kmax = M->Kmax[i];
    if (Ygw + Yunsat > Aq || M->u_deficit[i] < Yunsat) {
        M->u_qex[i] = fabs(Ygw + Yunsat - Aq) / Aq * Kmax;
        M->u_qi[i] = 0.;
    } else {
        M->u_qex[i] = 0.;
        if (av > 0. && M->u_deficit[i] > infD) {
            grad = 1. + av / infD;
            double infK = M->infKsatV[i], hA = M->hAreaF[i], macK = M->macKsatV[i];
            if (av > Kmax) M->u_effkInfi[i] = infK * (1 - hA) + hA * macK * M->u_satn[i];
            else if (av > infK) M->u_effkInfi[i] = M->u_satKr[i] * infK * (1 - hA) + hA * macK * M->u_satn[i];
            else M->u_effkInfi[i] = M->u_satKr[i] * infK * (1 - hA);
            M->u_qi[i] = grad * M->u_effkInfi[i];
            M->u_qi[i] = rmin(av, rmax(0., M->u_qi[i]));
        } else {
            M->u_qi[i] = 0;
        }
    }
}
/* Element.cpp:304-335 _Element::Flux_Recharge */
static double Flux_Recharge(OracleModel *M, int i, double Yunsat, double Ygw) {
    double ke = 0., grad, ku;
    double ThetaR = M->ThetaR[i], ThetaFC = M->ThetaS[i] * FieldCapacityRatio; /* copySoil, Element.cpp:399 */
    if (Ygw > M->AquiferDepth[i] - M->infD[i] && Yunsat < M->u_deficit[i]) {
        M->u_qr[i] = 0.;
        return M->u_qr[i];
    }
    if (M->u_theta[i] > ThetaR) {
        if (Yunsat <= EPSILON) grad = 0.;
        else { grad = (M->u_theta[i] - ThetaR) / (ThetaFC - ThetaR); grad = rmax(grad, 0.); }
    } else grad = 0.;
    if (M->infKsatV[i] <= 0. || M->KsatV[i] <= 0.) {
        M->u_qr[i] = 0.;
    } else {
        ku = M->infKsatV[i] * M->u_satKr[i];
        ke = meanHarmonic(ku, M->KsatV[i], M->u_deficit[i], Ygw);
        M->u_qr[i] = grad * ke;
    }
    return M->u_qr[i];
}

/* ===================== Model_Data RHS pieces ===================== */
/* MD_ET.cpp:343-404 Model_Data::f_etFlux; returns 0, or kind 1 (CheckNonNegative) / 2 (CheckNANi) */
static int f_etFlux(OracleModel *M, int i, int *warn) {
    double Es = 0., Eu = 0., Tu = 0., Eg = 0., Tg = 0.;
    double va = M->VegFrac[i], vb = 1. - M->VegFrac[i];
    double pj = 1. - M->ImpAF[i];
    double WetlandLevel = M->AquiferDepth[i] - M->infD[i];      /* Element.cpp:221 */
    double RootReachLevel = M->AquiferDepth[i] - M->RzD[i];     /* Element.cpp:222 */
    M->iBeta[i] = SoilMoistureStress(M->ThetaS[i], M->ThetaR[i], M->u_satn[i]);
    Es = rmin(rmax(0., M->uYsf[i]), M->qPotEvap[i]) * vb;
    if (Es < M->qPotEvap[i]) {
        if (M->uYgw[i] > WetlandLevel) {
            Eg = rmin(rmax(0., M->uYgw[i]), M->qPotEvap[i] - Es) * pj * vb;
            Eu = 0.;
        } else {
            Eg = 0.;
            Eu = rmin(rmax(0., M->uYus[i]), M->iBeta[i] * (M->qPotEvap[i] - Es)) * pj * vb;
        }
    } else {
        Eg = 0.; Eu = 0.;
    }
    if (M->t_lai[i] > ZERO) {
        if (M->qEleE_IC[i] >= M->qPotTran[i]) {
            Tg = Tu = 0.;
            M->qEleE_IC[i] = M->qPotTran[i] * pj * va;
        } else {
            if (M->uYgw[i] > RootReachLevel) {
                Tg = rmin(rmax(0., M->uYgw[i]), (M->qPotTran[i] - M->qEleE_IC[i])) * pj * va;
                Tu = 0.;
            } else {
                Tg = 0.;
                Tu = rmin(rmax(0., M->uYus[i]), M->iBeta[i] * (M->qPotTran[i] - M->qEleE_IC[i])) * pj * va;
            }
        }
    } else {
        Tg = Tu = M->qEleE_IC[i] = 0.;
    }
    M->qEs[i] = Es; M->qEu[i] = Eu; M->qEg[i] = Eg; M->qTu[i] = Tu; M->qTg[i] = Tg;
    M->qEleTrans[i] = Tg + Tu;
    M->qEleEvapo[i] = Eu + Eg + Es;
    M->qEleETA[i] = M->qEleE_IC[i] + M->qEleEvapo[i] + M->qEleTrans[i];
    if (M->qEleETA[i] > M->qEleETP[i] * 2.) *warn = 1;
    /* CheckNonNegative (functions.cpp:148-154) */
    double v[5] = {Es, Eu, Eg, Tu, Tg};
    for (int k = 0; k < 5; k++)
        if (v[k] < 0.0 || isnan(v[k]) || isinf(v[k]) || fabs(v[k] - NA_VALUE) < ZERO) return 1;
    double w[3] = {M->qEleETA[i], M->qEleEvapo[i], M->qEleTrans[i]};
    for (int k = 0; k < 3; k++)
        if (isnan(w[k]) || isinf(w[k])) return 2;
    return 0;
}

/* MD_update.cpp:102-189 Model_Data::f_update (serial) */
/* Lake.cpp:59-79 LakeBathymetry::toparea (the reference's own interpolation, kept as written) */
static double lake_toparea(OracleModel *M, int l, double y) {
    const double *yi = M->lake_y + M->lake_off[l], *ai = M->lake_a + M->lake_off[l];
    int nvalue = M->lake_off[l + 1] - M->lake_off[l];
    double ta = ai[0], dy, da;
    if (y <= yi[0]) {
        ta = ai[0];
    } else {
        for (int i = 1; i < nvalue; i++) {
            if (y < yi[i]) {
                da = (ai[i] - ta);
                dy = yi[i] - y;
                ta = da / dy * (y - yi[i - 1]) + ta;
                break;
            } else {
                ta = ai[i];
            }
        }
    }
    return ta;
}
/* Element.cpp:336-346 _Element::updateLakeElement */
static void updateLakeElement(OracleModel *M, int i) {
    M->u_effKH[i] = M->KsatH[i];
    M->u_deficit[i] = 0;
    M->Kmax[i] = M->infKsatV[i];
    M->u_deficit[i] = 0.;
    M->u_satn[i] = 1.;
    M->u_theta[i] = M->ThetaS[i];
    M->u_satKr[i] = 1.0;
    M->u_phius[i] = 0.;
    M->u_effkInfi[i] = M->infKsatV[i];
}
/* MD_ElementFlux.cpp:2-17 Model_Data::fun_Ele_lakeVertical */
static void fun_Ele_lakeVertical(OracleModel *M, int i) {
    M->qEleInfil[i] = 0.; M->qEleRecharge[i] = 0.; M->qEleExfil[i] = 0.; M->qEleTrans[i] = 0.;
    M->qEs[i] = 0.; M->qEu[i] = 0.; M->qEg[i] = 0.; M->qTu[i] = 0.; M->qTg[i] = 0.;
    M->qEleE_IC[i] = 0.; M->qEleTrans[i] = 0.;
    M->qEleEvapo[i] = M->qPotEvap[i];
    M->qEleETA[i] = M->qEleE_IC[i] + M->qEleEvapo[i] + M->qEleTrans[i];
}

static void f_update(OracleModel *M, const double *Y, double *DY, double t) {
    (void)t;
    int NE = M->NE, NR = M->NR;
    for (int i = 0; i < NE; i++) {
        for (int j = 0; j < 3; j++) { M->QeleSub[i * 3 + j] = 0.; M->QeleSurf[i * 3 + j] = 0.; }
        M->QeleSubTot[i] = 0.; M->QeleSurfTot[i] = 0.;
        M->uYsf[i] = Y[i];
        M->uYus[i] = Y[i + NE];
        if (M->ibc[i] == 0) {
            M->uYgw[i] = Y[i + 2 * NE];
            M->QBC[i] = 0.;
        } else if (M->ibc[i] > 0) {
            M->yBC[i] = M->eyBC[M->ibc[i]];
            M->uYgw[i] = M->yBC[i];
            M->QBC[i] = 0.;
        } else {
            M->QBC[i] = M->eqBC[-M->ibc[i]];       /* uYgw keeps its stale value */
        }
        M->qEleExfil[i] = 0.;
        M->qEleInfil[i] = 0.;
    }
    for (int i = 0; i < NR; i++) {
        M->uYriv[i] = Y[i + 3 * NE];
        updateRiver(M, i, M->uYriv[i]);
        M->r_qBC[i] = 0.0;
        if (M->riv_bc[i] == 0) {
        } else if (M->riv_bc[i] < 0) {
            M->r_qBC[i] = M->rqBC[-M->riv_bc[i]];
        } else {
            M->r_yBC[i] = M->ryBC[M->riv_bc[i]];
            M->uYriv[i] = M->r_yBC[i];
        }
    }
    for (int i = 0; i < NR; i++) { M->QrivSurf[i] = 0.; M->QrivSub[i] = 0.; M->QrivUp[i] = 0.; }
    for (int i = 0; i < NE; i++) { M->Qe2r_Surf[i] = 0.; M->Qe2r_Sub[i] = 0.; }
    for (int i = 0; i < M->NL; i++) {                         /* MD_update.cpp:174-185 */
        M->yLakeStg[i] = Y[3 * NE + NR + i];
        M->y2LakeArea[i] = lake_toparea(M, i, M->yLakeStg[i] + M->lake_y[M->lake_off[i]]);   /* _Lake::update */
        M->QLakeSub[i] = 0.; M->QLakeSurf[i] = 0.; M->qLakeEvap[i] = 0.; M->qLakePrcp[i] = 0.;
        M->QLakeRivIn[i] = 0.; M->QLakeRivOut[i] = 0.;
    }
    for (int i = 0; i < 3 * NE + NR + M->NL; i++) DY[i] = 0.;
}

/* MD_f_omp.cpp:104-170 Model_Data::f_update_omp */
static void f_update_omp(OracleModel *M, const double *Y, double *DY, double t) {
    (void)t;
    int NE = M->NE, NR = M->NR;
    for (int i = 0; i < 3 * NE + NR; i++) DY[i] = 0.;
#pragma omp parallel for num_threads(NT) schedule(static)
    for (int i = 0; i < NE; i++) {
        M->uYsf[i] = (Y[i] >= 0.) ? Y[i] : 0.;
        M->uYus[i] = (Y[i + NE] >= 0.) ? Y[i + NE] : 0.;
        if (M->ibc[i] == 0) {
            M->uYgw[i] = rmax(0.0, Y[i + 2 * NE]);
            M->QBC[i] = 0.;
        } else if (M->ibc[i] > 0) {
            M->yBC[i] = M->eyBC[M->ibc[i]];
            M->uYgw[i] = M->yBC[i];
            M->QBC[i] = 0.;
        } else {
            M->QBC[i] = M->eqBC[-M->ibc[i]];
        }
        M->qEleExfil[i] = 0.;
        M->qEleInfil[i] = 0.;
    }
#pragma omp parallel for num_threads(NT) schedule(static)
    for (int i = 0; i < NR; i++) {
        M->uYriv[i] = (Y[i + 3 * NE] >= 0.) ? Y[i + 3 * NE] : 0.;
        updateRiver(M, i, M->uYriv[i]);
        M->r_qBC[i] = 0.0;
        if (M->riv_bc[i] == 0) {
        } else if (M->riv_bc[i] < 0) {
            M->r_qBC[i] = M->rqBC[-M->riv_bc[i]];
        } else {
            M->r_yBC[i] = M->ryBC[M->riv_bc[i]];
            M->uYriv[i] = M->r_yBC[i];
        }
    }
}

/* MD_ElementFlux.cpp:30-34 */
static void fun_Ele_Infiltraion(OracleModel *M, int i) {
    Flux_Infiltration(M, i, M->uYsf[i], M->uYus[i], M->uYgw[i], M->qEleNetPrep[i]);
    M->qEleInfil[i] = M->u_qi[i] * M->fu_Surf[i];
    M->qEleExfil[i] = M->u_qex[i] * M->fu_Surf[i];
}
/* MD_ElementFlux.cpp:24-28 */
static void fun_Ele_Recharge(OracleModel *M, int i) {
    M->qEleRecharge[i] = Flux_Recharge(M, i, M->uYus[i], M->uYgw[i]);
    M->qEleRecharge[i] *= M->fu_Sub[i];
}
static double WeirFlow_jtoi(double zi, double yi, double zj, double yj, double zbank, double cwr,
                            double width, double threshold);
/* MD_ElementFlux.cpp:35-97 (QLakeSurf is accumulated by f_loop in reference order) */
static void fun_Ele_surface(OracleModel *M, int i) {
    double Ymean, dh, s, CrossA, Q, B, isf, nsf;
    isf = M->uYsf[i];
    isf = isf < 0. ? 0. : isf;
    for (int j = 0; j < 3; j++) {
        int inabr = M->nabr[i * 3 + j];
        int ilake = M->lakenabr[i * 3 + j] - 1;
        B = M->edge[i * 3 + j];
        if (ilake >= 0) {                            /* bank edge: weir to the lake (:46-53) */
            nsf = M->yLakeStg[ilake];
            nsf = nsf < 0. ? 0. : nsf;
            Q = WeirFlow_jtoi(M->lake_y[M->lake_off[ilake]], nsf, M->z_surf[i], isf, M->z_surf[i], 0.6, B, 0.01);
        } else if (inabr >= 0) {
            nsf = M->uYsf[inabr];
            nsf = nsf < 0. ? 0. : nsf;
            dh = (isf + M->z_surf[i]) - (nsf + M->z_surf[inabr]);
            Ymean = avgY_sf(M->z_surf[i], isf, M->z_surf[inabr], nsf, M->depression[i]);
            Ymean = rmin(Ymean, MAXYSURF);
            if (Ymean <= 0.) {
                Q = 0.;
            } else {
                s = dh / M->dist2nabor[i * 3 + j];
                CrossA = Ymean * B;
                if (s > 0 && isf <= 0) Q = 0.;
                else if (s < 0 && nsf <= 0) Q = 0.;
                else Q = ManningEquation(CrossA, M->avg_rough[i * 3 + j], Ymean, s);
            }
        } else {
            Q = 0;
            if (!M->close_boundary) {
                if (isf > M->depression[i]) {
                    s = isf / M->dist2edge[i * 3 + j] * 0.5;
                    if (s > 0.) Q = sqrt(s) * cbrt(isf * isf * isf * isf * isf) * B / M->rough[i];
                }
            }
        }
        M->QeleSurf[i * 3 + j] = Q;
    }
}
/* MD_ElementFlux.cpp:100-156 (QLakeSub is accumulated by f_loop in reference order) */
static void fun_Ele_sub(OracleModel *M, int i) {
    double Ymean, dh, Kmean, grad, Q;
    for (int j = 0; j < 3; j++) {
        int inabr = M->nabr[i * 3 + j];
        int ilake = M->lakenabr[i * 3 + j] - 1;
        if (ilake >= 0) {                            /* bank edge: Darcy to the lake (:107-121) */
            double zl = M->lake_y[M->lake_off[ilake]], yl = M->yLakeStg[ilake];
            dh = (M->uYgw[i] + M->z_bottom[i]) - (yl + zl);
            if (dh > 0. && M->uYgw[i] <= 0.02) Q = 0.;
            else if (dh < 0. && yl <= 0.02) Q = 0.;
            else {
                Ymean = avgY_gw(M->z_bottom[i], M->uYgw[i], zl, yl, 0.002);
                grad = dh / M->dist2nabor[i * 3 + j];
                Kmean = 0.5 * (M->u_effKH[i] + M->u_effKH[inabr]);   /* the lake element's KsatH */
                Q = Kmean * grad * Ymean * M->edge[i * 3 + j];
            }
            M->lakeQsub[i * 3 + j] = Q;
        } else if (inabr >= 0) {
            dh = (M->uYgw[i] + M->z_bottom[i]) - (M->uYgw[inabr] + M->z_bottom[inabr]);
            if (dh > 0. && M->uYgw[i] <= 0.02) Q = 0.;
            else if (dh < 0. && M->uYgw[inabr] <= 0.02) Q = 0.;
            else {
                Ymean = avgY_gw(M->z_bottom[i], M->uYgw[i], M->z_bottom[inabr], M->uYgw[inabr], 0.002);
                grad = dh / M->dist2nabor[i * 3 + j];
                Kmean = 0.5 * (M->u_effKH[i] + M->u_effKH[inabr]);
                Q = Kmean * grad * Ymean * M->edge[i * 3 + j];
            }
        } else {
            Q = 0;
            if (!M->close_boundary) {
                if (M->uYgw[i] > M->depression[i] * 10.) {
                    grad = M->uYgw[i] / M->dist2edge[i * 3 + j] * 0.5;
                    if (grad > 0.) Q = M->u_effKH[i] * grad;
                }
            }
        }
        M->QeleSub[i * 3 + j] = Q * M->fu_Sub[i];
    }
}
/* MD_RiverFlux.cpp:65-98 */
static double WeirFlow_jtoi(double zi, double yi, double zj, double yj, double zbank, double cwr,
                            double width, double threshold) {
    double hi, hj, Q = 0., dh, y;
    hi = yi + zi;
    hj = yj + zj;
    dh = hj - hi;
    if (dh > 0.) {
        y = hi - zbank;
        if ((y > 0.) & (yj > threshold)) {
            if (hi > zbank) y = dh;
            Q = cwr * sqrt(2. * GRAV * y) * width * y * 60.;
        } else Q = 0.;
    } else {
        y = hi - zbank;
        if (y > 0. && yi > threshold) {
            if (hj > zbank) y = -dh;
            Q = -1. * cwr * sqrt(2. * GRAV * y) * width * y * 60.;
        } else Q = 0.;
    }
    return Q;
}
/* MD_RiverFlux.cpp:100-113 (the racy/overwritten += into QrivSurf/Qe2r_Surf is redone by PassValue) */
static void fun_Seg_surface(OracleModel *M, int iEle, int iRiv, int i) {
    double isf = M->uYsf[iEle] - M->qEleInfil[iEle] + M->qEleExfil[iEle];
    isf = rmax(0., isf);
    double zbank = M->z_surf[iEle] + 0.0;          /* Riv.zbank is never set: 0.0 (River.hpp:67) */
    M->QsegSurf[i] = WeirFlow_jtoi(M->z_surf[iEle], isf, M->z_surf[iEle] - M->riv_depth[iRiv], M->uYriv[iRiv],
                                   zbank, M->seg_cwr[i], M->seg_length[i], M->depression[iEle]);
}
/* MD_RiverFlux.cpp:114-126 */
static void fun_Seg_sub(OracleModel *M, int iEle, int iRiv, int i) {
    M->QsegSub[i] = flux_R2E_GW(M->uYriv[iRiv], M->z_surf[iEle] - M->riv_depth[iRiv], M->uYgw[iEle],
                                M->z_bottom[iEle], M->u_effKH[iEle], M->riv_ksath[iRiv], M->seg_length[i],
                                M->riv_bedthick[iRiv]);
    M->QsegSub[i] *= M->fu_Sub[iEle];
}
/* MD_RiverFlux.cpp:5-63 (QLakeRivIn is accumulated by f_loop in reach order; invalid `down` rejected) */
static void Flux_RiverDown(OracleModel *M, int i) {
    double Distance, CSarea, Perem, R, s, n, sMean = 0.;
    int iDown = M->riv_down[i];
    n = M->riv_avg_rough[i];
    if (M->toLake[i] >= 0) {                          /* to a lake (:17-25) */
        Perem = M->r_CSperem[i];
        s = M->riv_bed_slope[i] + M->uYriv[i] * 2. / M->riv_length[i];
        CSarea = M->r_CSarea[i];
        R = (Perem <= 0.) ? 0. : (CSarea / Perem);
        M->QrivDown[i] = ManningEquation(CSarea, n, R, s);
    } else if (iDown >= 0) {
        sMean = (M->riv_bed_slope[i] + M->riv_bed_slope[iDown]) * 0.5;
        Distance = M->riv_dist2down[i];
        s = ((M->uYriv[i] - M->riv_depth[i]) - (M->uYriv[iDown] - M->riv_depth[iDown])) / Distance + sMean;
        CSarea = M->r_CSarea[i];
        Perem = M->r_CSperem[i];
        R = (Perem <= ZERO) ? 0. : (CSarea / Perem);
        M->QrivDown[i] = ManningEquation(CSarea, n, R, s);
    } else if (iDown == -1 || iDown == -2 || iDown == -3) {
        Perem = M->r_CSperem[i];
        s = M->riv_bed_slope[i] + M->uYriv[i] * 2. / M->riv_length[i];
        CSarea = M->r_CSarea[i];
        R = (Perem <= 0.) ? 0. : (CSarea / Perem);
        M->QrivDown[i] = ManningEquation(CSarea, n, R, s);
    } else { /* -4 */
        M->QrivDown[i] = M->r_CSarea[i] * sqrt(GRAV * M->uYriv[i]) * 60.;
    }
}
/* MD_f.cpp:217-257 Model_Data::PassValue (serial, index order) */
static void PassValue(OracleModel *M) {
    int NE = M->NE, NR = M->NR, NS = M->NS;
    for (int i = 0; i < NR; i++) { M->QrivSurf[i] = 0.; M->QrivSub[i] = 0.; M->QrivUp[i] = 0.; }
    for (int i = 0; i < NE; i++) { M->Qe2r_Surf[i] = 0.; M->Qe2r_Sub[i] = 0.; }
    for (int i = 0; i < NS; i++) {
        int ie = M->seg_ele[i], ir = M->seg_riv[i];
        M->QrivSurf[ir] += M->QsegSurf[i];
        M->QrivSub[ir] += M->QsegSub[i];
        M->Qe2r_Surf[ie] += -M->QsegSurf[i];
        M->Qe2r_Sub[ie] += -M->QsegSub[i];
    }
    for (int i = 0; i < NR; i++) {
        int d = M->riv_down[i];
        if (d >= 0) M->QrivUp[d] += -M->QrivDown[i];    /* toLake <= 0 holds: no lakes */
    }
}

static void note_exit(OracleModel *M, int code, int idx, int kind) {
    if (M->exit_code == 0) { M->exit_code = code; M->exit_index = idx; M->exit_kind = kind; }
}

/* MD_f.cpp:9-50 Model_Data::f_loop (serial semantics) / MD_f_omp.cpp:69-100 (omp) */
static int f_loop(OracleModel *M) {
    int NE = M->NE, NR = M->NR, NS = M->NS, omp = (M->mode == SHUD_MODE_OMP);
    int *aerr = (int *)calloc(NE ? NE : 1, sizeof(int));
    long long nwarn = 0;
    /* loop A (MD_f.cpp:11-26) */
#pragma omp parallel for num_threads(NT) schedule(static) reduction(+ : nwarn)
    for (int i = 0; i < NE; i++) {
        int bad = 0, warn = 0;
        if (M->lakeon && M->ilake[i] > 0) {          /* lake element (MD_f.cpp:12-17) */
            updateLakeElement(M, i);
            fun_Ele_lakeVertical(M, i);
            continue;
        }
        if (!omp) {
            int k = f_etFlux(M, i, &warn);
            nwarn += warn;
            if (k) { aerr[i] = k; continue; }             /* myexit inside f_etFlux */
        }
        updateElement(M, i, M->uYsf[i], M->uYus[i], M->uYgw[i], &bad);
        if (bad) { aerr[i] = 3; continue; }                 /* myexit inside effKH */
        fun_Ele_Infiltraion(M, i);
        fun_Ele_Recharge(M, i);
    }
    M->n_aet_warn += nwarn;
    for (int i = 0; i < NE; i++)                              /* the first exit in loop order */
        if (aerr[i]) {
            int k = aerr[i];
            note_exit(M, k == 3 ? 13 : 10, i, k == 1 ? SHUD_EF_ET_NEG : k == 2 ? SHUD_EF_ET_NAN : SHUD_EF_EFFKH);
            free(aerr);
            return M->exit_code;
        }
    free(aerr);
    for (int i = 0; i < NE; i++)                            /* MD_f.cpp:16-17, element order */
        if (M->lakeon && M->ilake[i] > 0) {
            int l = M->ilake[i] - 1;
            M->qLakeEvap[l] += M->qEleEvapo[i] / M->NumEleLake[l];
            M->qLakePrcp[l] += M->qElePrep[i] / M->NumEleLake[l];
        }
    /* loop B (MD_f.cpp:27-36) */
#pragma omp parallel for num_threads(NT) schedule(static)
    for (int i = 0; i < NE; i++) {
        if (M->lakeon && M->ilake[i] > 0) {          /* fun_Ele_lakeHorizon (MD_ElementFlux.cpp:18-23) */
            for (int j = 0; j < 3; j++) { M->QeleSurf[i * 3 + j] = 0.; M->QeleSub[i * 3 + j] = 0.; }
            continue;
        }
        fun_Ele_surface(M, i);
        fun_Ele_sub(M, i);
    }
    if (M->lakeon)                                            /* QLakeSurf/QLakeSub, element then edge order */
        for (int i = 0; i < NE; i++)
            for (int j = 0; j < 3; j++) {
                int l = M->lakenabr[i * 3 + j] - 1;
                if (l >= 0 && M->ilake[i] <= 0) {
                    M->QLakeSurf[l] += M->QeleSurf[i * 3 + j];
                    M->QLakeSub[l] += M->lakeQsub[i * 3 + j];
                }
            }
    /* loop C (MD_f.cpp:37-40) */
#pragma omp parallel for num_threads(NT) schedule(static)
    for (int i = 0; i < NS; i++) {
        fun_Seg_surface(M, M->seg_ele[i], M->seg_riv[i], i);
        fun_Seg_sub(M, M->seg_ele[i], M->seg_riv[i], i);
    }
    /* loop D (MD_f.cpp:41-43) */
#pragma omp parallel for num_threads(NT) schedule(static)
    for (int i = 0; i < NR; i++) Flux_RiverDown(M, i);
    for (int i = 0; i < NR; i++)                              /* MD_RiverFlux.cpp:24, reach order */
        if (M->toLake[i] >= 0) M->QLakeRivIn[M->toLake[i]] += M->QrivDown[i];
    for (int i = 0; i < M->NL; i++) {                         /* MD_f.cpp:44-47 */
        M->qLakeEvap[i] = rmin(M->qLakeEvap[i], M->qLakePrcp[i] + M->yLakeStg[i]);
        M->qLakeEvap[i] = rmax(0, M->qLakeEvap[i]);
    }
    PassValue(M);                                             /* MD_f.cpp:49 */
    return 0;
}

/* MD_f.cpp:52-215 Model_Data::f_applyDY (serial; wbdiag quad rates out of scope) */
static int f_applyDY(OracleModel *M, double *DY) {
    int NE = M->NE, NR = M->NR;
    for (int i = 0; i < NE; i++) {               /* serial: CheckNANij exits at the first NaN */
        for (int j = 0; j < 3; j++) {
            double a = M->QeleSurf[i * 3 + j], b = M->QeleSub[i * 3 + j];
            if (isnan(a) || isinf(a) || isnan(b) || isinf(b)) {
                note_exit(M, 10, i, SHUD_EF_NAN_QELE);
                return 10;
            }
        }
    }
#pragma omp parallel for num_threads(NT) schedule(static)
    for (int i = 0; i < NE; i++) {
        int isf = i, ius = i + NE, igw = i + 2 * NE;
        double area = M->area[i];
        M->QeleSurfTot[i] = M->Qe2r_Surf[i];
        M->QeleSubTot[i] = M->Qe2r_Sub[i];
        for (int j = 0; j < 3; j++) {
            M->QeleSurfTot[i] += M->QeleSurf[i * 3 + j];
            M->QeleSubTot[i] += M->QeleSub[i * 3 + j];
        }
        DY[i] = M->qEleNetPrep[i] - M->qEleInfil[i] + M->qEleExfil[i] - M->QeleSurfTot[i] / area - M->qEs[i];
        DY[ius] = M->qEleInfil[i] - M->qEleRecharge[i] - M->qEu[i] - M->qTu[i];
        DY[igw] = M->qEleRecharge[i] - M->qEleExfil[i] - M->QeleSubTot[i] / area - M->qEg[i] - M->qTg[i];
        if (M->ibc[i] == 0) {
        } else if (M->ibc[i] > 0) DY[igw] = 0;
        else DY[igw] += M->QBC[i] / area;
        if (M->iss[i] == 0) {
        } else if (M->iss[i] > 0) DY[isf] += 0.0 / area;     /* QSS is never assigned: 0 */
        else DY[igw] += 0.0 / area;
        DY[ius] /= M->Sy[i];
        DY[igw] /= M->Sy[i];
        if (M->ilake[i] > 0) { DY[isf] = 0.; DY[ius] = 0.; DY[igw] = 0.; }   /* MD_f.cpp:146-150 */
    }
#pragma omp parallel for num_threads(NT) schedule(static)
    for (int i = 0; i < NR; i++) {
        int iriv = i + 3 * NE;
        if (M->riv_bc[i] > 0) {
            DY[iriv] = 0.;
        } else {
            DY[iriv] = (-M->QrivUp[i] - M->QrivSurf[i] - M->QrivSub[i] - M->QrivDown[i] + M->r_qBC[i]) / M->riv_length[i];
            if (DY[iriv] < -1. * M->r_CSarea[i]) DY[iriv] = -1. * M->r_CSarea[i];
            DY[iriv] = fun_dAtodY(DY[iriv], M->r_topWidth[i], M->riv_bankslope[i]);
        }
    }
    for (int i = 0; i < M->NL; i++)                           /* MD_f.cpp:180-190 */
        DY[3 * NE + NR + i] = M->qLakePrcp[i] - M->qLakeEvap[i] +
                              (M->QLakeRivIn[i] - M->QLakeRivOut[i] + M->QLakeSub[i] + M->QLakeSurf[i]) / M->y2LakeArea[i];
    return 0;
}
/* MD_f_omp.cpp:9-67 Model_Data::f_applyDY_omp (race-free restatement of the shared area/isf/ius/igw) */
static void f_applyDY_omp(OracleModel *M, double *DY) {
    int NE = M->NE, NR = M->NR;
#pragma omp parallel for num_threads(NT) schedule(static)
    for (int i = 0; i < NE; i++) {
        int isf = i, ius = i + NE, igw = i + 2 * NE;
        double area = M->area[i];
        M->QeleSurfTot[i] = M->Qe2r_Surf[i];
        M->QeleSubTot[i] = M->Qe2r_Sub[i];
        for (int j = 0; j < 3; j++) {
            M->QeleSurfTot[i] += M->QeleSurf[i * 3 + j];
            M->QeleSubTot[i] += M->QeleSub[i * 3 + j];
        }
        DY[i] = M->qEleNetPrep[i] - M->qEleInfil[i] + M->qEleExfil[i] - M->QeleSurfTot[i] / area - M->qEs[i];
        DY[ius] = M->qEleInfil[i] - M->qEleRecharge[i] - M->qEu[i] - M->qTu[i];
        DY[igw] = M->qEleRecharge[i] - M->qEleExfil[i] - M->QeleSubTot[i] / area - M->qEg[i] - M->qTg[i];
        if (M->ibc[i] == 0) {
        } else if (M->ibc[i] > 0) DY[igw] = 0;
        else DY[igw] += M->QBC[i] / area;
        if (M->iss[i] == 0) {
        } else if (M->iss[i] > 0) DY[isf] += 0.0 / area;
        else DY[igw] += 0.0 / area;
        DY[ius] /= M->Sy[i];
        DY[igw] /= M->Sy[i];
    }
#pragma omp parallel for num_threads(NT) schedule(static)
    for (int i = 0; i < NR; i++) {
        int iriv = i + 3 * NE;
        if (M->riv_bc[i] > 0) DY[iriv] = 0.;
        else DY[iriv] = (-M->QrivUp[i] - M->QrivSurf[i] - M->QrivSub[i] - M->QrivDown[i] + M->r_qBC[i]) / M->r_TopArea[i];
    }
}

/* src/Model/f.cpp:2-32.  Returns the myexit() code the reference would have terminated with
 * (0 = normal return). */
int oracle_f(OracleModel *M, double t, const double *Y, double *DY) {
    M->exit_code = 0; M->exit_index = -1; M->exit_kind = 0;
    int rc;
    if (M->mode == SHUD_MODE_OMP) {
        f_update_omp(M, Y, DY, t);
        rc = f_loop(M);
        if (!rc) f_applyDY_omp(M, DY);
    } else {
        f_update(M, Y, DY, t);
        rc = f_loop(M);
        if (!rc) rc = f_applyDY(M, DY);
    }
    M->nFCall++;
    return M->exit_code;
}

int oracle_exit_index(OracleModel *M) { return M->exit_index; }
int oracle_exit_kind(OracleModel *M) { return M->exit_kind; }
long long oracle_num_calls(OracleModel *M) { return M->nFCall; }
long long oracle_num_warn(OracleModel *M) { return M->n_aet_warn; }

static void cp_out(double *dst, const double *src, int n) { if (dst) memcpy(dst, src, sizeof(double) * n); }
void oracle_get_diag(OracleModel *M, ShudFluxOut *o) {
    int NE = M->NE, NR = M->NR, NS = M->NS;
    if (o->qele_surf) for (int i = 0; i < NE; i++) for (int j = 0; j < 3; j++) o->qele_surf[j * NE + i] = M->QeleSurf[i * 3 + j];
    if (o->qele_sub) for (int i = 0; i < NE; i++) for (int j = 0; j < 3; j++) o->qele_sub[j * NE + i] = M->QeleSub[i * 3 + j];
    cp_out(o->qele_surf_tot, M->QeleSurfTot, NE); cp_out(o->qele_sub_tot, M->QeleSubTot, NE);
    cp_out(o->q_infil, M->qEleInfil, NE); cp_out(o->q_exfil, M->qEleExfil, NE); cp_out(o->q_recharge, M->qEleRecharge, NE);
    cp_out(o->q_es, M->qEs, NE); cp_out(o->q_eu, M->qEu, NE); cp_out(o->q_eg, M->qEg, NE);
    cp_out(o->q_tu, M->qTu, NE); cp_out(o->q_tg, M->qTg, NE); cp_out(o->q_eta, M->qEleETA, NE);
    cp_out(o->e_ic, M->qEleE_IC, NE); cp_out(o->u_satn, M->u_satn, NE); cp_out(o->i_beta, M->iBeta, NE);
    cp_out(o->eff_kh, M->u_effKH, NE);
    cp_out(o->qe2r_surf, M->Qe2r_Surf, NE); cp_out(o->qe2r_sub, M->Qe2r_Sub, NE);
    cp_out(o->qseg_surf, M->QsegSurf, NS); cp_out(o->qseg_sub, M->QsegSub, NS);
    cp_out(o->qriv_down, M->QrivDown, NR); cp_out(o->qriv_up, M->QrivUp, NR);
    cp_out(o->qriv_surf, M->QrivSurf, NR); cp_out(o->qriv_sub, M->QrivSub, NR);
    int NL = M->NL;
    cp_out(o->q_lake_surf, M->QLakeSurf, NL); cp_out(o->q_lake_sub, M->QLakeSub, NL);
    cp_out(o->q_lake_rivin, M->QLakeRivIn, NL); cp_out(o->q_lake_evap, M->qLakeEvap, NL);
    cp_out(o->q_lake_prcp, M->qLakePrcp, NL); cp_out(o->lake_toparea, M->y2LakeArea, NL);
}

void oracle_destroy(OracleModel *M) {
    if (!M) return;
    void **p = (void **)&M->nabr;
    /* every pointer member from nabr up to QsegSub is a heap array */
    void **end = (void **)&M->QsegSub;
    for (; p <= end; p++) free(*p);
    free(M);
}

/* ===================== known-answer entry =====================
 * oracle_kat(fn, in, n, out): the leaf equations above on n input tuples (row-major, kat_nin(fn) doubles
 * each), one output per tuple.  The device side (shud-up_amd/csrc/shud_kat.hip) evaluates the same ids
 * with the kernels' own device functions; tests/test_kat.py compares them on edge-case grids. */
enum { KAT_MANNING, KAT_EFFKH, KAT_WEIR, KAT_R2E, KAT_SATK, KAT_SMS, KAT_DADY, KAT_AREA, KAT_PEREM, KAT_TOPW,
       KAT_TOPAREA, KAT_COUNT };
static const int kat_nin_tab[KAT_COUNT] = {4, 6, 8, 8, 2, 3, 3, 4, 4, 4, 4};
int oracle_kat_nin(int fn) { return (fn >= 0 && fn < KAT_COUNT) ? kat_nin_tab[fn] : -1; }
int oracle_kat(int fn, const double *in, int n, double *out) {
    if (fn < 0 || fn >= KAT_COUNT) return -1;
    const int k = kat_nin_tab[fn];
    for (int t = 0; t < n; t++) {
        const double *x = in + (size_t)t * k;
        double r = 0.;
        int bad = 0;
        switch (fn) {
            case KAT_MANNING: r = ManningEquation(x[0], x[1], x[2], x[3]); break;
            case KAT_EFFKH: r = effKH(x[0], x[1], x[2], x[3], x[4], x[5], &bad); break;
            case KAT_WEIR: r = WeirFlow_jtoi(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]); break;
            case KAT_R2E: r = flux_R2E_GW(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]); break;
            case KAT_SATK: r = satKfun(x[0], x[1]); break;
            case KAT_SMS: r = SoilMoistureStress(x[0], x[1], x[2]); break;
            case KAT_DADY: r = fun_dAtodY(x[0], x[1], x[2]); break;
            case KAT_AREA: r = fixMaxValue(fun_CrossArea(x[3], x[0], x[1]), 0.); break;
            case KAT_PEREM: r = fixMaxValue(fun_CrossPerem(x[3], x[0], x[1]), 0.); break;
            case KAT_TOPW: r = fixMaxValue(fun_TopWidth(x[3], x[0], x[1]), 0.); break;
            case KAT_TOPAREA: r = fixMaxValue(fun_EqWidth(x[3], x[0], x[1]) * x[2], 0.); break;
        }
        out[t] = r;
    }
    return 0;
}
