/* oracle/shud_oracle_ode.c — TEST INFRASTRUCTURE ONLY (the checker for the device integrator, never shipped).
 *
 * CPU restatement of the time integrator the reference drives its RHS with: SUNDIALS CVODE 6.0.0 (the version
 * the reference's installer pins, configure:17; SUNDIALS itself is not vendored under /root/reference and is not
 * installed here) configured as SetCVODE does (src/Equations/cvode_config.cpp:149-197):
 *   CVodeCreate(CV_BDF)                                   variable-order (1..5) variable-step BDF, Nordsieck form
 *   CVodeSStolerances(reltol, abstol)                     ewt = 1/(reltol|y| + abstol)
 *   SUNLinSol_SPGMR(udata, 0, 0) + CVodeSetLinearSolver   Newton iteration, GMRES maxl 5, no preconditioner,
 *                                                         modified Gram-Schmidt, 0 restarts, DQ J*v products
 *   CVodeSetMinStep(1e-6), SetMaxNumSteps(1e6), SetInitStep(InitStep), SetMaxStep(MaxStep)
 * and driven as SHUD() does (src/Model/shud.cpp:89-131): CVode(mem, tout, y, &t, CV_NORMAL) per solver step, with
 * CVodeSetStopTime(tout) when ET sub-stepping is on.
 *
 * The algorithm restated is CVODE's published one (Hindmarsh et al., ACM TOMS 31(3) 2005; CVODE v6 user guide
 * §2 "Mathematical considerations"), routine by routine: cvStep, cvPredict, cvSetBDF/cvSetTqBDF, cvNls with the
 * Newton SUNNonlinearSolver and its convergence test, cvLsSolve + SPGMR (SUNModifiedGS, SUNQRfact, SUNQRsol),
 * cvLsDQJtimes, cvDoErrorTest, cvCompleteStep, cvPrepareNextStep/cvChooseEta/cvSetEta, cvAdjustOrder
 * (cvIncreaseBDF/cvDecreaseBDF), cvRescale, cvRestore, CVodeGetDky, the CVode stop-condition logic, and the
 * N_Vector serial kernels' arithmetic special cases (N_VLinearSum's a=±1/b=±1/a=±b forms).  cvHin is not restated:
 * every SHUD configuration sets INIT_SOLVER_STEP > 0 (Model_Control.hpp:178), and init_step <= 0 is rejected.
 *
 * Parity status: SUNDIALS cannot run here, so this restatement is pinned by published known answers
 * (Robertson kinetics, linear decay vs exp; tests/test_ode.py), not by CVODE itself ("parity unpinned" w.r.t.
 * SUNDIALS).  The device integrator (shud-up_amd/csrc/shud_ode.cpp) is checked against this file.
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ODE_SUCCESS 0
#define ODE_TSTOP_RETURN 1
#define ODE_TOO_MUCH_WORK -1
#define ODE_TOO_MUCH_ACC -2
#define ODE_ERR_FAILURE -3
#define ODE_CONV_FAILURE -4
#define ODE_LSOLVE_FAIL -7
#define ODE_RHSFUNC_FAIL -8
#define ODE_ILL_INPUT -22
#define ODE_BAD_T -25

/* cvode.c constants */
#define UROUND DBL_EPSILON
#define FUZZ_FACTOR 100.0
#define ETAMX1 10000.0
#define ETAMX2 10.0
#define ETAMX3 10.0
#define ETAMXF 0.2
#define ETAMIN 0.1
#define ETACF 0.25
#define ADDON 0.000001
#define BIAS1 6.0
#define BIAS2 6.0
#define BIAS3 10.0
#define ONEPSM 1.000001
#define THRESH 1.5
#define SMALL_NST 10
#define MXNCF 10
#define MXNEF 7
#define MXNEF1 3
#define SMALL_NEF 2
#define LONG_WAIT 10
#define MSBP 20
#define DGMAX 0.3
#define CRDOWN 0.3
#define RDIV 2.0
#define NLS_MAXCOR 3
#define NLSCOEF 0.1
/* cvode_ls.c */
#define CVLS_EPLIN 0.05
#define CVLS_MSBJ 51
#define CVLS_DGMAX 0.2
#define MAX_DQITERS 3
/* cvNls flags */
#define FIRST_CALL 0
#define PREV_CONV_FAIL 1
#define PREV_ERR_FAIL 2
#define CV_NO_FAILURES 0
#define CV_FAIL_BAD_J 1
#define CV_FAIL_OTHER 2
#define NLS_CONTINUE 901
#define NLS_CONV_RECVR 902
#define DO_ERROR_TEST 2
#define PREDICT_AGAIN 3
#define TRY_AGAIN 5
#define QMAX 5
#define MAXL_MAX 32

typedef int (*ode_rhs_fn)(double t, const double *y, double *ydot, void *user);

typedef struct {
    long n;
    ode_rhs_fn f;
    void *user;
    double rtol, atol, hin, hmin, hmax_inv;
    long mxstep;
    int maxl, qmax, gstype;
    /* vectors */
    double *zn[QMAX + 1], *ewt, *y, *acor, *tempv, *ftemp, *delta, *work, *jv;   /* jv: SPGMR solution x */
    double *V[MAXL_MAX + 1], *xcor, *vtemp;
    double Hes[MAXL_MAX + 1][MAXL_MAX], givens[2 * MAXL_MAX], yg[MAXL_MAX + 1];
    /* integrator scalars (cvode_impl.h names) */
    double tn, h, hprime, next_h, eta, etamax, hscale, h0u, hu, tau[QMAX + 2], tq[6], l[QMAX + 1];
    double rl1, gamma, gammap, gamrat, crate, delp, acnrm, saved_tq5, tstop, tretlast, tolsf;
    double etaq, etaqm1, etaqp1, nrmfac;
    int tstopset, q, qprime, next_q, qwait, L, qu, indx_acor, convfail, jcur, jbad, curiter;
    long nst, nscon, nstlp, nfe, nfeDQ, nni, nnf, ncfn, netf, nsetups, nli, ncfl, njtimes, nhnil;
    int initialized;
} OracleOde;

/* ---------------- N_Vector serial arithmetic (nvector_serial.c) ---------------- */
static void v_const(long n, double c, double *z) { for (long i = 0; i < n; ++i) z[i] = c; }

static void v_scale(long n, double c, const double *x, double *z) {
    if (z == x) { for (long i = 0; i < n; ++i) z[i] *= c; return; }
    if (c == 1.0) { for (long i = 0; i < n; ++i) z[i] = x[i]; return; }
    if (c == -1.0) { for (long i = 0; i < n; ++i) z[i] = -x[i]; return; }
    for (long i = 0; i < n; ++i) z[i] = c * x[i];
}

static void v_axpy(long n, double a, const double *x, double *y) {  /* Vaxpy_Serial */
    if (a == 1.0) { for (long i = 0; i < n; ++i) y[i] += x[i]; return; }
    if (a == -1.0) { for (long i = 0; i < n; ++i) y[i] -= x[i]; return; }
    for (long i = 0; i < n; ++i) y[i] += a * x[i];
}

static void v_linear_sum(long n, double a, const double *x, double b, const double *y, double *z) {
    int test;
    const double *v1, *v2;
    double c;
    if (b == 1.0 && z == y) { v_axpy(n, a, x, (double *)y); return; }
    if (a == 1.0 && z == x) { v_axpy(n, b, y, (double *)x); return; }
    if (a == 1.0 && b == 1.0) { for (long i = 0; i < n; ++i) z[i] = x[i] + y[i]; return; }
    if ((test = (a == 1.0 && b == -1.0)) || (a == -1.0 && b == 1.0)) {
        v1 = test ? y : x; v2 = test ? x : y;
        for (long i = 0; i < n; ++i) z[i] = v2[i] - v1[i];
        return;
    }
    if ((test = (a == 1.0)) || b == 1.0) {
        c = test ? b : a; v1 = test ? y : x; v2 = test ? x : y;
        for (long i = 0; i < n; ++i) z[i] = (c * v1[i]) + v2[i];
        return;
    }
    if ((test = (a == -1.0)) || b == -1.0) {
        c = test ? b : a; v1 = test ? y : x; v2 = test ? x : y;
        for (long i = 0; i < n; ++i) z[i] = (c * v1[i]) - v2[i];
        return;
    }
    if (a == b) { for (long i = 0; i < n; ++i) z[i] = a * (x[i] + y[i]); return; }
    if (a == -b) { for (long i = 0; i < n; ++i) z[i] = a * (x[i] - y[i]); return; }
    for (long i = 0; i < n; ++i) z[i] = (a * x[i]) + (b * y[i]);
}

/* Reduction order.  0: the serial N_Vector's (one left-to-right sum, nvector_serial.c) — CVODE's own order.
 * 1: the device integrator's fixed order (shud-up_amd/csrc/shud_ode_kernels.hip, round 3): one entry per thread on
 * a grid of B = ceil(n/1024) blocks x 1024 threads; thread (b, t) holds 0.0 + term[b*1024 + t] (0.0 past n); each
 * 64-lane wave combines by an xor butterfly (offsets 32..1, own value first) and lane 0 keeps the result; the block
 * combines its 16 wave results by an xor butterfly over offsets 8..1 (lane 0) into partial[b].  The one-block finalize (1024 threads): thread t keeps 4
 * accumulators from 0.0, acc[k] += partial[t + (4j + k)*1024] for j = 0, 1, ... (0.0 past B); x = (acc0 + acc1) +
 * (acc2 + acc3); wave butterfly; the 16 wave results by the 16-lane butterfly.  With order 1 the restatement reproduces the
 * device integrator bit for bit wherever the RHS is IEEE-exact (tests/test_gpu_ode.py).  (Round 2's order — a
 * 2048-block grid-stride loop of 256-thread blocks — ran the five-operand passes at 4.7 TB/s against 5.7 TB/s
 * one-shot: profiles/r03/ode/.) */
#define ORACLE_RED_THREADS 1024   /* shud_ode_dev.h kRedThreads */
#define ORACLE_FIN_THREADS 1024   /* kFinThreads */
#define ORACLE_FIN_ACC 4          /* kFinAcc */
static int g_red_order = 0;
void oracle_ode_set_reduction_order(int order) { g_red_order = order; }

static double wave_butterfly(double *x) {        /* x[64], destroyed; returns lane 0 */
    double y[64];
    for (int off = 32; off >= 1; off >>= 1) {
        for (int l = 0; l < 64; ++l) y[l] = x[l] + x[l ^ off];
        memcpy(x, y, sizeof(y));
    }
    return x[0];
}

/* lanes[nthreads] -> each wave's butterfly result, then those nw = nthreads/64 results by an xor butterfly over
 * offsets nw/2 .. 1 (kernel waves_tree), lane 0 */
static double waves_in_order(double *lanes, int nthreads) {
    const int nw = nthreads / 64;
    double w[64], y[64];
    for (int k = 0; k < nw; ++k) w[k] = wave_butterfly(lanes + 64 * k);
    for (int off = nw / 2; off >= 1; off >>= 1) {
        for (int l = 0; l < nw; ++l) y[l] = w[l] + w[l ^ off];
        memcpy(w, y, nw * sizeof(double));
    }
    return w[0];
}

static double device_order_sum(long n, const double *term) {
    long nb = (n + ORACLE_RED_THREADS - 1) / ORACLE_RED_THREADS;
    if (nb < 1) nb = 1;
    static double *part = NULL;
    static long part_n = 0;
    if (nb > part_n) { free(part); part = (double *)malloc(nb * sizeof(double)); part_n = nb; }
    double lanes[ORACLE_RED_THREADS > ORACLE_FIN_THREADS ? ORACLE_RED_THREADS : ORACLE_FIN_THREADS];
    for (long b = 0; b < nb; ++b) {
        for (int t = 0; t < ORACLE_RED_THREADS; ++t) {
            const long i = b * ORACLE_RED_THREADS + t;
            lanes[t] = i < n ? 0.0 + term[i] : 0.0;
        }
        part[b] = waves_in_order(lanes, ORACLE_RED_THREADS);
    }
    for (int t = 0; t < ORACLE_FIN_THREADS; ++t) {
        double acc[ORACLE_FIN_ACC];
        for (int k = 0; k < ORACLE_FIN_ACC; ++k) acc[k] = 0.0;
        for (long b0 = t; b0 < nb; b0 += (long)ORACLE_FIN_ACC * ORACLE_FIN_THREADS)
            for (int k = 0; k < ORACLE_FIN_ACC; ++k) {
                const long b = b0 + (long)k * ORACLE_FIN_THREADS;
                acc[k] = acc[k] + (b < nb ? part[b] : 0.0);
            }
        lanes[t] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    }
    return waves_in_order(lanes, ORACLE_FIN_THREADS);
}

static double *g_term = NULL;
static long g_term_n = 0;
static double *term_buf(long n) {
    if (n > g_term_n) { free(g_term); g_term = (double *)malloc(n * sizeof(double)); g_term_n = n; }
    return g_term;
}

static double v_dot(long n, const double *x, const double *y) {
    if (g_red_order == 1) {
        double *t = term_buf(n);
        for (long i = 0; i < n; ++i) t[i] = x[i] * y[i];
        return device_order_sum(n, t);
    }
    double s = 0.0;
    for (long i = 0; i < n; ++i) s += x[i] * y[i];
    return s;
}

static double v_wrms(long n, const double *x, const double *w) {
    if (g_red_order == 1) {
        double *t = term_buf(n);
        for (long i = 0; i < n; ++i) { double p = x[i] * w[i]; t[i] = p * p; }
        return sqrt(device_order_sum(n, t) / (double)n);
    }
    double s = 0.0;
    for (long i = 0; i < n; ++i) { double p = x[i] * w[i]; s += p * p; }
    return sqrt(s / (double)n);
}

/* N_VLinearCombination_Serial: z = sum c[i] X[i] */
static void v_lincomb(long n, int nvec, const double *c, double *const *X, double *z) {
    if (nvec == 1) { v_scale(n, c[0], X[0], z); return; }
    if (nvec == 2) { v_linear_sum(n, c[0], X[0], c[1], X[1], z); return; }
    if (X[0] == z) {
        if (c[0] == 1.0) {
            for (int i = 1; i < nvec; ++i) for (long j = 0; j < n; ++j) z[j] += c[i] * X[i][j];
            return;
        }
        for (long j = 0; j < n; ++j) z[j] *= c[0];
        for (int i = 1; i < nvec; ++i) for (long j = 0; j < n; ++j) z[j] += c[i] * X[i][j];
        return;
    }
    for (long j = 0; j < n; ++j) z[j] = c[0] * X[0][j];
    for (int i = 1; i < nvec; ++i) for (long j = 0; j < n; ++j) z[j] += c[i] * X[i][j];
}

static double rpower_r(double base, double e) { return base <= 0.0 ? 0.0 : pow(base, e); }  /* SUNRpowerR */
static double rpower_i(double base, int e) {                                                /* SUNRpowerI */
    double p = 1.0;
    for (int i = 1; i <= abs(e); ++i) p *= base;
    return e < 0 ? 1.0 / p : p;
}

/* cvEwtSetSS */
static int ewt_set(OracleOde *O, const double *ycur) {
    double mn = INFINITY;
    for (long i = 0; i < O->n; ++i) {
        double t = O->rtol * fabs(ycur[i]) + O->atol;
        if (t < mn) mn = t;
        O->tempv[i] = t;
    }
    if (mn <= 0.0) return -1;
    for (long i = 0; i < O->n; ++i) O->ewt[i] = 1.0 / O->tempv[i];
    return 0;
}

/* ---------------- create / destroy ---------------- */
OracleOde *oracle_ode_create(long n, ode_rhs_fn f, void *user, double t0, const double *y0, double rtol, double atol,
                             double init_step, double max_step, double min_step, long max_num_steps, int maxl,
                             int max_order) {
    if (n <= 0 || !f || !(init_step > 0.0) || rtol < 0.0 || atol < 0.0) return NULL;
    if (maxl <= 0) maxl = 5;                             /* SUNSPGMR_MAXL_DEFAULT */
    if (maxl > MAXL_MAX) return NULL;
    if (max_order <= 0 || max_order > QMAX) max_order = QMAX;
    OracleOde *O = (OracleOde *)calloc(1, sizeof(OracleOde));
    O->n = n; O->f = f; O->user = user;
    O->rtol = rtol; O->atol = atol; O->hin = init_step;
    O->hmin = min_step > 0.0 ? min_step : 0.0;
    O->hmax_inv = max_step > 0.0 ? 1.0 / max_step : 0.0;
    O->mxstep = max_num_steps > 0 ? max_num_steps : 500;
    O->maxl = maxl; O->qmax = max_order;
    for (int j = 0; j <= O->qmax; ++j) O->zn[j] = (double *)calloc(n, sizeof(double));
    double **vecs[] = {&O->ewt, &O->y, &O->acor, &O->tempv, &O->ftemp, &O->delta, &O->work, &O->jv, &O->xcor,
                       &O->vtemp};
    for (unsigned k = 0; k < sizeof(vecs) / sizeof(vecs[0]); ++k) *vecs[k] = (double *)calloc(n, sizeof(double));
    for (int j = 0; j <= maxl; ++j) O->V[j] = (double *)calloc(n, sizeof(double));
    /* CVodeInit (cvode.c): zn[0] = y0, q = 1, L = 2, qwait = L, etamax = ETAMX1 */
    memcpy(O->zn[0], y0, n * sizeof(double));
    O->tn = t0; O->q = 1; O->L = 2; O->qwait = O->L; O->etamax = ETAMX1;
    O->qu = 0; O->hu = 0.0; O->tolsf = 1.0; O->indx_acor = O->qmax;
    O->nrmfac = sqrt((double)n);                         /* cvLs: sqrt(N) converts WRMS to 2-norm tolerance */
    return O;
}

void oracle_ode_destroy(OracleOde *O) {
    if (!O) return;
    for (int j = 0; j <= O->qmax; ++j) free(O->zn[j]);
    free(O->ewt); free(O->y); free(O->acor); free(O->tempv); free(O->ftemp); free(O->delta); free(O->work);
    free(O->jv); free(O->xcor); free(O->vtemp);
    for (int j = 0; j <= O->maxl; ++j) free(O->V[j]);
    free(O);
}

void oracle_ode_set_stop_time(OracleOde *O, double tstop) { O->tstop = tstop; O->tstopset = 1; }

/* ---------------- BDF coefficient / history management ---------------- */
static void set_tq_bdf(OracleOde *O, double hsum, double alpha0, double alpha0_hat, double xi_inv,
                       double xistar_inv) {                                     /* cvSetTqBDF */
    double A1 = 1.0 - alpha0_hat + alpha0;
    double A2 = 1.0 + O->q * A1;
    O->tq[2] = fabs(A1 / (alpha0 * A2));
    O->tq[5] = fabs(A2 * xistar_inv / (O->l[O->q] * xi_inv));
    if (O->qwait == 1) {
        if (O->q > 1) {
            double C = xistar_inv / O->l[O->q];
            double A3 = alpha0 + 1.0 / O->q;
            double A4 = alpha0_hat + xi_inv;
            double Cpinv = (1.0 - A4 + A3) / A3;
            O->tq[1] = fabs(C * Cpinv);
        } else {
            O->tq[1] = 1.0;
        }
        hsum += O->tau[O->q];
        xi_inv = O->h / hsum;
        double A5 = alpha0 - (1.0 / (O->q + 1));
        double A6 = alpha0_hat - xi_inv;
        double Cppinv = (1.0 - A6 + A5) / A2;
        O->tq[3] = fabs(Cppinv / (xi_inv * (O->q + 2) * A5));
    }
    O->tq[4] = NLSCOEF / O->tq[2];
}

static void set_bdf(OracleOde *O) {                                              /* cvSetBDF */
    double alpha0, alpha0_hat, xi_inv, xistar_inv, hsum;
    O->l[0] = O->l[1] = xi_inv = xistar_inv = 1.0;
    for (int i = 2; i <= O->q; ++i) O->l[i] = 0.0;
    alpha0 = alpha0_hat = -1.0;
    hsum = O->h;
    if (O->q > 1) {
        for (int j = 2; j < O->q; ++j) {
            hsum += O->tau[j - 1];
            xi_inv = O->h / hsum;
            alpha0 -= 1.0 / j;
            for (int i = j; i >= 1; --i) O->l[i] += O->l[i - 1] * xi_inv;
        }
        alpha0 -= 1.0 / O->q;
        xistar_inv = -O->l[1] - alpha0;
        hsum += O->tau[O->q - 1];
        xi_inv = O->h / hsum;
        alpha0_hat = -O->l[1] - xi_inv;
        for (int i = O->q; i >= 1; --i) O->l[i] += O->l[i - 1] * xistar_inv;
    }
    set_tq_bdf(O, hsum, alpha0, alpha0_hat, xi_inv, xistar_inv);
}

static void cv_set(OracleOde *O) {                                               /* cvSet */
    set_bdf(O);
    O->rl1 = 1.0 / O->l[1];
    O->gamma = O->h * O->rl1;
    if (O->nst == 0) O->gammap = O->gamma;
    O->gamrat = (O->nst > 0) ? O->gamma / O->gammap : 1.0;
}

static void predict(OracleOde *O) {                                              /* cvPredict */
    long n = O->n;
    O->tn += O->h;
    if (O->tstopset && (O->tn - O->tstop) * O->h > 0.0) O->tn = O->tstop;
    for (int k = 1; k <= O->q; ++k)
        for (int j = O->q; j >= k; --j) v_linear_sum(n, 1.0, O->zn[j - 1], 1.0, O->zn[j], O->zn[j - 1]);
}

static void restore(OracleOde *O, double saved_t) {                              /* cvRestore */
    long n = O->n;
    O->tn = saved_t;
    for (int k = 1; k <= O->q; ++k)
        for (int j = O->q; j >= k; --j) v_linear_sum(n, 1.0, O->zn[j - 1], -1.0, O->zn[j], O->zn[j - 1]);
}

static void rescale(OracleOde *O) {                                              /* cvRescale */
    double c = O->eta;
    for (int j = 1; j <= O->q; ++j) {
        for (long i = 0; i < O->n; ++i) O->zn[j][i] *= c;                        /* N_VScaleVectorArray */
        c = O->eta * c;
    }
    O->h = O->hscale * O->eta;
    O->next_h = O->h;
    O->hscale = O->h;
    O->nscon = 0;
}

static void increase_bdf(OracleOde *O) {                                         /* cvIncreaseBDF */
    double alpha0, alpha1, prod, xi, xiold, hsum, A1;
    for (int i = 0; i <= O->qmax; ++i) O->l[i] = 0.0;
    O->l[2] = alpha1 = prod = xiold = 1.0;
    alpha0 = -1.0;
    hsum = O->hscale;
    if (O->q > 1) {
        for (int j = 1; j < O->q; ++j) {
            hsum += O->tau[j + 1];
            xi = hsum / O->hscale;
            prod *= xi;
            alpha0 -= 1.0 / (j + 1);
            alpha1 += 1.0 / xi;
            for (int i = j + 2; i >= 2; --i) O->l[i] = O->l[i] * xiold + O->l[i - 1];
            xiold = xi;
        }
    }
    A1 = (-alpha0 - alpha1) / prod;
    v_scale(O->n, A1, O->zn[O->indx_acor], O->zn[O->L]);
    for (int j = 2; j <= O->q; ++j)                                              /* N_VScaleAddMulti */
        for (long i = 0; i < O->n; ++i) O->zn[j][i] = O->l[j] * O->zn[O->L][i] + O->zn[j][i];
}

static void decrease_bdf(OracleOde *O) {                                         /* cvDecreaseBDF */
    double hsum, xi;
    for (int i = 0; i <= O->qmax; ++i) O->l[i] = 0.0;
    O->l[2] = 1.0;
    hsum = 0.0;
    for (int j = 1; j <= O->q - 2; ++j) {
        hsum += O->tau[j];
        xi = hsum / O->hscale;
        for (int i = j + 2; i >= 2; --i) O->l[i] = O->l[i] * xi + O->l[i - 1];
    }
    for (int j = 2; j < O->q; ++j)
        for (long i = 0; i < O->n; ++i) O->zn[j][i] = -O->l[j] * O->zn[O->q][i] + O->zn[j][i];
}

static void adjust_order(OracleOde *O, int deltaq) {                             /* cvAdjustOrder (BDF) */
    if (O->q == 2 && deltaq != 1) return;                                        /* cvAdjustOrder: q==2 && deltaq!=1 */
    if (deltaq == 1) increase_bdf(O);
    else if (deltaq == -1) decrease_bdf(O);
}

static void adjust_params(OracleOde *O) {                                        /* cvAdjustParams */
    if (O->qprime != O->q) {
        adjust_order(O, O->qprime - O->q);
        O->q = O->qprime;
        O->L = O->q + 1;
        O->qwait = O->L;
    }
    rescale(O);
}

/* ---------------- linear solver: cvLsSolve + SPGMR + cvLsDQJtimes ---------------- */
static int dq_jtimes(OracleOde *O, const double *v, double *Jv) {               /* cvLsDQJtimes */
    long n = O->n;
    double sig = 1.0 / v_wrms(n, v, O->ewt);
    int rv = 0;
    for (int it = 0; it < MAX_DQITERS; ++it) {
        v_linear_sum(n, sig, v, 1.0, O->y, O->work);
        rv = O->f(O->tn, O->work, Jv, O->user);
        O->nfeDQ++;
        if (rv == 0) break;
        if (rv < 0) return -1;
        sig *= 0.25;
    }
    if (rv > 0) return 1;
    double siginv = 1.0 / sig;
    v_linear_sum(n, siginv, Jv, -siginv, O->ftemp, Jv);
    return 0;
}

static int atimes(OracleOde *O, const double *v, double *z) {                   /* cvLsATimes */
    int rv = dq_jtimes(O, v, z);
    O->njtimes++;
    if (rv != 0) return rv;
    v_linear_sum(O->n, 1.0, v, -O->gamma, z, z);
    return 0;
}

static int modified_gs(OracleOde *O, int k, double *new_vk_norm) {              /* SUNModifiedGS */
    long n = O->n;
    double **v = O->V;
    double vk_norm = sqrt(v_dot(n, v[k], v[k]));
    int i0 = k - O->maxl > 0 ? k - O->maxl : 0;
    for (int i = i0; i < k; ++i) {
        O->Hes[i][k - 1] = v_dot(n, v[i], v[k]);
        v_linear_sum(n, 1.0, v[k], -O->Hes[i][k - 1], v[i], v[k]);
    }
    *new_vk_norm = sqrt(v_dot(n, v[k], v[k]));
    double temp = 1000.0 * vk_norm;
    if ((temp + (*new_vk_norm)) != temp) return 0;
    double new_norm_2 = 0.0;
    for (int i = i0; i < k; ++i) {
        double new_product = v_dot(n, v[i], v[k]);
        if (new_product == 0.0) continue;
        O->Hes[i][k - 1] += new_product;
        v_linear_sum(n, 1.0, v[k], -new_product, v[i], v[k]);
        new_norm_2 += new_product * new_product;
    }
    if (new_norm_2 != 0.0) {
        new_norm_2 = (*new_vk_norm) * (*new_vk_norm) - new_norm_2;
        *new_vk_norm = (new_norm_2 > 0.0) ? sqrt(new_norm_2) : 0.0;
    }
    return 0;
}

static void givens(double t1, double t2, double *c, double *s) {
    if (t2 == 0.0) { *c = 1.0; *s = 0.0; }
    else if (fabs(t2) >= fabs(t1)) { double t3 = t1 / t2; *s = -1.0 / sqrt(1.0 + t3 * t3); *c = -(*s) * t3; }
    else { double t3 = t2 / t1; *c = 1.0 / sqrt(1.0 + t3 * t3); *s = -(*c) * t3; }
}

static int qr_fact(OracleOde *O, int n, int job) {                              /* SUNQRfact */
    double (*h)[MAXL_MAX] = O->Hes;
    double *q = O->givens, c, s, t1, t2;
    int code = 0;
    if (job == 0) {
        for (int k = 0; k < n; ++k) {
            for (int j = 0; j < k - 1; ++j) {
                int i = 2 * j;
                t1 = h[j][k]; t2 = h[j + 1][k]; c = q[i]; s = q[i + 1];
                h[j][k] = c * t1 - s * t2;
                h[j + 1][k] = s * t1 + c * t2;
            }
            t1 = h[k][k]; t2 = h[k + 1][k];
            givens(t1, t2, &c, &s);
            q[2 * k] = c; q[2 * k + 1] = s;
            if ((h[k][k] = c * t1 - s * t2) == 0.0) code = k + 1;
        }
    } else {
        int nm1 = n - 1;
        for (int k = 0; k < nm1; ++k) {
            int i = 2 * k;
            t1 = h[k][nm1]; t2 = h[k + 1][nm1]; c = q[i]; s = q[i + 1];
            h[k][nm1] = c * t1 - s * t2;
            h[k + 1][nm1] = s * t1 + c * t2;
        }
        t1 = h[nm1][nm1]; t2 = h[n][nm1];
        givens(t1, t2, &c, &s);
        q[2 * nm1] = c; q[2 * nm1 + 1] = s;
        if ((h[nm1][nm1] = c * t1 - s * t2) == 0.0) code = n;
    }
    return code;
}

static int qr_sol(OracleOde *O, int n) {                                         /* SUNQRsol */
    double (*h)[MAXL_MAX] = O->Hes;
    double *q = O->givens, *b = O->yg;
    for (int k = 0; k < n; ++k) {
        double c = q[2 * k], s = q[2 * k + 1], t1 = b[k], t2 = b[k + 1];
        b[k] = c * t1 - s * t2;
        b[k + 1] = s * t1 + c * t2;
    }
    for (int k = n - 1; k >= 0; --k) {
        if (h[k][k] == 0.0) return k + 1;
        b[k] /= h[k][k];
        for (int i = 0; i < k; ++i) b[i] -= b[k] * h[i][k];
    }
    return 0;
}

#define LS_SUCCESS 0
#define LS_RES_REDUCED 1
#define LS_CONV_FAIL 2
#define LS_ATIMES_FAIL_REC 3
#define LS_ATIMES_FAIL_UNREC (-3)
#define LS_GS_FAIL (-5)
#define LS_QRSOL_FAIL (-6)

/* SUNLinSolSolve_SPGMR with s1 = s2 = ewt, no preconditioner, zero initial guess, max_restarts 0 */
static int spgmr_solve(OracleOde *O, double *x, const double *b, double delta, int *nli) {
    long n = O->n;
    const double *s = O->ewt;
    double **V = O->V, r_norm, beta, rho, rotation_product;
    int krydim = 0, converged = 0;
    *nli = 0;
    v_scale(n, 1.0, b, V[0]);                                 /* r_0 = b (x_0 = 0) */
    for (long i = 0; i < n; ++i) O->vtemp[i] = s[i] * V[0][i];/* left scaling: N_VProd(s1, V[0], vtemp) */
    r_norm = beta = sqrt(v_dot(n, O->vtemp, O->vtemp));
    if (r_norm <= delta) { v_const(n, 0.0, x); return LS_SUCCESS; }
    rho = beta;
    v_const(n, 0.0, O->xcor);
    for (int i = 0; i <= O->maxl; ++i) for (int j = 0; j < O->maxl; ++j) O->Hes[i][j] = 0.0;
    rotation_product = 1.0;
    v_scale(n, 1.0 / r_norm, O->vtemp, V[0]);
    for (int l = 0; l < O->maxl; ++l) {
        (*nli)++;
        krydim = l + 1;
        for (long i = 0; i < n; ++i) O->vtemp[i] = V[l][i] / s[i];   /* right scaling: N_VDiv(V[l], s2, vtemp) */
        int rv = atimes(O, O->vtemp, V[l + 1]);
        if (rv != 0) return rv < 0 ? LS_ATIMES_FAIL_UNREC : LS_ATIMES_FAIL_REC;
        for (long i = 0; i < n; ++i) O->vtemp[i] = V[l + 1][i];
        for (long i = 0; i < n; ++i) V[l + 1][i] = s[i] * O->vtemp[i];   /* N_VProd(s1, vtemp, V[l+1]) */
        if (modified_gs(O, l + 1, &O->Hes[l + 1][l]) != 0) return LS_GS_FAIL;
        if (qr_fact(O, krydim, l) != 0) return LS_QRSOL_FAIL;      /* SUNLS_QRFACT_FAIL */
        rotation_product *= O->givens[2 * l + 1];
        rho = fabs(rotation_product * r_norm);
        if (rho <= delta) { converged = 1; break; }
        v_scale(n, 1.0 / O->Hes[l + 1][l], V[l + 1], V[l + 1]);
    }
    O->yg[0] = r_norm;
    for (int i = 1; i <= krydim; ++i) O->yg[i] = 0.0;
    if (qr_sol(O, krydim) != 0) return LS_QRSOL_FAIL;
    {
        double cv[MAXL_MAX + 1];
        double *Xv[MAXL_MAX + 1];
        cv[0] = 1.0; Xv[0] = O->xcor;
        for (int k = 0; k < krydim; ++k) { cv[k + 1] = O->yg[k]; Xv[k + 1] = V[k]; }
        v_lincomb(n, krydim + 1, cv, Xv, O->xcor);
    }
    if (converged || rho < beta) {
        for (long i = 0; i < n; ++i) x[i] = O->xcor[i] / s[i];     /* N_VDiv(xcor, s2, xcor); x = xcor */
        return converged ? LS_SUCCESS : LS_RES_REDUCED;
    }
    return LS_CONV_FAIL;
}

static int ls_solve(OracleOde *O, double *b) {                                    /* cvLsSolve */
    long n = O->n;
    double deltar = CVLS_EPLIN * O->tq[4];
    double bnorm = v_wrms(n, b, O->ewt);
    if (bnorm <= deltar) {
        if (O->curiter > 0) v_const(n, 0.0, b);
        return 0;
    }
    double delta = deltar * O->nrmfac;
    int nli = 0;
    int rv = spgmr_solve(O, O->jv, b, delta, &nli);                   /* x = cvls_mem->x (scratch) */
    if (rv == LS_SUCCESS || rv == LS_RES_REDUCED) v_scale(n, 1.0, O->jv, b);   /* N_VScale(ONE, x, b) */
    O->nli += nli;
    if (rv != LS_SUCCESS) O->ncfl++;
    switch (rv) {
    case LS_SUCCESS: return 0;
    case LS_RES_REDUCED: return O->curiter == 0 ? 0 : 1;
    case LS_CONV_FAIL: case LS_ATIMES_FAIL_REC: return 1;
    default: return -1;
    }
}

/* ---------------- nonlinear solve: cvNls + SUNNonlinSol_Newton ---------------- */
static int nls_residual(OracleOde *O, const double *ycor, double *res) {          /* cvNlsResidual */
    long n = O->n;
    v_linear_sum(n, 1.0, O->zn[0], 1.0, ycor, O->y);
    int rv = O->f(O->tn, O->y, O->ftemp, O->user);
    O->nfe++;
    if (rv < 0) return ODE_RHSFUNC_FAIL;
    if (rv > 0) return NLS_CONV_RECVR;                                           /* RHSFUNC_RECVR */
    v_linear_sum(n, O->rl1, O->zn[1], 1.0, ycor, res);
    v_linear_sum(n, -O->gamma, O->ftemp, 1.0, res, res);
    return 0;
}

static int nls_lsetup(OracleOde *O, int jbad_in) {                                /* cvNlsLSetup + cvLsSetup */
    if (jbad_in) O->convfail = CV_FAIL_BAD_J;
    double dgamma = fabs((O->gamma / O->gammap) - 1.0);
    O->jbad = (O->nst == 0) || (O->nst >= 0 + CVLS_MSBJ) ||   /* nstlj stays 0: matrix-free */
              ((O->convfail == CV_FAIL_BAD_J) && (dgamma < CVLS_DGMAX)) || (O->convfail == CV_FAIL_OTHER);
    if (O->jbad) O->jcur = 1;                                  /* no preconditioner: SPGMR setup is a no-op */
    O->nsetups++;
    O->gamrat = 1.0;
    O->gammap = O->gamma;
    O->crate = 1.0;
    O->nstlp = O->nst;
    return 0;
}

static int nls_conv_test(OracleOde *O, const double *ycor, const double *del_v, double tol) {   /* cvNlsConvTest */
    double del = v_wrms(O->n, del_v, O->ewt);
    if (O->curiter > 0) O->crate = fmax(CRDOWN * O->crate, del / O->delp);
    double dcon = del * fmin(1.0, O->crate) / tol;
    if (dcon <= 1.0) {
        O->acnrm = (O->curiter == 0) ? del : v_wrms(O->n, ycor, O->ewt);
        return 0;
    }
    if (O->curiter >= 1 && del > RDIV * O->delp) return NLS_CONV_RECVR;
    O->delp = del;
    return NLS_CONTINUE;
}

static int nls(OracleOde *O, int nflag) {                                         /* cvNls + Newton solve */
    long n = O->n;
    int callSetup;
    O->convfail = (nflag == FIRST_CALL || nflag == PREV_ERR_FAIL) ? CV_NO_FAILURES : CV_FAIL_OTHER;
    callSetup = (nflag == PREV_CONV_FAIL) || (nflag == PREV_ERR_FAIL) || (O->nst == 0) ||
                (O->nst >= O->nstlp + MSBP) || (fabs(O->gamrat - 1.0) > DGMAX);
    v_const(n, 0.0, O->acor);
    double *ycor = O->acor, *delta = O->delta;
    int jbad = 0, rv = 0;
    for (;;) {
        rv = nls_residual(O, ycor, delta);
        if (rv != 0) break;
        if (callSetup) {
            rv = nls_lsetup(O, jbad);
            if (rv != 0) break;
        }
        O->curiter = 0;
        for (;;) {
            O->nni++;
            v_scale(n, -1.0, delta, delta);
            rv = ls_solve(O, delta);
            if (rv != 0) { rv = rv < 0 ? ODE_LSOLVE_FAIL : NLS_CONV_RECVR; break; }
            v_linear_sum(n, 1.0, ycor, 1.0, delta, ycor);
            rv = nls_conv_test(O, ycor, delta, O->tq[4]);
            if (rv == 0) { O->jcur = 0; return 0; }
            if (rv != NLS_CONTINUE) break;
            O->curiter++;
            if (O->curiter >= NLS_MAXCOR) { rv = NLS_CONV_RECVR; break; }
            rv = nls_residual(O, ycor, delta);
            if (rv != 0) break;
        }
        if (rv == NLS_CONV_RECVR && !O->jcur) {
            O->nnf++;
            callSetup = 1;
            jbad = 1;
            v_const(n, 0.0, ycor);
            continue;
        }
        break;
    }
    O->nnf++;
    return rv;
}

static int handle_nflag(OracleOde *O, int *nflagPtr, double saved_t, int *ncfPtr) {   /* cvHandleNFlag */
    int nflag = *nflagPtr;
    if (nflag == 0) return DO_ERROR_TEST;
    O->ncfn++;
    restore(O, saved_t);
    if (nflag < 0) return nflag;
    (*ncfPtr)++;
    O->etamax = 1.0;
    if (fabs(O->h) <= O->hmin * ONEPSM || *ncfPtr == MXNCF) return ODE_CONV_FAILURE;
    O->eta = fmax(ETACF, O->hmin / fabs(O->h));
    *nflagPtr = PREV_CONV_FAIL;
    rescale(O);
    return PREDICT_AGAIN;
}

static int do_error_test(OracleOde *O, int *nflagPtr, double saved_t, int *nefPtr, double *dsmPtr) {  /* cvDoErrorTest */
    double dsm = O->acnrm * O->tq[2];
    *dsmPtr = dsm;
    if (dsm <= 1.0) return ODE_SUCCESS;
    (*nefPtr)++;
    O->netf++;
    *nflagPtr = PREV_ERR_FAIL;
    restore(O, saved_t);
    if (fabs(O->h) <= O->hmin * ONEPSM || *nefPtr == MXNEF) return ODE_ERR_FAILURE;
    O->etamax = 1.0;
    if (*nefPtr <= MXNEF1) {
        O->eta = 1.0 / (rpower_r(BIAS2 * dsm, 1.0 / O->L) + ADDON);
        O->eta = fmax(ETAMIN, fmax(O->eta, O->hmin / fabs(O->h)));
        if (*nefPtr >= SMALL_NEF) O->eta = fmin(O->eta, ETAMXF);
        rescale(O);
        return TRY_AGAIN;
    }
    if (O->q > 1) {
        O->eta = fmax(ETAMIN, O->hmin / fabs(O->h));
        adjust_order(O, -1);
        O->L = O->q;
        O->q--;
        O->qwait = O->L;
        rescale(O);
        return TRY_AGAIN;
    }
    O->eta = fmax(ETAMIN, O->hmin / fabs(O->h));
    O->h *= O->eta;
    O->next_h = O->h;
    O->hscale = O->h;
    O->qwait = LONG_WAIT;
    O->nscon = 0;
    int rv = O->f(O->tn, O->zn[0], O->tempv, O->user);
    O->nfe++;
    if (rv != 0) return ODE_RHSFUNC_FAIL;
    v_scale(O->n, O->h, O->tempv, O->zn[1]);
    return TRY_AGAIN;
}

static void complete_step(OracleOde *O) {                                         /* cvCompleteStep */
    O->nst++;
    O->nscon++;
    O->hu = O->h;
    O->qu = O->q;
    for (int i = O->q; i >= 2; --i) O->tau[i] = O->tau[i - 1];
    if (O->q == 1 && O->nst > 1) O->tau[2] = O->tau[1];
    O->tau[1] = O->h;
    for (int j = 0; j <= O->q; ++j)                                              /* N_VScaleAddMulti */
        for (long i = 0; i < O->n; ++i) O->zn[j][i] = O->l[j] * O->acor[i] + O->zn[j][i];
    O->qwait--;
    if (O->qwait == 1 && O->q != O->qmax) {
        v_scale(O->n, 1.0, O->acor, O->zn[O->qmax]);
        O->saved_tq5 = O->tq[5];
        O->indx_acor = O->qmax;
    }
}

static void set_eta(OracleOde *O) {                                               /* cvSetEta */
    if (O->eta < THRESH) {
        O->eta = 1.0;
        O->hprime = O->h;
    } else {
        O->eta = fmin(O->eta, O->etamax);
        O->eta /= fmax(1.0, fabs(O->h) * O->hmax_inv * O->eta);
        O->hprime = O->h * O->eta;
        if (O->qprime < O->q) O->nscon = 0;
    }
}

static void prepare_next_step(OracleOde *O, double dsm) {                        /* cvPrepareNextStep */
    long n = O->n;
    if (O->etamax == 1.0) {
        O->qwait = O->qwait > 2 ? O->qwait : 2;
        O->qprime = O->q;
        O->hprime = O->h;
        O->eta = 1.0;
        return;
    }
    O->etaq = 1.0 / (rpower_r(BIAS2 * dsm, 1.0 / O->L) + ADDON);
    if (O->qwait != 0) {
        O->eta = O->etaq;
        O->qprime = O->q;
        set_eta(O);
        return;
    }
    O->qwait = 2;
    O->etaqm1 = 0.0;                                                             /* cvComputeEtaqm1 */
    if (O->q > 1) {
        double ddn = v_wrms(n, O->zn[O->q], O->ewt) * O->tq[1];
        O->etaqm1 = 1.0 / (rpower_r(BIAS1 * ddn, 1.0 / O->q) + ADDON);
    }
    O->etaqp1 = 0.0;                                                             /* cvComputeEtaqp1 */
    if (O->q != O->qmax && O->saved_tq5 != 0.0) {
        double cquot = (O->tq[5] / O->saved_tq5) * rpower_i(O->h / O->tau[2], O->L);
        v_linear_sum(n, -cquot, O->zn[O->qmax], 1.0, O->acor, O->tempv);
        double dup = v_wrms(n, O->tempv, O->ewt) * O->tq[3];
        O->etaqp1 = 1.0 / (rpower_r(BIAS3 * dup, 1.0 / (O->L + 1)) + ADDON);
    }
    double etam = fmax(O->etaqm1, fmax(O->etaq, O->etaqp1));                    /* cvChooseEta */
    if (etam < THRESH) {
        O->eta = 1.0;
        O->qprime = O->q;
    } else if (etam == O->etaq) {
        O->eta = O->etaq;
        O->qprime = O->q;
    } else if (etam == O->etaqm1) {
        O->eta = O->etaqm1;
        O->qprime = O->q - 1;
    } else {
        O->eta = O->etaqp1;
        O->qprime = O->q + 1;
        v_scale(n, 1.0, O->acor, O->zn[O->qmax]);
    }
    set_eta(O);
}

static int cv_step(OracleOde *O) {                                                /* cvStep */
    double saved_t = O->tn, dsm = 0.0;
    int ncf = 0, nef = 0, nflag = FIRST_CALL, kflag, eflag;
    if (O->nst > 0 && O->hprime != O->h) adjust_params(O);
    for (;;) {
        predict(O);
        cv_set(O);
        nflag = nls(O, nflag);
        kflag = handle_nflag(O, &nflag, saved_t, &ncf);
        if (kflag == PREDICT_AGAIN) continue;
        if (kflag != DO_ERROR_TEST) return kflag;
        eflag = do_error_test(O, &nflag, saved_t, &nef, &dsm);
        if (eflag == TRY_AGAIN) continue;
        if (eflag != ODE_SUCCESS) return eflag;
        break;
    }
    complete_step(O);
    prepare_next_step(O, dsm);
    O->etamax = (O->nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
    v_scale(O->n, O->tq[2], O->acor, O->acor);
    return ODE_SUCCESS;
}

int oracle_ode_get_dky(OracleOde *O, double t, int k, double *dky) {             /* CVodeGetDky */
    if (k < 0 || k > O->q) return -24;
    double tfuzz = FUZZ_FACTOR * UROUND * (fabs(O->tn) + fabs(O->hu));
    if (O->hu < 0.0) tfuzz = -tfuzz;
    double tp = O->tn - O->hu - tfuzz, tn1 = O->tn + tfuzz;
    if ((t - tp) * (t - tn1) > 0.0) return ODE_BAD_T;
    double s = (t - O->tn) / O->h, cvals[QMAX + 1];
    double *X[QMAX + 1];
    int nvec = 0;
    for (int j = O->q; j >= k; --j) {
        double c = 1.0;
        for (int i = j; i >= j - k + 1; --i) c *= i;
        for (int i = 0; i < j - k; ++i) c *= s;
        cvals[nvec] = c;
        X[nvec] = O->zn[j];
        nvec++;
    }
    v_lincomb(O->n, nvec, cvals, X, dky);
    if (k == 0) return ODE_SUCCESS;
    v_scale(O->n, rpower_i(O->h, -k), dky, dky);
    return ODE_SUCCESS;
}

/* CVode(mem, tout, yout, &tret, itask): itask 1 = CV_NORMAL, 2 = CV_ONE_STEP */
int oracle_ode_solve(OracleOde *O, double tout, double *yout, double *tret, int itask) {
    long n = O->n;
    int istate = ODE_SUCCESS;
    if (!O->initialized) {                                                       /* first call: nst == 0 */
        O->tretlast = *tret = O->tn;
        if (ewt_set(O, O->zn[0]) != 0) return ODE_ILL_INPUT;
        int rv = O->f(O->tn, O->zn[0], O->zn[1], O->user);
        O->nfe++;
        if (rv != 0) return -9;                                                  /* CV_FIRST_RHSFUNC_ERR */
        if (O->tstopset && (O->tstop - O->tn) * (tout - O->tn) <= 0.0) return ODE_ILL_INPUT;
        O->h = O->hin;
        if ((tout - O->tn) * O->h < 0.0) return ODE_ILL_INPUT;
        double rh = fabs(O->h) * O->hmax_inv;
        if (rh > 1.0) O->h /= rh;
        if (fabs(O->h) < O->hmin) O->h *= O->hmin / fabs(O->h);
        if (O->tstopset && (O->tn + O->h - O->tstop) * O->h > 0.0) O->h = (O->tstop - O->tn) * (1.0 - 4.0 * UROUND);
        O->hscale = O->h;
        O->h0u = O->h;
        O->hprime = O->h;
        v_scale(n, O->h, O->zn[1], O->zn[1]);
        O->initialized = 1;
    } else {
        double troundoff = FUZZ_FACTOR * UROUND * (fabs(O->tn) + fabs(O->h));
        if (itask == 1 && (O->tn - tout) * O->h >= 0.0) {
            O->tretlast = *tret = tout;
            return oracle_ode_get_dky(O, tout, 0, yout) == 0 ? ODE_SUCCESS : ODE_BAD_T;
        }
        if (itask == 2 && fabs(O->tn - O->tretlast) > troundoff) {
            O->tretlast = *tret = O->tn;
            v_scale(n, 1.0, O->zn[0], yout);
            return ODE_SUCCESS;
        }
        if (O->tstopset) {
            if (fabs(O->tn - O->tstop) <= troundoff) {
                if (oracle_ode_get_dky(O, O->tstop, 0, yout) != 0) return ODE_ILL_INPUT;
                O->tretlast = *tret = O->tstop;
                O->tstopset = 0;
                return ODE_TSTOP_RETURN;
            }
            if ((O->tn + O->hprime - O->tstop) * O->h > 0.0) {
                O->hprime = (O->tstop - O->tn) * (1.0 - 4.0 * UROUND);
                O->eta = O->hprime / O->h;
            }
        }
    }
    long nstloc = 0;
    for (;;) {
        O->next_h = O->h;
        O->next_q = O->q;
        if (O->nst > 0 && ewt_set(O, O->zn[0]) != 0) { istate = ODE_ILL_INPUT; *tret = O->tretlast = O->tn; v_scale(n, 1.0, O->zn[0], yout); break; }
        if (O->mxstep > 0 && nstloc >= O->mxstep) {
            istate = ODE_TOO_MUCH_WORK; *tret = O->tretlast = O->tn; v_scale(n, 1.0, O->zn[0], yout); break;
        }
        double nrm = v_wrms(n, O->zn[0], O->ewt);
        O->tolsf = UROUND * nrm;
        if (O->tolsf > 1.0) {
            istate = ODE_TOO_MUCH_ACC; *tret = O->tretlast = O->tn; v_scale(n, 1.0, O->zn[0], yout);
            O->tolsf *= 2.0; break;
        }
        O->tolsf = 1.0;
        if (O->tn + O->h == O->tn) O->nhnil++;
        int kflag = cv_step(O);
        if (kflag != ODE_SUCCESS) {
            istate = kflag; *tret = O->tretlast = O->tn; v_scale(n, 1.0, O->zn[0], yout); break;
        }
        nstloc++;
        if (itask == 1 && (O->tn - tout) * O->h >= 0.0) {
            istate = ODE_SUCCESS;
            O->tretlast = *tret = tout;
            oracle_ode_get_dky(O, tout, 0, yout);
            O->next_q = O->qprime;
            O->next_h = O->hprime;
            break;
        }
        if (O->tstopset) {
            double troundoff = FUZZ_FACTOR * UROUND * (fabs(O->tn) + fabs(O->h));
            if (fabs(O->tn - O->tstop) <= troundoff) {
                oracle_ode_get_dky(O, O->tstop, 0, yout);
                O->tretlast = *tret = O->tstop;
                O->tstopset = 0;
                istate = ODE_TSTOP_RETURN;
                break;
            }
            if ((O->tn + O->hprime - O->tstop) * O->h > 0.0) {
                O->hprime = (O->tstop - O->tn) * (1.0 - 4.0 * UROUND);
                O->eta = O->hprime / O->h;
            }
        }
        if (itask == 2) {
            istate = ODE_SUCCESS;
            O->tretlast = *tret = O->tn;
            v_scale(n, 1.0, O->zn[0], yout);
            O->next_q = O->qprime;
            O->next_h = O->hprime;
            break;
        }
    }
    return istate;
}

/* counters, in ShudOdeStats order (include/shud_ode.h) */
void oracle_ode_get_stats(const OracleOde *O, long *c, double *r) {
    c[0] = O->nst; c[1] = O->nfe; c[2] = O->nfeDQ; c[3] = O->nni; c[4] = O->ncfn; c[5] = O->nnf; c[6] = O->netf;
    c[7] = O->nsetups; c[8] = O->nli; c[9] = O->ncfl; c[10] = O->njtimes; c[11] = O->qu; c[12] = O->q;
    r[0] = O->hu; r[1] = O->h; r[2] = O->tn; r[3] = O->hprime;
}

/* ---------------- RHS adapters ---------------- */
typedef struct OracleModel OracleModel;
int oracle_f(OracleModel *M, double t, const double *Y, double *DY);

/* the SHUD RHS (shud_oracle.c): a reference exit (10/13) is an unrecoverable RHS failure */
static int shud_rhs_adapter(double t, const double *y, double *ydot, void *user) {
    return oracle_f((OracleModel *)user, t, y, ydot) == 0 ? 0 : -1;
}

OracleOde *oracle_ode_create_shud(OracleModel *M, long ny, double t0, const double *y0, double rtol, double atol,
                                  double init_step, double max_step, double min_step, long max_num_steps, int maxl) {
    return oracle_ode_create(ny, shud_rhs_adapter, M, t0, y0, rtol, atol, init_step, max_step, min_step,
                             max_num_steps, maxl, QMAX);
}

/* published test problems (known answers: tests/test_ode.py) */
static int robertson_rhs(double t, const double *y, double *yd, void *user) {   /* Robertson (1966) kinetics */
    (void)t; (void)user;
    double y1 = y[0], y2 = y[1], y3 = y[2];
    const double a = -0.04 * y1 + 1.0e4 * y2 * y3;
    const double c = 3.0e7 * y2 * y2;
    yd[0] = a;
    yd[2] = c;
    yd[1] = -a - c;
    return 0;
}

static int decay_rhs(double t, const double *y, double *yd, void *user) {        /* y_i' = -lambda_i y_i */
    (void)t;
    const double *lam = (const double *)user;
    yd[0] = -lam[0] * y[0];
    yd[1] = -lam[1] * y[1];
    yd[2] = -lam[2] * y[2];
    return 0;
}

static const double DECAY_LAMBDA[3] = {1.0, 10.0, 1000.0};
static const double DECAYN_LAMBDA[7] = {0.01, 0.1, 1.0, 10.0, 100.0, 1000.0, 10000.0};

static int decayn_rhs(double t, const double *y, double *yd, void *user) {      /* y_i' = -lambda_{i mod 7} y_i */
    (void)t;
    long n = *(const long *)user;
    for (long i = 0; i < n; ++i) yd[i] = -DECAYN_LAMBDA[i % 7] * y[i];
    return 0;
}
static long decayn_n = 0;

/* problem 1 = Robertson (n = 3), 2 = three-rate decay (n = 3), 3 = n-component seven-rate decay */
OracleOde *oracle_ode_create_test(int problem, long n, double t0, const double *y0, double rtol, double atol,
                                  double init_step, double max_step, double min_step, long max_num_steps, int maxl) {
    if (problem == 3) {
        decayn_n = n;
        return oracle_ode_create(n, decayn_rhs, (void *)&decayn_n, t0, y0, rtol, atol, init_step, max_step, min_step,
                                 max_num_steps, maxl, QMAX);
    }
    if (problem == 1)
        return oracle_ode_create(3, robertson_rhs, NULL, t0, y0, rtol, atol, init_step, max_step, min_step,
                                 max_num_steps, maxl, QMAX);
    if (problem == 2)
        return oracle_ode_create(3, decay_rhs, (void *)DECAY_LAMBDA, t0, y0, rtol, atol, init_step, max_step,
                                 min_step, max_num_steps, maxl, QMAX);
    return NULL;
}
