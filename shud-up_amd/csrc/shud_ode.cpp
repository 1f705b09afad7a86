// shud_ode.cpp — device-resident time integrator (include/shud_ode.h).
//
// Restates SUNDIALS CVODE 6.0.0 (the reference's pinned solver, configure:17) as SetCVODE configures it
// (src/Equations/cvode_config.cpp:149-197): BDF orders 1..5 in Nordsieck form, Newton iteration, SPGMR (maxl 5,
// no preconditioner, modified Gram-Schmidt, no restarts) with difference-quotient J*v, scalar tolerances,
// min/max/initial step, max steps, stop time.  The routine structure follows cvode.c (cvStep, cvNls,
// cvDoErrorTest, cvCompleteStep, cvPrepareNextStep, ...) and sunlinsol_spgmr.c; oracle/shud_oracle_ode.c is the
// sequential CPU restatement the tests compare against.
//
// MI355X layout: the N_Vectors are NY-long fp64 arrays in HBM that never leave the device — the Nordsieck array
// zn[0..qmax] and the Krylov basis V[0..maxl] are contiguous slabs, the RHS is evaluated on device pointers on
// the handle's stream, and CVODE's chains of N_Vector calls are fused into single streaming passes
// (shud_ode_kernels.hip).  Scalar control (step size, order, error test, Givens QR of the Hessenberg matrix)
// runs on the host; reductions land in device scalar slots that later kernels read directly (the DQ
// perturbation sigma, the Gram-Schmidt coefficients), and the host fetches them only where CVODE branches on
// them: once per step (ewt/tolsf check), per Newton iteration (residual norm, convergence test) and per Krylov
// iteration (Hessenberg column).  Not restated: cvHin (SHUD always sets INIT_SOLVER_STEP > 0), root finding,
// stability-limit detection (off in SetCVODE), the DQ perturbation retry after a recoverable RHS failure
// (SHUD's f never fails recoverably: it exits), and the final N_VScale(tq[2], acor) of cvStep (acor is dead
// after it in this configuration).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "shud_handle.h"
#include "shud_ode.h"
#include "shud_ode_dev.h"

// A fetch polls the last finalize's completion word in host-mapped memory instead of blocking in
// hipStreamSynchronize (A/B 4.39 vs 4.43 ms per step, profiles/r04/ode_spin/).  The round 3-5 A/B switches of this
// file (synchronize-only fetches, eager cvCompleteStep, stored zn[0]) were removed in round 6; commit a4b4e96 holds them.

using namespace shud::ode;

namespace {
// cvode.c / cvode_ls.c constants
constexpr double UROUND = DBL_EPSILON, FUZZ_FACTOR = 100.0;
constexpr double ETAMX1 = 10000.0, ETAMX2 = 10.0, ETAMX3 = 10.0, ETAMXF = 0.2, ETAMIN = 0.1, ETACF = 0.25;
constexpr double ADDON = 0.000001, BIAS1 = 6.0, BIAS2 = 6.0, BIAS3 = 10.0, ONEPSM = 1.000001, THRESH = 1.5;
constexpr int SMALL_NST = 10, MXNCF = 10, MXNEF = 7, MXNEF1 = 3, SMALL_NEF = 2, LONG_WAIT = 10, MSBP = 20;
constexpr double DGMAX = 0.3, CRDOWN = 0.3, RDIV = 2.0, NLSCOEF = 0.1;
constexpr int NLS_MAXCOR = 3;
// cvCompleteStep: its pass forms zn[0]'s new value for the next error weights without storing it; zn[0..q] and the
// acor copy are deferred into the next predict (ode::Pend; 4.48 vs 4.58 ms per step eager, profiles/r04/ode_lazy_*)
constexpr double CVLS_EPLIN = 0.05, CVLS_DGMAX = 0.2;
constexpr int CVLS_MSBJ = 51;
enum { FIRST_CALL = 0, PREV_CONV_FAIL = 1, PREV_ERR_FAIL = 2 };
enum { CV_NO_FAILURES = 0, CV_FAIL_BAD_J = 1, CV_FAIL_OTHER = 2 };
constexpr int NLS_CONV_RECVR = 902;
constexpr int DO_ERROR_TEST = 2, PREDICT_AGAIN = 3, TRY_AGAIN = 5;
enum { LS_SUCCESS = 0, LS_RES_REDUCED = 1, LS_CONV_FAIL = 2, LS_QR_FAIL = -6 };

double rpower_r(double b, double e) { return b <= 0.0 ? 0.0 : std::pow(b, e); }   // SUNRpowerR
double rpower_i(double b, int e) {                                              // SUNRpowerI
    double p = 1.0;
    for (int i = 1; i <= std::abs(e); ++i) p *= b;
    return e < 0 ? 1.0 / p : p;
}
void givens(double t1, double t2, double *c, double *s) {                       // SUNQRfact rotation
    if (t2 == 0.0) { *c = 1.0; *s = 0.0; }
    else if (std::fabs(t2) >= std::fabs(t1)) { double t3 = t1 / t2; *s = -1.0 / std::sqrt(1.0 + t3 * t3); *c = -(*s) * t3; }
    else { double t3 = t2 / t1; *c = 1.0 / std::sqrt(1.0 + t3 * t3); *s = -(*c) * t3; }
}
}  // namespace

struct shud_ode {
    int64_t n = 0;
    ShudOdeRhsFn f = nullptr;
    void *user = nullptr;
    shud_rhs *rh = nullptr;                 // SHUD RHS handle (physics error word), or null
    hipStream_t s = nullptr;
    int device = 0;
    double rtol = 0, atol = 0, hin = 0, hmin = 0, hmax_inv = 0;
    int64_t mxstep = 500;
    int maxl = 5, qmax = 5;
    // device vectors
    double *base = nullptr, *zn = nullptr, *ewt = nullptr, *y = nullptr, *acor = nullptr, *ftemp = nullptr;
    double *tempv = nullptr, *delta = nullptr, *work = nullptr, *V = nullptr;
    // the next step's error weights, computed by the fused complete+ewt pass; swapped in by ewt_and_norm
    double *ewt_alt = nullptr;
    bool ewt_pending = false;
    int64_t ewt_fin_sync = 0;           // n_sync when the fused pass's finalize was enqueued
    double *d_part = nullptr, *d_ds = nullptr, *h_ds = nullptr;
    Red red{};
    Red rs(int slot) const { Red r = red; r.slot0 = slot; return r; }   // this reduction's result slots
    uint64_t fin_seq = 0;   // finalizes enqueued so far (each stores its number into h_ds[S_COUNT + 1] last)
    void fin(int slot, int nacc, unsigned minmask) {
        Red r = rs(slot);
        r.seq = ++fin_seq;
        finalize(r, nacc, minmask, s);
    }
    // SPGMR host state
    double Hes[kMaxL + 1][kMaxL]{}, gv[2 * kMaxL]{}, yg[kMaxL + 1]{};
    // integrator scalars (cvode_impl.h names)
    double tn = 0, h = 0, hprime = 0, next_h = 0, eta = 1, etamax = ETAMX1, hscale = 0, h0u = 0, hu = 0;
    double tau[kQMax + 2]{}, tq[6]{}, l[kQMax + 1]{};
    double rl1 = 0, gamma = 0, gammap = 0, gamrat = 1, crate = 1, delp = 0, acnrm = 0, saved_tq5 = 0;
    double tstop = 0, tretlast = 0, tolsf = 1, etaq = 0, etaqm1 = 0, etaqp1 = 0, nrmfac = 1;
    bool acor_zero = false;
    // acor_lazy: acor is logically all +0.0 but was never stored (the last predict skipped the fill,
    // ode::lazy_ycor()); cleared by the first newton_update, which writes all of acor
    bool acor_lazy = false;
    int tstopset = 0, q = 1, qprime = 1, next_q = 1, qwait = 2, L = 2, qu = 0, indx_acor = 5;
    int convfail = 0, jcur = 0, jbad = 0, curiter = 0, initialized = 0;
    int64_t nst = 0, nscon = 0, nstlp = 0, nfe = 0, nfeDQ = 0, nni = 0, nnf = 0, ncfn = 0, netf = 0, nsetups = 0;
    int64_t nli = 0, ncfl = 0, njtimes = 0, nhnil = 0, n_sync = 0;
    bool rhs_failed = false, hip_failed = false;

    double *Z(int j) const { return zn + (int64_t)j * n; }
    double *VV(int j) const { return V + (int64_t)j * n; }
    double wrms_of(int slot) const { return std::sqrt(h_ds[slot] / (double)n); }

    // ---- device helpers ----
    int rhs(double t, const double *yy, double *yd) {
        int rv = f(t, yy, yd, user);
        if (rv != 0) hip_failed = true;
        return rv;
    }
    // host view of the scalar slots (+ the RHS physics error word): every finalize writes them into host-mapped
    // memory (shud_ode_kernels.hip k_finalize), so a fetch is one stream synchronize
    bool fetch() {
        hipError_t e = hipSuccess;
        // poll the last enqueued finalize's completion word (host-mapped, coherent) instead of blocking in the
        // runtime; after ~2 s, or with no finalize yet, synchronize (which also reports a device fault)
        bool done = false;
        if (fin_seq > 0) {
            const uint64_t *w = reinterpret_cast<const uint64_t *>(h_ds + S_COUNT + 1);
            const auto t0 = std::chrono::steady_clock::now();
            for (uint32_t k = 1;; k++) {
                if (__atomic_load_n(w, __ATOMIC_ACQUIRE) >= fin_seq) { done = true; break; }
                if ((k & 4095u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
                __builtin_ia32_pause();
            }
        }
        if (!done) e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipGetLastError();
        n_sync++;
        if (e != hipSuccess) {
            shud_fail(SHUD_ERR_HIP, "integrator: %s", hipGetErrorString(e));
            hip_failed = true;
            return false;
        }
        if (rh) {
            uint32_t fl;
            memcpy(&fl, h_ds + S_COUNT, sizeof(fl));
            const uint32_t fatal = SHUD_EF_NAN_QELE | SHUD_EF_EFFKH | SHUD_EF_ET_NEG | SHUD_EF_ET_NAN;
            if (fl & fatal) {
                rhs_failed = true;
                return false;
            }
        }
        return true;
    }
    int fail_code() const { return hip_failed && !rhs_failed ? SHUD_ODE_DEVICE_ERR : SHUD_ODE_RHSFUNC_FAIL; }

    // ---- cvSetBDF / cvSetTqBDF / cvSet ----
    void set_tq_bdf(double hsum, double alpha0, double alpha0_hat, double xi_inv, double xistar_inv) {
        double A1 = 1.0 - alpha0_hat + alpha0;
        double A2 = 1.0 + q * A1;
        tq[2] = std::fabs(A1 / (alpha0 * A2));
        tq[5] = std::fabs(A2 * xistar_inv / (l[q] * xi_inv));
        if (qwait == 1) {
            if (q > 1) {
                double C = xistar_inv / l[q];
                double A3 = alpha0 + 1.0 / q;
                double A4 = alpha0_hat + xi_inv;
                double Cpinv = (1.0 - A4 + A3) / A3;
                tq[1] = std::fabs(C * Cpinv);
            } else {
                tq[1] = 1.0;
            }
            hsum += tau[q];
            xi_inv = h / hsum;
            double A5 = alpha0 - (1.0 / (q + 1));
            double A6 = alpha0_hat - xi_inv;
            double Cppinv = (1.0 - A6 + A5) / A2;
            tq[3] = std::fabs(Cppinv / (xi_inv * (q + 2) * A5));
        }
        tq[4] = NLSCOEF / tq[2];
    }
    void set_bdf() {
        double alpha0, alpha0_hat, xi_inv, xistar_inv, hsum;
        l[0] = l[1] = xi_inv = xistar_inv = 1.0;
        for (int i = 2; i <= q; ++i) l[i] = 0.0;
        alpha0 = alpha0_hat = -1.0;
        hsum = h;
        if (q > 1) {
            for (int j = 2; j < q; ++j) {
                hsum += tau[j - 1];
                xi_inv = h / hsum;
                alpha0 -= 1.0 / j;
                for (int i = j; i >= 1; --i) l[i] += l[i - 1] * xi_inv;
            }
            alpha0 -= 1.0 / q;
            xistar_inv = -l[1] - alpha0;
            hsum += tau[q - 1];
            xi_inv = h / hsum;
            alpha0_hat = -l[1] - xi_inv;
            for (int i = q; i >= 1; --i) l[i] += l[i - 1] * xistar_inv;
        }
        set_tq_bdf(hsum, alpha0, alpha0_hat, xi_inv, xistar_inv);
    }
    void cv_set() {
        set_bdf();
        rl1 = 1.0 / l[1];
        gamma = h * rl1;
        if (nst == 0) gammap = gamma;
        gamrat = (nst > 0) ? gamma / gammap : 1.0;
    }
    // ---- cvPredict / cvRestore / cvRescale ----
    // y_pred: the last predict also wrote y = zn[0] + 0 and set acor = 0 (k_pascal; with lazy_ycor the zeros are
    // not stored, acor_lazy), which the cvNls start that always follows it would otherwise do in a separate pass
    // (k_vsum_zero)
    bool y_pred = false;
    // the last step's cvCompleteStep on zn[0..q] (+ zn[qmax] = acor) and a following cvRescale, deferred into the
    // next pass that reads zn (ode::Pend; complete_step_ewt forms zn[0]'s new value for the error weights only)
    ode::Pend pend{};
    void materialize() {                                             // apply a deferred completion now
        if (!pend.acor) return;
        complete_step(n, zn, pend.acor, pend.l, pend.j0, pend.q, pend.copy_to, s);
        if (pend.resc) ode::rescale(n, zn, pend.q, pend.r, s);
        pend = ode::Pend{};
    }
    void materialize0() {                                            // zn[0] only (an API read of y(tcur))
        if (!pend.acor || pend.j0 != 0) return;
        complete_step(n, zn, pend.acor, pend.l, 0, 0, -1, s);
        pend.j0 = 1;
    }
    void predict() {
        tn += h;
        if (tstopset && (tn - tstop) * h > 0.0) tn = tstop;
        if (pend.acor && pend.q == q) ode::predict_pend(n, zn, q, y, acor, pend, s);
        else {
            materialize();
            ode::predict(n, zn, q, y, acor, s);
        }
        pend = ode::Pend{};
        y_pred = true;
        acor_lazy = ode::lazy_ycor() != 0;
    }
    void restore(double saved_t) {
        tn = saved_t;
        materialize();                // (never pending here: a restore follows a predict)
        ode::restore(n, zn, q, s);
        y_pred = false;               // (acor_lazy kept: a failed attempt's acor is still logically +0.0)
    }
    void rescale() {
        Coefs c{};
        double x = eta;
        for (int j = 1; j <= q; ++j) { c.c[j] = x; x = eta * x; }
        if (pend.acor && !pend.resc && pend.q == q) {                 // after a deferred completion: fused too
            pend.r = c;
            pend.resc = 1;
        } else {
            materialize();
            ode::rescale(n, zn, q, c, s);
        }
        h = hscale * eta;
        next_h = h;
        hscale = h;
        nscon = 0;
    }
    // ---- cvAdjustOrder (BDF) ----
    void increase_bdf() {
        double alpha0, alpha1, prod, xi, xiold, hsum, A1;
        for (int i = 0; i <= qmax; ++i) l[i] = 0.0;
        l[2] = alpha1 = prod = xiold = 1.0;
        alpha0 = -1.0;
        hsum = hscale;
        if (q > 1) {
            for (int j = 1; j < q; ++j) {
                hsum += tau[j + 1];
                xi = hsum / hscale;
                prod *= xi;
                alpha0 -= 1.0 / (j + 1);
                alpha1 += 1.0 / xi;
                for (int i = j + 2; i >= 2; --i) l[i] = l[i] * xiold + l[i - 1];
                xiold = xi;
            }
        }
        A1 = (-alpha0 - alpha1) / prod;
        scale_to(n, A1, Z(indx_acor), Z(L), s);
        Coefs c{};
        for (int j = 2; j <= q; ++j) c.c[j] = l[j];
        axpy_multi(n, zn, L, c, 2, q, s);
    }
    void decrease_bdf() {
        double hsum, xi;
        for (int i = 0; i <= qmax; ++i) l[i] = 0.0;
        l[2] = 1.0;
        hsum = 0.0;
        for (int j = 1; j <= q - 2; ++j) {
            hsum += tau[j];
            xi = hsum / hscale;
            for (int i = j + 2; i >= 2; --i) l[i] = l[i] * xi + l[i - 1];
        }
        Coefs c{};
        for (int j = 2; j < q; ++j) c.c[j] = -l[j];
        axpy_multi(n, zn, q, c, 2, q - 1, s);
    }
    void adjust_order(int dq) {
        if (q == 2 && dq != 1) return;
        if (dq == 1) increase_bdf();
        else if (dq == -1) decrease_bdf();
    }
    void adjust_params() {
        if (qprime != q) {
            materialize();                                           // cvAdjustOrder reads zn[2..q] and zn[qmax]
            adjust_order(qprime - q);
            q = qprime;
            L = q + 1;
            qwait = L;
        }
        rescale();
    }

    bool take_lazy() {
        const bool z = acor_lazy;
        acor_lazy = false;
        return z;
    }
    // ---- cvLsSolve + SPGMR (zero guess, s1 = s2 = ewt, no preconditioner, 0 restarts) ----
    // returns 0 ok (ycor updated, del/ycor norms in h_ds), 1 recoverable failure, < 0 unrecoverable
    int ls_solve_and_update() {
        const double deltar = CVLS_EPLIN * tq[4];
        const double bnorm = wrms_of(S_RES);
        Coefs none{};
        if (bnorm <= deltar) {                                       // cvLsSolve: small rhs
            newton_update(n, nullptr, n, 0, none, curiter > 0 ? nullptr : delta, ewt, acor, take_lazy(), rs(S_DEL), s);
            fin(S_DEL, 2, 0u);
            return fetch() ? 0 : -1;
        }
        const double delta_tol = deltar * nrmfac;
        const double r_norm = std::sqrt(h_ds[S_RES]), beta = r_norm;
        if (r_norm <= delta_tol) {                                   // SPGMR: x = x0 = 0
            newton_update(n, nullptr, n, 0, none, nullptr, ewt, acor, take_lazy(), rs(S_DEL), s);
            fin(S_DEL, 2, 0u);
            return fetch() ? 0 : -1;
        }
        double rho = beta, rotation_product = 1.0;
        int krydim = 0, converged = 0, nl = 0;
        for (int i = 0; i <= maxl; ++i)
            for (int j = 0; j < maxl; ++j) Hes[i][j] = 0.0;
        krylov_v0(n, delta, ewt, 1.0 / r_norm, VV(0), rs(S_SIG), s);
        fin(S_SIG, 1, 0u);
        int rv = LS_CONV_FAIL;
        for (int ll = 0; ll < maxl; ++ll) {
            nl++;
            krydim = ll + 1;
            // cvLsATimes(V[ll]/s2) -> DQ J*v (one RHS call) -> z = v - gamma*Jv -> V[ll+1] = s1*z
            dq_work(n, VV(ll), ewt, y, work, d_ds, s);
            if (rhs(tn, work, VV(ll + 1)) != 0) return -1;
            nfeDQ++;
            njtimes++;
            atimes(n, VV(ll + 1), ftemp, VV(ll), ewt, VV(0), -gamma, d_ds, rs(S_W), s);                    // [S_W, S_H0] = [||w||^2, V[0].w]
            fin(S_W, 2, 0u);
            // SUNModifiedGS: w -= h[i-1] V[i-1] fused with h[i] = V[i].w; last pass gives the new ||w||^2
            int hs = S_H0;                                           // slot of h[i-1]
            for (int i = 1; i <= ll; ++i) {
                mgs(n, VV(ll + 1), VV(i - 1), d_ds, hs, VV(i), rs(S_H0 + i), s);
                fin(S_H0 + i, 1, 0u);
                hs = S_H0 + i;
            }
            mgs(n, VV(ll + 1), VV(ll), d_ds, hs, nullptr, rs(S_WN), s);
            fin(S_WN, 1, 0u);
            if (!fetch()) return -1;
            const double vk_norm = std::sqrt(h_ds[S_W]);
            double new_vk_norm = std::sqrt(h_ds[S_WN]);
            for (int i = 0; i <= ll; ++i) Hes[i][ll] = h_ds[S_H0 + i];
            const double temp = 1000.0 * vk_norm;
            if ((temp + new_vk_norm) == temp) {                      // reorthogonalise (rare)
                double new_norm_2 = 0.0;
                for (int i = 0; i <= ll; ++i) {
                    mgs(n, VV(ll + 1), nullptr, d_ds, 0, VV(i), rs(S_R0 + i), s);
                    fin(S_R0 + i, 1, 0u);
                    if (!fetch()) return -1;
                    const double np = h_ds[S_R0 + i];
                    if (np == 0.0) continue;
                    Hes[i][ll] += np;
                    mgs(n, VV(ll + 1), VV(i), d_ds, S_R0 + i, nullptr, rs(S_SCRATCH), s);   // w -= np V[i]
                    new_norm_2 += np * np;
                }
                if (new_norm_2 != 0.0) {
                    new_norm_2 = new_vk_norm * new_vk_norm - new_norm_2;
                    new_vk_norm = (new_norm_2 > 0.0) ? std::sqrt(new_norm_2) : 0.0;
                }
            }
            Hes[ll + 1][ll] = new_vk_norm;
            // SUNQRfact(krydim, Hes, givens, ll)
            {
                int code = 0;
                if (ll == 0) {
                    double c, sn, t1 = Hes[0][0], t2 = Hes[1][0];
                    givens(t1, t2, &c, &sn);
                    gv[0] = c; gv[1] = sn;
                    if ((Hes[0][0] = c * t1 - sn * t2) == 0.0) code = 1;
                } else {
                    const int nm1 = krydim - 1;
                    for (int k = 0; k < nm1; ++k) {
                        double t1 = Hes[k][nm1], t2 = Hes[k + 1][nm1], c = gv[2 * k], sn = gv[2 * k + 1];
                        Hes[k][nm1] = c * t1 - sn * t2;
                        Hes[k + 1][nm1] = sn * t1 + c * t2;
                    }
                    double c, sn, t1 = Hes[nm1][nm1], t2 = Hes[krydim][nm1];
                    givens(t1, t2, &c, &sn);
                    gv[2 * nm1] = c; gv[2 * nm1 + 1] = sn;
                    if ((Hes[nm1][nm1] = c * t1 - sn * t2) == 0.0) code = krydim;
                }
                if (code != 0) { rv = LS_QR_FAIL; break; }
            }
            rotation_product *= gv[2 * ll + 1];
            rho = std::fabs(rotation_product * r_norm);
            if (rho <= delta_tol) { converged = 1; break; }
            normalize(n, VV(ll + 1), 1.0 / Hes[ll + 1][ll], ewt, rs(S_SIG), s);
            fin(S_SIG, 1, 0u);
        }
        nli += nl;
        if (rv == LS_QR_FAIL) { ncfl++; return -1; }
        // SUNQRsol
        yg[0] = r_norm;
        for (int i = 1; i <= krydim; ++i) yg[i] = 0.0;
        for (int k = 0; k < krydim; ++k) {
            double c = gv[2 * k], sn = gv[2 * k + 1], t1 = yg[k], t2 = yg[k + 1];
            yg[k] = c * t1 - sn * t2;
            yg[k + 1] = sn * t1 + c * t2;
        }
        for (int k = krydim - 1; k >= 0; --k) {
            if (Hes[k][k] == 0.0) { ncfl++; return -1; }
            yg[k] /= Hes[k][k];
            for (int i = 0; i < k; ++i) yg[i] -= yg[k] * Hes[i][k];
        }
        if (converged) rv = LS_SUCCESS;
        else if (rho < beta) rv = LS_RES_REDUCED;
        else rv = LS_CONV_FAIL;
        if (rv != LS_SUCCESS) ncfl++;
        if (rv == LS_CONV_FAIL) return 1;
        if (rv == LS_RES_REDUCED && curiter != 0) return 1;
        Coefs c{};
        for (int k = 0; k < krydim; ++k) c.c[k] = yg[k];
        newton_update(n, V, n, krydim, c, nullptr, ewt, acor, take_lazy(), rs(S_DEL), s);
        fin(S_DEL, 2, 0u);
        return fetch() ? 0 : -1;
    }

    // ---- cvNls with the Newton SUNNonlinearSolver ----
    int nls_residual() {                                             // cvNlsResidual (+ -delta, + bnorm)
        // acor_zero: cvNls has just set ycor = 0; the zero fill is fused into the y = zn[0] + ycor pass and
        // the residual reads no ycor (identical operands, one fewer pass over HBM)
        const bool az = acor_zero;
        acor_zero = false;
        if (az && !y_pred) { vsum_zero(n, Z(0), acor, y, s); acor_lazy = false; }
        else if (!az) vsum(n, Z(0), acor, y, s);
        y_pred = false;
        if (rhs(tn, y, ftemp) != 0) return SHUD_ODE_RHSFUNC_FAIL;
        nfe++;
        residual(n, Z(1), az ? nullptr : acor, ftemp, rl1, -gamma, ewt, delta, rs(S_RES), s);
        fin(S_RES, 1, 0u);
        if (!fetch()) return SHUD_ODE_RHSFUNC_FAIL;
        return 0;
    }
    void nls_lsetup(int jbad_in) {                                   // cvNlsLSetup + cvLsSetup (matrix-free)
        if (jbad_in) convfail = CV_FAIL_BAD_J;
        const double dgamma = std::fabs((gamma / gammap) - 1.0);
        jbad = (nst == 0) || (nst >= 0 + CVLS_MSBJ) || ((convfail == CV_FAIL_BAD_J) && (dgamma < CVLS_DGMAX)) ||
               (convfail == CV_FAIL_OTHER);
        if (jbad) jcur = 1;
        nsetups++;
        gamrat = 1.0;
        gammap = gamma;
        crate = 1.0;
        nstlp = nst;
    }
    int nls(int nflag) {
        convfail = (nflag == FIRST_CALL || nflag == PREV_ERR_FAIL) ? CV_NO_FAILURES : CV_FAIL_OTHER;
        int callSetup = (nflag == PREV_CONV_FAIL) || (nflag == PREV_ERR_FAIL) || (nst == 0) ||
                        (nst >= nstlp + MSBP) || (std::fabs(gamrat - 1.0) > DGMAX);
        acor_zero = true;                              // N_VConst(0, ycor), fused (nls_residual)
        int jb = 0, rv = 0;
        for (;;) {
            rv = nls_residual();
            if (rv != 0) break;
            if (callSetup) nls_lsetup(jb);
            curiter = 0;
            for (;;) {
                nni++;
                const int lr = ls_solve_and_update();
                if (lr != 0) { rv = lr < 0 ? (rhs_failed || hip_failed ? SHUD_ODE_RHSFUNC_FAIL : SHUD_ODE_LSOLVE_FAIL) : NLS_CONV_RECVR; break; }
                // cvNlsConvTest
                const double del = wrms_of(S_DEL);
                if (curiter > 0) crate = std::fmax(CRDOWN * crate, del / delp);
                const double dcon = del * std::fmin(1.0, crate) / tq[4];
                if (dcon <= 1.0) {
                    acnrm = (curiter == 0) ? del : wrms_of(S_YCOR);
                    jcur = 0;
                    return 0;
                }
                if (curiter >= 1 && del > RDIV * delp) { rv = NLS_CONV_RECVR; break; }
                delp = del;
                curiter++;
                if (curiter >= NLS_MAXCOR) { rv = NLS_CONV_RECVR; break; }
                rv = nls_residual();
                if (rv != 0) break;
            }
            if (rv == NLS_CONV_RECVR && !jcur) {
                nnf++;
                callSetup = 1;
                jb = 1;
                acor_zero = true;                              // N_VConst(0, ycor), fused (nls_residual)
                continue;
            }
            break;
        }
        nnf++;
        return rv;
    }
    int handle_nflag(int *nflagPtr, double saved_t, int *ncfPtr) {   // cvHandleNFlag
        int nflag = *nflagPtr;
        if (nflag == 0) return DO_ERROR_TEST;
        ncfn++;
        restore(saved_t);
        if (nflag < 0) return nflag;
        (*ncfPtr)++;
        etamax = 1.0;
        if (std::fabs(h) <= hmin * ONEPSM || *ncfPtr == MXNCF) return SHUD_ODE_CONV_FAILURE;
        eta = std::fmax(ETACF, hmin / std::fabs(h));
        *nflagPtr = PREV_CONV_FAIL;
        rescale();
        return PREDICT_AGAIN;
    }
    int do_error_test(int *nflagPtr, double saved_t, int *nefPtr, double *dsmPtr) {   // cvDoErrorTest
        const double dsm = acnrm * tq[2];
        *dsmPtr = dsm;
        if (dsm <= 1.0) return SHUD_ODE_SUCCESS;
        (*nefPtr)++;
        netf++;
        *nflagPtr = PREV_ERR_FAIL;
        restore(saved_t);
        if (std::fabs(h) <= hmin * ONEPSM || *nefPtr == MXNEF) return SHUD_ODE_ERR_FAILURE;
        etamax = 1.0;
        if (*nefPtr <= MXNEF1) {
            eta = 1.0 / (rpower_r(BIAS2 * dsm, 1.0 / L) + ADDON);
            eta = std::fmax(ETAMIN, std::fmax(eta, hmin / std::fabs(h)));
            if (*nefPtr >= SMALL_NEF) eta = std::fmin(eta, ETAMXF);
            rescale();
            return TRY_AGAIN;
        }
        if (q > 1) {
            eta = std::fmax(ETAMIN, hmin / std::fabs(h));
            adjust_order(-1);
            L = q;
            q--;
            qwait = L;
            rescale();
            return TRY_AGAIN;
        }
        eta = std::fmax(ETAMIN, hmin / std::fabs(h));
        h *= eta;
        next_h = h;
        hscale = h;
        qwait = LONG_WAIT;
        nscon = 0;
        if (rhs(tn, Z(0), tempv) != 0) return SHUD_ODE_RHSFUNC_FAIL;
        nfe++;
        scale_to(n, h, tempv, Z(1), s);
        return TRY_AGAIN;
    }
    void set_eta() {                                                  // cvSetEta
        if (eta < THRESH) {
            eta = 1.0;
            hprime = h;
        } else {
            eta = std::fmin(eta, etamax);
            eta /= std::fmax(1.0, std::fabs(h) * hmax_inv * eta);
            hprime = h * eta;
            if (qprime < q) nscon = 0;
        }
    }
    // cvCompleteStep + cvPrepareNextStep
    int complete_and_prepare(double dsm) {
        nst++;
        nscon++;
        hu = h;
        qu = q;
        for (int i = q; i >= 2; --i) tau[i] = tau[i - 1];
        if (q == 1 && nst > 1) tau[2] = tau[1];
        tau[1] = h;
        Coefs lc{};
        for (int j = 0; j <= q; ++j) lc.c[j] = l[j];
        qwait--;
        int copy_to = -1;
        if (qwait == 1 && q != qmax) {
            copy_to = qmax;
            saved_tq5 = tq[5];
            indx_acor = qmax;
        }
        // cvCompleteStep + the next loop iteration's cvEwtSet / N_VWrmsNorm(zn[0]) in one pass (ewt_and_norm);
        // that pass completes nothing in memory: zn[0..q] and the acor copy ride in the next predict (ode::Pend)
        complete_step_ewt(n, zn, acor, lc, 0, -1, 1, rtol, atol, ewt_alt, rs(S_EWTMIN), s);
        pend = ode::Pend{};
        pend.acor = acor;
        pend.l = lc;
        pend.q = q;
        pend.copy_to = copy_to;
        pend.j0 = 0;
        fin(S_EWTMIN, 2, 1u);
        ewt_pending = true;
        ewt_fin_sync = n_sync;
        // cvPrepareNextStep
        if (etamax == 1.0) {
            qwait = qwait > 2 ? qwait : 2;
            qprime = q;
            hprime = h;
            eta = 1.0;
            return 0;
        }
        etaq = 1.0 / (rpower_r(BIAS2 * dsm, 1.0 / L) + ADDON);
        if (qwait != 0) {
            eta = etaq;
            qprime = q;
            set_eta();
            return 0;
        }
        qwait = 2;
        etaqm1 = 0.0;
        etaqp1 = 0.0;
        const bool qm1 = q > 1, qp1 = (q != qmax && saved_tq5 != 0.0);
        double cquot = 0.0;
        if (qp1) cquot = (tq[5] / saved_tq5) * rpower_i(h / tau[2], L);
        if (qm1 || qp1) {
            const bool pq = qm1 && pend.acor && q >= 1 && q <= pend.q;
            eta_norms(n, qm1 ? Z(q) : nullptr, qp1 ? Z(qmax) : nullptr, acor, -cquot, ewt, pq ? 1 : 0,
                      pq ? pend.l.c[q] : 0.0, rs(S_ETAQM1), s);
            fin(S_ETAQM1, 2, 0u);
            if (!fetch()) return -1;
        }
        if (qm1) {
            const double ddn = wrms_of(S_ETAQM1) * tq[1];
            etaqm1 = 1.0 / (rpower_r(BIAS1 * ddn, 1.0 / q) + ADDON);
        }
        if (qp1) {
            const double dup = wrms_of(S_ETAQP1) * tq[3];
            etaqp1 = 1.0 / (rpower_r(BIAS3 * dup, 1.0 / (L + 1)) + ADDON);
        }
        const double etam = std::fmax(etaqm1, std::fmax(etaq, etaqp1));   // cvChooseEta
        if (etam < THRESH) {
            eta = 1.0;
            qprime = q;
        } else if (etam == etaq) {
            eta = etaq;
            qprime = q;
        } else if (etam == etaqm1) {
            eta = etaqm1;
            qprime = q - 1;
        } else {
            eta = etaqp1;
            qprime = q + 1;
            copy(n, acor, Z(qmax), s);     // (a pending completion has copy_to < 0 here: qwait was 0, not 1)
        }
        set_eta();
        return 0;
    }
    int cv_step() {                                                    // cvStep
        const double saved_t = tn;
        double dsm = 0.0;
        int ncf = 0, nef = 0, nflag = FIRST_CALL, kflag, eflag;
        if (nst > 0 && hprime != h) adjust_params();
        for (;;) {
            predict();
            cv_set();
            nflag = nls(nflag);
            kflag = handle_nflag(&nflag, saved_t, &ncf);
            if (kflag == PREDICT_AGAIN) continue;
            if (kflag != DO_ERROR_TEST) return kflag;
            eflag = do_error_test(&nflag, saved_t, &nef, &dsm);
            if (eflag == TRY_AGAIN) continue;
            if (eflag != SHUD_ODE_SUCCESS) return eflag;
            break;
        }
        if (complete_and_prepare(dsm) != 0) return fail_code();
        etamax = (nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
        return SHUD_ODE_SUCCESS;
    }
    int get_dky(double t, int k, double *out) {                       // CVodeGetDky
        if (k < 0 || k > q) return SHUD_ODE_BAD_K;
        double tfuzz = FUZZ_FACTOR * UROUND * (std::fabs(tn) + std::fabs(hu));
        if (hu < 0.0) tfuzz = -tfuzz;
        const double tp = tn - hu - tfuzz, tn1 = tn + tfuzz;
        if ((t - tp) * (t - tn1) > 0.0) return SHUD_ODE_BAD_T;
        if (!out) return SHUD_ODE_SUCCESS;
        const double sv = (t - tn) / h;
        Coefs c{};
        int js[kQMax + 1];
        int nvec = 0;
        for (int j = q; j >= k; --j) {
            double cc = 1.0;
            for (int i = j; i >= j - k + 1; --i) cc *= i;
            for (int i = 0; i < j - k; ++i) cc *= sv;
            c.c[nvec] = cc;
            js[nvec] = j;
            nvec++;
        }
        ode::dky(n, zn, n, js, c, nvec, k == 0 ? 0.0 : rpower_i(h, -k), out, pend, s);
        return SHUD_ODE_SUCCESS;
    }
    int ewt_and_norm() {                                              // cvEwtSet + N_VWrmsNorm(zn[0])
        if (ewt_pending) {              // computed by the last complete_step_ewt on this zn[0]
            std::swap(ewt, ewt_alt);
            ewt_pending = false;
            if (n_sync == ewt_fin_sync && !fetch()) return -1;          // no synchronize since its finalize
            return h_ds[S_EWTMIN] <= 0.0 ? 1 : 0;
        }
        materialize0();
        ewt_set(n, Z(0), ewt, rtol, atol, rs(S_EWTMIN), s);
        fin(S_EWTMIN, 2, 1u);
        if (!fetch()) return -1;
        return h_ds[S_EWTMIN] <= 0.0 ? 1 : 0;
    }
    void out_y(double *yout) {
        if (!yout) return;
        materialize0();
        copy(n, Z(0), yout, s);
    }

    int solve(double tout, double *yout, double *tret, int itask) {   // CVode
        int istate = SHUD_ODE_SUCCESS;
        if (!initialized) {
            tretlast = *tret = tn;
            const int e = ewt_and_norm();
            if (e < 0) return fail_code();
            if (e > 0) return SHUD_ODE_ILL_INPUT;
            if (rhs(tn, Z(0), Z(1)) != 0) return SHUD_ODE_FIRST_RHSFUNC_ERR;
            nfe++;
            if (tstopset && (tstop - tn) * (tout - tn) <= 0.0) return SHUD_ODE_ILL_INPUT;
            h = hin;
            if ((tout - tn) * h < 0.0) return SHUD_ODE_ILL_INPUT;
            const double rh_ = std::fabs(h) * hmax_inv;
            if (rh_ > 1.0) h /= rh_;
            if (std::fabs(h) < hmin) h *= hmin / std::fabs(h);
            if (tstopset && (tn + h - tstop) * h > 0.0) h = (tstop - tn) * (1.0 - 4.0 * UROUND);
            hscale = h;
            h0u = h;
            hprime = h;
            scale_to(n, h, Z(1), Z(1), s);
            initialized = 1;
        } else {
            const double troundoff = FUZZ_FACTOR * UROUND * (std::fabs(tn) + std::fabs(h));
            if (itask == SHUD_ODE_NORMAL && (tn - tout) * h >= 0.0) {
                tretlast = *tret = tout;
                return get_dky(tout, 0, yout) == 0 ? SHUD_ODE_SUCCESS : SHUD_ODE_BAD_T;
            }
            if (itask == SHUD_ODE_ONE_STEP && std::fabs(tn - tretlast) > troundoff) {
                tretlast = *tret = tn;
                out_y(yout);
                return SHUD_ODE_SUCCESS;
            }
            if (tstopset) {
                if (std::fabs(tn - tstop) <= troundoff) {
                    if (get_dky(tstop, 0, yout) != 0) return SHUD_ODE_ILL_INPUT;
                    tretlast = *tret = tstop;
                    tstopset = 0;
                    return SHUD_ODE_TSTOP_RETURN;
                }
                if ((tn + hprime - tstop) * h > 0.0) {
                    hprime = (tstop - tn) * (1.0 - 4.0 * UROUND);
                    eta = hprime / h;
                }
            }
        }
        int64_t nstloc = 0;
        for (;;) {
            next_h = h;
            next_q = q;
            if (nst > 0) {
                const int e = ewt_and_norm();
                if (e < 0) return fail_code();
                if (e > 0) { istate = SHUD_ODE_ILL_INPUT; *tret = tretlast = tn; out_y(yout); break; }
            }
            if (mxstep > 0 && nstloc >= mxstep) {
                istate = SHUD_ODE_TOO_MUCH_WORK; *tret = tretlast = tn; out_y(yout); break;
            }
            const double nrm = wrms_of(S_NRM);
            tolsf = UROUND * nrm;
            if (tolsf > 1.0) {
                istate = SHUD_ODE_TOO_MUCH_ACC; *tret = tretlast = tn; out_y(yout);
                tolsf *= 2.0;
                break;
            }
            tolsf = 1.0;
            if (tn + h == tn) nhnil++;
            const int kflag = cv_step();
            if (rhs_failed || hip_failed) return fail_code();
            if (kflag != SHUD_ODE_SUCCESS) {
                istate = kflag; *tret = tretlast = tn; out_y(yout); break;
            }
            nstloc++;
            if (itask == SHUD_ODE_NORMAL && (tn - tout) * h >= 0.0) {
                istate = SHUD_ODE_SUCCESS;
                tretlast = *tret = tout;
                get_dky(tout, 0, yout);
                next_q = qprime;
                next_h = hprime;
                break;
            }
            if (tstopset) {
                const double troundoff = FUZZ_FACTOR * UROUND * (std::fabs(tn) + std::fabs(h));
                if (std::fabs(tn - tstop) <= troundoff) {
                    get_dky(tstop, 0, yout);
                    tretlast = *tret = tstop;
                    tstopset = 0;
                    istate = SHUD_ODE_TSTOP_RETURN;
                    break;
                }
                if ((tn + hprime - tstop) * h > 0.0) {
                    hprime = (tstop - tn) * (1.0 - 4.0 * UROUND);
                    eta = hprime / h;
                }
            }
            if (itask == SHUD_ODE_ONE_STEP) {
                istate = SHUD_ODE_SUCCESS;
                tretlast = *tret = tn;
                out_y(yout);
                next_q = qprime;
                next_h = hprime;
                break;
            }
        }
        return istate;
    }
};

// ---------------------------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------------------------
static int shud_rhs_ode_fn(double t, const double *d_y, double *d_ydot, void *user) {
    return shud_rhs_eval((shud_rhs_t)user, t, d_y, d_ydot, SHUD_WHERE_DEVICE) == SHUD_OK ? 0 : -1;
}

static int ode_alloc(shud_ode *o, double t0, const double *y0, int where, const ShudOdeOptions *opt) {
    if (!opt || !(opt->init_step > 0.0) || opt->reltol < 0.0 || opt->abstol < 0.0)
        return shud_fail(SHUD_ERR_ARG, "shud_ode: init_step must be > 0 and tolerances >= 0");
    o->rtol = opt->reltol;
    o->atol = opt->abstol;
    o->hin = opt->init_step;
    o->hmin = opt->min_step > 0.0 ? opt->min_step : 0.0;
    o->hmax_inv = opt->max_step > 0.0 ? 1.0 / opt->max_step : 0.0;
    o->mxstep = opt->max_num_steps > 0 ? opt->max_num_steps : 500;
    o->maxl = opt->maxl > 0 ? opt->maxl : 5;
    if (o->maxl > kMaxL) return shud_fail(SHUD_ERR_ARG, "shud_ode: maxl > %d", kMaxL);
    o->qmax = (opt->max_order > 0 && opt->max_order <= kQMax) ? opt->max_order : kQMax;
    o->indx_acor = o->qmax;
    o->tn = t0;
    o->nrmfac = std::sqrt((double)o->n);
    const int64_t n = o->n;
    const int64_t nvec = (o->qmax + 1) + 8 + (o->maxl + 1);
    HIP_TRY(hipMalloc(&o->base, nvec * n * sizeof(double)));
    double *p = o->base;
    o->zn = p; p += (int64_t)(o->qmax + 1) * n;
    o->ewt = p; p += n;
    o->y = p; p += n;
    o->acor = p; p += n;
    o->ftemp = p; p += n;
    o->tempv = p; p += n;
    o->delta = p; p += n;
    o->work = p; p += n;
    o->ewt_alt = p; p += n;
    o->V = p;
    HIP_TRY(hipMemsetAsync(o->base, 0, nvec * n * sizeof(double), o->s));
    HIP_TRY(hipMalloc(&o->d_part, (size_t)kMaxAcc * grid_blocks(n) * sizeof(double)));
    HIP_TRY(hipMalloc(&o->d_ds, S_COUNT * sizeof(double)));
    HIP_TRY(hipMemsetAsync(o->d_ds, 0, S_COUNT * sizeof(double), o->s));
    HIP_TRY(hipHostMalloc(&o->h_ds, (S_COUNT + 2) * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent));
    memset(o->h_ds, 0, (S_COUNT + 2) * sizeof(double));
    o->red.part = o->d_part;
    o->red.nblk = grid_blocks(n);
    HIP_TRY(hipHostGetDevicePointer((void **)&o->red.hds, o->h_ds, 0));
    o->red.ds = o->d_ds;
    o->red.err = o->rh ? &o->rh->d_err->flags : nullptr;
    HIP_TRY(hipMemcpyAsync(o->zn, y0, n * sizeof(double),
                           where == SHUD_WHERE_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, o->s));
    HIP_TRY(hipStreamSynchronize(o->s));
    return SHUD_OK;
}

static void ode_free(shud_ode *o) {
    if (!o) return;
    if (o->base) (void)hipFree(o->base);
    if (o->d_part) (void)hipFree(o->d_part);
    if (o->d_ds) (void)hipFree(o->d_ds);
    if (o->h_ds) (void)hipHostFree(o->h_ds);
    delete o;
}

extern "C" int shud_ode_create(shud_rhs_t rhs, double t0, const double *y0, int where, const ShudOdeOptions *opt,
                               shud_ode_t *out) {
    if (!rhs || !y0 || !out) return shud_fail(SHUD_ERR_ARG, "null argument");
    if (rhs->partitioned) return shud_fail(SHUD_ERR_UNSUPPORTED, "shud_ode: partitioned handles are not supported");
    *out = nullptr;
    HIP_TRY(hipSetDevice(rhs->device));
    shud_ode *o = new shud_ode();
    o->n = 3 * (int64_t)rhs->n_own + rhs->n_own_riv + rhs->NL;
    o->f = shud_rhs_ode_fn;
    o->user = rhs;
    o->rh = rhs;
    o->s = rhs->stream;
    o->device = rhs->device;
    int rc = ode_alloc(o, t0, y0, where, opt);
    if (rc != SHUD_OK) { ode_free(o); return rc; }
    *out = o;
    return SHUD_OK;
}

extern "C" int shud_ode_create_fn(int64_t n, ShudOdeRhsFn f, void *user, void *stream, double t0, const double *y0,
                                  int where, const ShudOdeOptions *opt, shud_ode_t *out) {
    if (n <= 0 || !f || !y0 || !out) return shud_fail(SHUD_ERR_ARG, "null argument");
    *out = nullptr;
    shud_ode *o = new shud_ode();
    o->n = n;
    o->f = f;
    o->user = user;
    o->s = (hipStream_t)stream;
    HIP_TRY(hipGetDevice(&o->device));
    int rc = ode_alloc(o, t0, y0, where, opt);
    if (rc != SHUD_OK) { ode_free(o); return rc; }
    *out = o;
    return SHUD_OK;
}

extern "C" int shud_ode_set_stop_time(shud_ode_t o, double tstop) {
    if (!o) return SHUD_ODE_MEM_NULL;
    o->tstop = tstop;
    o->tstopset = 1;
    return SHUD_ODE_SUCCESS;
}

extern "C" int shud_ode_solve(shud_ode_t o, double tout, double *y_out, int where, double *tret, int itask) {
    if (!o || !tret) return SHUD_ODE_MEM_NULL;
    if (itask != SHUD_ODE_NORMAL && itask != SHUD_ODE_ONE_STEP) return SHUD_ODE_ILL_INPUT;
    if (hipSetDevice(o->device) != hipSuccess) return SHUD_ODE_DEVICE_ERR;
    double *dst = (y_out && where == SHUD_WHERE_HOST) ? o->tempv : y_out;   // tempv is free between calls
    int rc = o->solve(tout, dst, tret, itask);
    if (y_out && where == SHUD_WHERE_HOST && rc >= 0) {
        if (hipMemcpyAsync(y_out, o->tempv, o->n * sizeof(double), hipMemcpyDeviceToHost, o->s) != hipSuccess)
            return SHUD_ODE_DEVICE_ERR;
    }
    if (hipStreamSynchronize(o->s) != hipSuccess) return SHUD_ODE_DEVICE_ERR;
    return rc;
}

extern "C" int shud_ode_get_dky(shud_ode_t o, double t, int k, double *dky, int where) {
    if (!o || !dky) return SHUD_ODE_MEM_NULL;
    double *dst = where == SHUD_WHERE_HOST ? o->tempv : dky;
    int rc = o->get_dky(t, k, dst);
    if (rc != SHUD_ODE_SUCCESS) return rc;
    if (where == SHUD_WHERE_HOST &&
        hipMemcpyAsync(dky, o->tempv, o->n * sizeof(double), hipMemcpyDeviceToHost, o->s) != hipSuccess)
        return SHUD_ODE_DEVICE_ERR;
    if (hipStreamSynchronize(o->s) != hipSuccess) return SHUD_ODE_DEVICE_ERR;
    return SHUD_ODE_SUCCESS;
}

extern "C" int shud_ode_get_stats(shud_ode_t o, ShudOdeStats *st) {
    if (!o || !st) return SHUD_ODE_MEM_NULL;
    st->nst = o->nst; st->nfe = o->nfe; st->nfe_ls = o->nfeDQ; st->nni = o->nni; st->ncfn = o->ncfn;
    st->nnf = o->nnf; st->netf = o->netf; st->nsetups = o->nsetups; st->nli = o->nli; st->ncfl = o->ncfl;
    st->njtimes = o->njtimes; st->qlast = o->qu; st->qcur = o->q;
    st->hlast = o->hu; st->hcur = o->h; st->tcur = o->tn; st->hnext = o->hprime;
    st->n_sync = o->n_sync;
    return SHUD_ODE_SUCCESS;
}

extern "C" const double *shud_ode_state_device(shud_ode_t o) {
    if (!o) return nullptr;
    if (hipSetDevice(o->device) != hipSuccess) return nullptr;
    o->materialize0();                 // zn[0]'s completion may still be pending (ode::Pend)
    if (hipGetLastError() != hipSuccess) return nullptr;
    // the completion (and anything else the last solve left queued) runs on the integrator's non-blocking stream:
    // finish it here, so a consumer on another stream or the default stream never reads a stale y(tcur)
    if (hipStreamSynchronize(o->s) != hipSuccess) return nullptr;
    return o->zn;
}

extern "C" int shud_ode_destroy(shud_ode_t o) {
    if (!o) return SHUD_ODE_MEM_NULL;
    (void)hipSetDevice(o->device);
    (void)hipStreamSynchronize(o->s);
    ode_free(o);
    return SHUD_ODE_SUCCESS;
}
