// shud_ode_dev.h — internal: device vector kernels of the integrator (shud_ode_kernels.hip), called by the
// host controller (shud_ode.cpp).  Not part of the C-ABI.
//
// Every kernel is one streaming pass over NY-long fp64 vectors in HBM, fusing the N_Vector operations that
// CVODE issues back to back (cvode.c / sunlinsol_spgmr.c / nvector_serial.c) so each pass reads every operand
// once.  Per element the arithmetic is exactly the serial N_Vector kernel's (same operations, same order, no
// FMA contraction: -ffp-contract=off).  Reductions (dot products, WRMS norms, min) are deterministic: one entry
// per thread on a full grid of kRedThreads-thread blocks writes per-block partials (waves in order), and a
// one-block finalize kernel (kFinThreads threads, kFinAcc interleaved accumulators each) sums them in a fixed order
// into a device scalar slot `ds[slot]` that later kernels read directly, and into its host-mapped twin
// `hds[slot]` (with the RHS error word) that the host reads after a stream synchronize — no copy per fetch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace shud {
namespace ode {

constexpr int kThreads = 256;       // element-wise passes
constexpr int kRedThreads = 1024;   // reduction passes: one entry per thread, ceil(n / 1024) blocks
constexpr int kFinThreads = 1024;   // finalize: thread t sums partials t + (kFinAcc*j + k)*kFinThreads into acc k
constexpr int kFinAcc = 4;
constexpr int kMaxAcc = 4;
constexpr int kMaxL = 32;     // SPGMR Krylov dimension bound (maxl)
constexpr int kQMax = 5;      // BDF

// device scalar slots
enum Slot : int {
    S_EWTMIN = 0,   // min(rtol|y| + atol)
    S_NRM,          // sum (zn0*ewt)^2
    S_RES,          // sum (delta*ewt)^2 of the Newton residual (bnorm and SPGMR beta)
    S_SIG,          // sum ((V/ewt)*ewt)^2 of the current Krylov vector (DQ perturbation)
    S_WN,           // sum w*w after Gram-Schmidt (new_vk_norm^2)
    S_DEL,          // sum (delta*ewt)^2 of the Newton update
    S_YCOR,         // sum (ycor*ewt)^2
    S_ETAQM1,       // sum (zn[q]*ewt)^2
    S_ETAQP1,       // sum (((-cquot) zn[qmax] + acor)*ewt)^2
    S_SCRATCH,      // results nobody reads (the reorthogonalisation's w -= np V[i] pass)
    S_W = 15,       // sum w*w before Gram-Schmidt (vk_norm^2); atimes writes [S_W, S_H0]
    S_H0 = 16,      // S_H0 + i: Gram-Schmidt coefficient h[i][l] (first pass), i <= kMaxL
    S_R0 = S_H0 + kMaxL + 1,   // S_R0 + i: reorthogonalisation products
    S_COUNT = S_R0 + kMaxL + 1
};

struct Red {           // partial-sum scratch of one reduction launch and where its result goes
    double *part;      // [kMaxAcc][nblk]
    int nblk;          // blocks of the producing grid, ceil(n / kRedThreads) (fixed per n); also the stride of part
    double *ds;        // device scalar slots [S_COUNT]
    double *hds;       // host-mapped twin [S_COUNT + 2]; hds[S_COUNT] carries the RHS error word, hds[S_COUNT + 1]
                       // the sequence number of the last finalize done (uint64 bits, stored last, release)
    const uint32_t *err;   // RHS error flags (DevErr::flags) or null
    int slot0;         // first slot of this reduction's results
    uint64_t seq;      // this finalize's sequence number (host counter)
};

struct Coefs {         // small host-computed coefficient arrays passed by value
    double c[kMaxL + 1];
};

// A deferred cvCompleteStep on zn[j0..q] (zn[j] = l[j]*acor + zn[j]) and its zn[copy_to] = acor, and a deferred
// cvRescale after it (zn[j] *= r[j], j = 1..q): applied in registers by the first pass that reads zn (the next
// cvPredict, a CVodeGetDky, cvComputeEtaqm1's norm), or materialized before an order change / a read of zn[0]
// through the API.  j0 = 0: zn[0] pending too (the ewt pass computes it without storing it).  acor == nullptr:
// nothing pending.
struct Pend {
    const double *acor;
    Coefs l, r;
    int q, copy_to, resc, j0;
};

// ---- launchers (hipStream_t s); a reduction kernel leaves per-block partials, finalize(r, nacc, minmask) writes
// its nacc results to slots [r.slot0, r.slot0 + nacc) ----
void finalize(const Red &r, int nacc, unsigned minmask, hipStream_t s);

void ewt_set(int64_t n, const double *zn0, double *ewt, double rtol, double atol, const Red &r, hipStream_t s);
// cvPredict; with y/ycor != null also ycor = 0 and y = zn[0] + 0.0 (the following cvNls start)
void predict(int64_t n, double *zn, int q, double *y, double *ycor, hipStream_t s);
// predict with a pending complete (+ rescale) applied first: pd.q == q, pd.acor != null
void predict_pend(int64_t n, double *zn, int q, double *y, double *ycor, const Pend &pd, hipStream_t s);
void restore(int64_t n, double *zn, int q, hipStream_t s);
void rescale(int64_t n, double *zn, int q, const Coefs &c, hipStream_t s);
void vsum(int64_t n, const double *x, const double *y, double *z, hipStream_t s);
void vsum_zero(int64_t n, const double *x, double *ycor, double *z, hipStream_t s);   // ycor = 0; z = x + 0
void copy(int64_t n, const double *x, double *z, hipStream_t s);
void scale_to(int64_t n, double c, const double *x, double *z, hipStream_t s);
void zero(int64_t n, double *z, hipStream_t s);
// zn[j] = coef[j] * zn[src] + zn[j], j in [jlo, jhi]
void axpy_multi(int64_t n, double *zn, int src, const Coefs &coef, int jlo, int jhi, hipStream_t s);
// Newton residual: delta = -((rl1*zn1 + ycor) + ngamma*ftemp); r: sum (delta*ewt)^2
void residual(int64_t n, const double *zn1, const double *ycor, const double *ftemp, double rl1, double ngamma,
              const double *ewt, double *delta, const Red &r, hipStream_t s);
// V0 = c * (ewt*delta); r: sum ((V0/ewt)*ewt)^2
void krylov_v0(int64_t n, const double *delta, const double *ewt, double c, double *V0, const Red &r, hipStream_t s);
// work = sig*(V/ewt) + y, sig = 1/sqrt(ds[S_SIG]/n)
void dq_work(int64_t n, const double *V, const double *ewt, const double *y, double *work, const double *ds,
             hipStream_t s);
// w (in: f(work)) = ewt * ((-gamma)*(siginv*(w - fy)) + V/ewt); r: [sum w*w, sum V0*w]
void atimes(int64_t n, double *w, const double *fy, const double *V, const double *ewt, const double *V0,
            double ngamma, const double *ds, const Red &r, hipStream_t s);
// w = w + (-ds[hslot])*Vprev (if Vprev); r: sum Vnext*w (Vnext) or sum w*w
void mgs(int64_t n, double *w, const double *Vprev, const double *ds, int hslot, const double *Vnext, const Red &r,
         hipStream_t s);
// w = c*w; r: sum ((w/ewt)*ewt)^2
void normalize(int64_t n, double *w, double c, const double *ewt, const Red &r, hipStream_t s);
// Newton update: delta = (sum_k yg[k] V_k)/ewt (krydim > 0), or delta = dsrc (krydim 0; NULL = 0);
// ycor += delta; r: [sum (delta*ewt)^2, sum (ycor*ewt)^2]
void newton_update(int64_t n, const double *V, int64_t vstride, int krydim, const Coefs &yg, const double *dsrc,
                   const double *ewt, double *ycor, bool ycor_zero, const Red &r, hipStream_t s);
// 1: predict() leaves ycor unwritten: the caller then passes ycor_zero until the first
// newton_update after a predict
int lazy_ycor();
// zn[j] = l[j]*acor + zn[j], j = jlo..q; if copy_to >= 0: zn[copy_to] = acor
void complete_step(int64_t n, double *zn, const double *acor, const Coefs &l, int jlo, int q, int copy_to,
                   hipStream_t s);
// complete_step (columns jst..q stored; zn[0]'s value is formed either way), then ewt_set's arithmetic on the new
// zn[0] into ewt_next; r: [min(rtol|y| + atol), sum (y*w)^2]
void complete_step_ewt(int64_t n, double *zn, const double *acor, const Coefs &l, int q, int copy_to, int jst,
                       double rtol, double atol, double *ewt_next, const Red &r, hipStream_t s);
// r: [sum (zn_q*ewt)^2 (zn_q != NULL), sum (((-cquot)*zn_qmax + acor)*ewt)^2 (zn_qmax != NULL)]; pend_q: zn_q's
// completion is pending, zn_q = lq*acor + zn_q on the fly
void eta_norms(int64_t n, const double *zn_q, const double *zn_qmax, const double *acor, double ncquot,
               const double *ewt, int pend_q, double lq, const Red &r, hipStream_t s);
// dky = lincomb(c, zn[js]) (N_VLinearCombination), then dky *= rscale if rscale != 0; zn[j] with a pending
// completion (pd.acor, 1 <= j <= pd.q) taken on the fly
void dky(int64_t n, const double *zn, int64_t stride, const int *js, const Coefs &c, int nvec, double rscale,
         double *out, const Pend &pd, hipStream_t s);
int grid_blocks(int64_t n);

}  // namespace ode
}  // namespace shud
