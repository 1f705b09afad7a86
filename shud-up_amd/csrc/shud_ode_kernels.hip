// shud_ode_kernels.hip — device vector kernels of the integrator (see shud_ode_dev.h).
//
// Streaming passes over fp64 vectors of NY entries, one entry per thread on a full grid (element-wise passes in
// 256-thread blocks, reductions in kRedThreads-thread blocks whose partials a one-block finalize sums in a fixed
// order, so every reduction is deterministic), with non-temporal loads and stores.  Per element each kernel applies exactly the serial N_Vector operations CVODE
// issues (nvector_serial.c: N_VLinearSum special cases, N_VScale, N_VProd/N_VDiv, N_VLinearCombination,
// N_VScaleAddMulti) in the same order; the host controller (shud_ode.cpp) cites the CVODE routine each call
// replaces.  The bound is HBM bandwidth: bytes per entry are listed at each kernel.
#include "shud_ode_dev.h"

#include <cmath>
#include <cstdlib>

namespace shud {
namespace ode {

int grid_blocks(int64_t n) {
    const int64_t b = (n + kRedThreads - 1) / kRedThreads;
    return (int)(b < 1 ? 1 : b);
}

// element-wise grid: one entry per thread (full occupancy; measured 15-20% faster than the 2048-block
// grid-stride loop at syn-10M: dq_work 214 -> 179 us, pascal<3> 395 -> 323 us)
static int ew_blocks(int64_t n) {
    const int64_t b = (n + kThreads - 1) / kThreads;
    return (int)(b < 1 ? 1 : b);
}

// single-use streams: non-temporal loads and stores (global_load/store ... nt).  The vectors are NY-long (250 MB
// at syn-10M), far beyond L2; nt loads+stores measured 7 % faster on the five-operand pass
// (profiles/r03/ode/ode_red_bench.log)
template <class T>
__device__ __forceinline__ T ldn(const T *p) { return __builtin_nontemporal_load(p); }
template <class T>
__device__ __forceinline__ void stn(T *p, T v) { __builtin_nontemporal_store(v, p); }

// One entry per thread: use(i, load(i)) for i = block * BS + thread when i < n (BS = blockDim.x).  Reductions run
// on the full one-shot grid (ceil(n / kRedThreads) blocks) rather than a grid-stride loop: the grid-stride form
// kept one load batch per wave in flight and ran at 4.7 TB/s against 5.7 TB/s one-shot (ode_red_bench).
template <class T, class Load, class Use>
__device__ __forceinline__ void one(int64_t n, Load load, Use use) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) use(i, load(i));
}
struct D1 { double a; };
struct D2 { double a, b; };
struct D3 { double a, b, c; };
struct D4 { double a, b, c, d; };
template <int N>
struct DN { double v[N]; };

// reduction kernel on the one-shot reduction grid
#define LAUNCH_RED(K, r, s, ...) K<1><<<(r).nblk, kRedThreads, 0, (s)>>>(__VA_ARGS__, (r))
// element-wise kernel
#define LAUNCH_EW(K, n, s, ...) K<1><<<ew_blocks(n), kThreads, 0, (s)>>>(n, __VA_ARGS__)

__device__ inline double comb(double a, double b, bool mn) { return mn ? fmin(a, b) : a + b; }

// the NW = threads/64 wave results of a block (sm[0..NW), one per wave) combined by wave 0: lane l < NW holds
// sm[l], an xor butterfly over offsets NW/2 .. 1 (lanes >= NW never mix in), lane 0 keeps the result.  A fixed
// tree order (oracle: waves_tree) in 4 shuffles — round 2's serial sum on thread 0 (16 dependent LDS reads per
// accumulator) held every 1024-thread block's slot for ~1.5 us and slowed the light passes (k_ewt 105 -> 173 us)
template <int NW>
__device__ inline double waves_tree(const double *sm, bool mn, int lane) {
    static_assert(NW <= 64 && (NW & (NW - 1)) == 0, "power-of-two wave count");
    double x = lane < NW ? sm[lane] : (mn ? INFINITY : 0.0);
#pragma unroll
    for (int off = NW / 2; off >= 1; off >>= 1) x = comb(x, __shfl_xor(x, off, 64), mn);
    return x;
}

// block partials: wave64 butterfly per wave, then the wave results by waves_tree (deterministic)
template <int NACC>
__device__ inline void block_partial(double (&v)[NACC], unsigned minmask, const Red &r) {
    constexpr int NW = kRedThreads / 64;
    __shared__ double sm[NACC][NW];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < NACC; ++a) {
        const bool mn = (minmask >> a) & 1u;
        double x = v[a];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) x = comb(x, __shfl_xor(x, off, 64), mn);
        if (lane == 0) sm[a][wid] = x;
    }
    __syncthreads();
    if (wid == 0) {
#pragma unroll
        for (int a = 0; a < NACC; ++a) {
            const bool mn = (minmask >> a) & 1u;
            const double s = waves_tree<NW>(sm[a], mn, lane);
            if (lane == 0) r.part[(int64_t)a * r.nblk + blockIdx.x] = s;
        }
    }
}

// the nblk partials of one reduction in a fixed order into the device slot ds[slot0 + a] (read by later kernels)
// and its host-mapped twin hds[slot0 + a]; hds[S_COUNT] receives the RHS error word, so a host fetch is one stream
// synchronize.  Order (restated by oracle/shud_oracle_ode.c device_order_sum): thread t keeps kFinAcc
// accumulators, acc[k] over partials t + (kFinAcc*j + k)*kFinThreads for j = 0, 1, ... (the kFinAcc loads of one j
// in flight together); x = (acc0 + acc1) + (acc2 + acc3); wave64 butterfly; the kFinThreads/64 wave results by
// waves_tree.  (Finalizing in the producer's last-arriving block instead measured slower: tickets on one counter.)
__global__ void __launch_bounds__(kFinThreads) k_finalize(Red r, int nacc, unsigned minmask) {
    constexpr int NW = kFinThreads / 64;
    __shared__ double sm[NW];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int a = 0; a < nacc; ++a) {
        const bool mn = (minmask >> a) & 1u;
        const double id = mn ? INFINITY : 0.0;
        const double *pp = r.part + (int64_t)a * r.nblk;
        double acc[kFinAcc];
#pragma unroll
        for (int k = 0; k < kFinAcc; ++k) acc[k] = id;
        for (int b0 = threadIdx.x; b0 < r.nblk; b0 += kFinAcc * kFinThreads) {
            double v[kFinAcc];
#pragma unroll
            for (int k = 0; k < kFinAcc; ++k) {
                const int b = b0 + k * kFinThreads;
                v[k] = b < r.nblk ? pp[b] : id;
            }
#pragma unroll
            for (int k = 0; k < kFinAcc; ++k) acc[k] = comb(acc[k], v[k], mn);
        }
        double x = comb(comb(acc[0], acc[1], mn), comb(acc[2], acc[3], mn), mn);
        for (int off = 32; off >= 1; off >>= 1) x = comb(x, __shfl_xor(x, off, 64), mn);
        if (lane == 0) sm[wid] = x;
        __syncthreads();
        if (wid == 0) {
            const double s = waves_tree<NW>(sm, mn, lane);
            if (lane == 0) {
                r.ds[r.slot0 + a] = s;
                r.hds[r.slot0 + a] = s;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && r.err) {
        const uint32_t fl = *(const volatile uint32_t *)r.err;
        double w = 0.0;
        __builtin_memcpy(&w, &fl, sizeof(fl));
        r.hds[S_COUNT] = w;
    }
    // completion word for a host that polls instead of synchronizing (shud_ode.cpp fetch): thread 0 made every
    // hds store of this kernel; the release store at system scope orders them before it
    if (threadIdx.x == 0)
        __hip_atomic_store(reinterpret_cast<uint64_t *>(r.hds + S_COUNT + 1), r.seq, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

void finalize(const Red &r, int nacc, unsigned minmask, hipStream_t s) {
    k_finalize<<<1, kFinThreads, 0, s>>>(r, nacc, minmask);
}

// cvEwtSetSS + the N_VWrmsNorm(zn[0], ewt) of CVode's "too much accuracy" check.  24 B/entry.
template <int U>
__global__ void __launch_bounds__(kRedThreads) k_ewt(int64_t n, const double *__restrict__ zn0, double *__restrict__ ewt,
                                                  double rtol, double atol, Red r) {
    double v[2] = {INFINITY, 0.0};
    one<D1>(n, [&](int64_t i) { return D1{ldn(zn0 + i)}; }, [&](int64_t i, const D1 &o) {
        const double y = o.a;
        const double t = rtol * fabs(y) + atol;
        const double w = 1.0 / t;
        stn(ewt + i, w);
        v[0] = fmin(v[0], t);
        const double p = y * w;
        v[1] += p * p;
    });
    block_partial<2>(v, 1u, r);
}
void ewt_set(int64_t n, const double *zn0, double *ewt, double rtol, double atol, const Red &r, hipStream_t s) {
    LAUNCH_RED(k_ewt, r, s, n, zn0, ewt, rtol, atol);
}

// cvPredict / cvRestore: Pascal-triangle update of the Nordsieck array in registers.  2*8*(q+1) B/entry.
// cvPredict with y != null also performs the next cvNls start (every predict is followed by one): ycor = 0
// (N_VConst) and y = zn[0] + ycor (N_VLinearSum) on the new zn[0] — the same add as k_vsum_zero, so -0.0
// becomes +0.0 exactly as there — saving that pass's re-read of zn[0] (+8 B/entry here, -24 B/entry there).
// The ycor = 0 fill is not stored at all — the controller marks ycor "all +0.0"
// and its only readers before the first Newton update (k_residual, k_newton_update) take the zeros as operands
// instead of loading them (identical values; -8 B/entry here and in that k_newton_update)
// PEND (cvPredict after a deferred cvCompleteStep, Pend): zn[j] = l[j]*acor + zn[j] and zn[j] *= r[j] (j = 1..Q) in
// registers first — k_complete's and k_rescale's arithmetic — then the Pascal update; zn[Q] is stored too, and
// zn[copy_to] = acor.  Saves the completion's own pass over zn[1..Q] (+16 B/entry here, -16*Q B/entry there).
// ycor is not __restrict__: predict_pend passes acor as both ycor and pd.acor (it is never stored here)
template <int Q, bool FWD, bool PEND, int U>
__global__ void __launch_bounds__(kThreads) k_pascal(int64_t n, double *__restrict__ zn, double *__restrict__ y,
                                                     double *ycor, Pend pd) {
    using T = DN<Q + 2>;                  // [0..Q] zn, [Q + 1] acor (PEND)
    one<T>(n, [&](int64_t i) {
        T a;
#pragma unroll
        for (int j = 0; j <= Q; ++j) a.v[j] = ldn(zn + (int64_t)j * n + i);
        a.v[Q + 1] = PEND ? ldn(pd.acor + i) : 0.0;
        return a;
    }, [&](int64_t i, T a) {
        if (PEND) {
            if (pd.j0 == 0) a.v[0] = pd.l.c[0] * a.v[Q + 1] + a.v[0];
#pragma unroll
            for (int j = 1; j <= Q; ++j) a.v[j] = pd.l.c[j] * a.v[Q + 1] + a.v[j];
            if (pd.resc) {
#pragma unroll
                for (int j = 1; j <= Q; ++j) a.v[j] = a.v[j] * pd.r.c[j];
            }
        }
#pragma unroll
        for (int k = 1; k <= Q; ++k)
#pragma unroll
            for (int j = Q; j >= k; --j) a.v[j - 1] = FWD ? a.v[j - 1] + a.v[j] : a.v[j - 1] - a.v[j];
#pragma unroll
        for (int j = 0; j < Q; ++j) stn(zn + (int64_t)j * n + i, a.v[j]);
        if (PEND) {
            stn(zn + (int64_t)Q * n + i, a.v[Q]);
            if (pd.copy_to >= 0) stn(zn + (int64_t)pd.copy_to * n + i, a.v[Q + 1]);
        }
        if (FWD && y) {
            const double zero = 0.0;
            stn(y + i, a.v[0] + zero);
        }
    });
}
template <int Q, bool FWD, bool PEND>
static void pascal_q(int64_t n, double *zn, double *y, double *ycor, const Pend &pd, hipStream_t s) {
    k_pascal<Q, FWD, PEND, 1><<<ew_blocks(n), kThreads, 0, s>>>(n, zn, y, ycor, pd);
}
template <bool FWD, bool PEND>
static void pascal(int64_t n, double *zn, int q, double *y, double *ycor, const Pend &pd, hipStream_t s) {
    switch (q) {
    case 1: pascal_q<1, FWD, PEND>(n, zn, y, ycor, pd, s); break;
    case 2: pascal_q<2, FWD, PEND>(n, zn, y, ycor, pd, s); break;
    case 3: pascal_q<3, FWD, PEND>(n, zn, y, ycor, pd, s); break;
    case 4: pascal_q<4, FWD, PEND>(n, zn, y, ycor, pd, s); break;
    default: pascal_q<5, FWD, PEND>(n, zn, y, ycor, pd, s); break;
    }
}
int lazy_ycor() { return 1; }
void predict(int64_t n, double *zn, int q, double *y, double *ycor, hipStream_t s) {
    pascal<true, false>(n, zn, q, y, ycor, Pend{}, s);
}
void predict_pend(int64_t n, double *zn, int q, double *y, double *ycor, const Pend &pd, hipStream_t s) {
    pascal<true, true>(n, zn, q, y, ycor, pd, s);
}
void restore(int64_t n, double *zn, int q, hipStream_t s) { pascal<false, false>(n, zn, q, nullptr, nullptr, Pend{}, s); }

// cvRescale: zn[j] *= eta^j (N_VScaleVectorArray).  16*q B/entry.
template <int U>
__global__ void __launch_bounds__(kThreads) k_rescale(int64_t n, double *__restrict__ zn, int q, Coefs c) {
    using T = DN<kQMax>;
    one<T>(n, [&](int64_t i) {
        T a;
#pragma unroll
        for (int j = 1; j <= kQMax; ++j)
            if (j <= q) a.v[j - 1] = ldn(zn + (int64_t)j * n + i);
        return a;
    }, [&](int64_t i, const T &a) {
#pragma unroll
        for (int j = 1; j <= kQMax; ++j)
            if (j <= q) stn(zn + (int64_t)j * n + i, a.v[j - 1] * c.c[j]);
    });
}
void rescale(int64_t n, double *zn, int q, const Coefs &c, hipStream_t s) {
    LAUNCH_EW(k_rescale, n, s, zn, q, c);
}

template <int U>
__global__ void __launch_bounds__(kThreads) k_vsum(int64_t n, const double *__restrict__ x, const double *__restrict__ y,
                                                   double *__restrict__ z) {
    one<D2>(n, [&](int64_t i) { return D2{ldn(x + i), ldn(y + i)}; }, [&](int64_t i, const D2 &o) { stn(z + i, o.a + o.b); });
}
void vsum(int64_t n, const double *x, const double *y, double *z, hipStream_t s) {
    LAUNCH_EW(k_vsum, n, s, x, y, z);
}
// cvNls's N_VConst(0, ycor) fused into cvNlsResidual's N_VLinearSum(1, zn[0], 1, ycor, y): ycor = 0 and
// z = x + 0.0 (the same add as k_vsum with a zero operand, so -0.0 becomes +0.0 exactly as there).  24 B/entry
// instead of a 8 B/entry fill plus 24 B/entry.
template <int U>
__global__ void __launch_bounds__(kThreads) k_vsum_zero(int64_t n, const double *__restrict__ x,
                                                        double *__restrict__ ycor, double *__restrict__ z) {
    one<D1>(n, [&](int64_t i) { return D1{ldn(x + i)}; }, [&](int64_t i, const D1 &o) {
        const double zero = 0.0;
        stn(ycor + i, zero);
        stn(z + i, o.a + zero);
    });
}
void vsum_zero(int64_t n, const double *x, double *ycor, double *z, hipStream_t s) {
    LAUNCH_EW(k_vsum_zero, n, s, x, ycor, z);
}

template <int U>
__global__ void __launch_bounds__(kThreads) k_scale_to(int64_t n, double c, const double *x, double *z) {
    // x may alias z (N_VScale in place): each index is loaded before it is stored
    one<D1>(n, [&](int64_t i) { return D1{ldn(x + i)}; }, [&](int64_t i, const D1 &o) { stn(z + i, c * o.a); });
}
void scale_to(int64_t n, double c, const double *x, double *z, hipStream_t s) {
    LAUNCH_EW(k_scale_to, n, s, c, x, z);
}
void copy(int64_t n, const double *x, double *z, hipStream_t s) {
    (void)hipMemcpyAsync(z, x, n * sizeof(double), hipMemcpyDeviceToDevice, s);
}
void zero(int64_t n, double *z, hipStream_t s) { (void)hipMemsetAsync(z, 0, n * sizeof(double), s); }

// cvIncreaseBDF / cvDecreaseBDF: zn[j] = coef[j]*zn[src] + zn[j] (N_VScaleAddMulti / Vaxpy)
template <int U>
__global__ void __launch_bounds__(kThreads) k_axpy_multi(int64_t n, double *__restrict__ zn, int src, Coefs c, int jlo,
                                                         int jhi) {
    using T = DN<kQMax + 2>;              // [0]: zn[src]; [j]: zn[j], j in [jlo, jhi] (1 <= jlo)
    one<T>(n, [&](int64_t i) {
        T a;
        a.v[0] = ldn(zn + (int64_t)src * n + i);
#pragma unroll
        for (int j = 1; j <= kQMax + 1; ++j)
            if (j >= jlo && j <= jhi) a.v[j] = ldn(zn + (int64_t)j * n + i);
        return a;
    }, [&](int64_t i, const T &a) {
#pragma unroll
        for (int j = 1; j <= kQMax + 1; ++j)
            if (j >= jlo && j <= jhi) stn(zn + (int64_t)j * n + i, c.c[j] * a.v[0] + a.v[j]);
    });
}
void axpy_multi(int64_t n, double *zn, int src, const Coefs &coef, int jlo, int jhi, hipStream_t s) {
    if (jhi < jlo) return;
    LAUNCH_EW(k_axpy_multi, n, s, zn, src, coef, jlo, jhi);
}

// cvNlsResidual (res = rl1*zn[1] + ycor; res += (-gamma)*ftemp) + Newton's N_VScale(-1, delta, delta)
// + cvLsSolve's N_VWrmsNorm(b, ewt) (= SPGMR's ||s1*b||_2 / sqrt(N)).  40 B/entry.
template <int U>
__global__ void __launch_bounds__(kRedThreads) k_residual(int64_t n, const double *__restrict__ zn1,
                                                       const double *__restrict__ ycor, const double *__restrict__ ftemp,
                                                       double rl1, double ngamma, const double *__restrict__ ewt,
                                                       double *__restrict__ delta, Red r) {
    double v[1] = {0.0};
    one<D4>(n, [&](int64_t i) {
        return D4{ldn(zn1 + i), ycor ? ldn(ycor + i) : 0.0, ldn(ftemp + i), ldn(ewt + i)};      // ycor == nullptr: ycor is all +0.0
    }, [&](int64_t i, const D4 &o) {
        const double r1 = rl1 * o.a + o.b;
        const double r2 = r1 + ngamma * o.c;
        const double d = -r2;
        stn(delta + i, d);
        const double p = d * o.d;
        v[0] += p * p;
    });
    block_partial<1>(v, 0u, r);
}
void residual(int64_t n, const double *zn1, const double *ycor, const double *ftemp, double rl1, double ngamma,
              const double *ewt, double *delta, const Red &r, hipStream_t s) {
    LAUNCH_RED(k_residual, r, s, n, zn1, ycor, ftemp, rl1, ngamma, ewt, delta);
}

// SPGMR: vtemp = s1*r0; V[0] = (1/r_norm)*vtemp; and the WRMS norm of V[0]/s2 for the first DQ perturbation.
template <int U>
__global__ void __launch_bounds__(kRedThreads) k_krylov_v0(int64_t n, const double *__restrict__ delta,
                                                        const double *__restrict__ ewt, double c,
                                                        double *__restrict__ V0, Red r) {
    double v[1] = {0.0};
    one<D2>(n, [&](int64_t i) { return D2{ldn(ewt + i), ldn(delta + i)}; }, [&](int64_t i, const D2 &o) {
        const double w = o.a;
        const double x = c * (w * o.b);
        stn(V0 + i, x);
        const double p = (x / w) * w;
        v[0] += p * p;
    });
    block_partial<1>(v, 0u, r);
}
void krylov_v0(int64_t n, const double *delta, const double *ewt, double c, double *V0, const Red &r, hipStream_t s) {
    LAUNCH_RED(k_krylov_v0, r, s, n, delta, ewt, c, V0);
}

__device__ inline double dq_sig(const double *ds, int64_t n) { return 1.0 / sqrt(ds[S_SIG] / (double)n); }

// cvLsDQJtimes: work = sig*v + y with v = V[l]/s2 (N_VDiv) and sig = 1/||v||_wrms.  32 B/entry.
template <int U>
__global__ void __launch_bounds__(kThreads) k_dq_work(int64_t n, const double *__restrict__ V,
                                                      const double *__restrict__ ewt, const double *__restrict__ y,
                                                      double *__restrict__ work, const double *__restrict__ ds) {
    const double sig = dq_sig(ds, n);
    one<D3>(n, [&](int64_t i) { return D3{ldn(V + i), ldn(ewt + i), ldn(y + i)}; },
                  [&](int64_t i, const D3 &o) { stn(work + i, sig * (o.a / o.b) + o.c); });
}
void dq_work(int64_t n, const double *V, const double *ewt, const double *y, double *work, const double *ds,
             hipStream_t s) {
    LAUNCH_EW(k_dq_work, n, s, V, ewt, y, work, ds);
}

// cvLsDQJtimes tail (Jv = siginv*(f(work) - fy)), cvLsATimes (z = v - gamma*Jv), SPGMR left scaling
// (V[l+1] = s1*z), and the first two Gram-Schmidt reductions (||V[l+1]||^2, V[0].V[l+1]).  48 B/entry.
template <int U>
__global__ void __launch_bounds__(kRedThreads) k_atimes(int64_t n, double *__restrict__ w, const double *__restrict__ fy,
                                                     const double *__restrict__ V, const double *__restrict__ ewt,
                                                     const double *__restrict__ V0, double ngamma,
                                                     const double *__restrict__ ds, Red r) {
    const double sig = dq_sig(ds, n);
    const double siginv = 1.0 / sig;
    double v[2] = {0.0, 0.0};
    using T = DN<5>;
    one<T>(n, [&](int64_t i) { return T{{ldn(ewt + i), ldn(w + i), ldn(fy + i), ldn(V + i), ldn(V0 + i)}}; }, [&](int64_t i, const T &o) {
        const double e = o.v[0];
        const double jv = siginv * (o.v[1] - o.v[2]);
        const double z = ngamma * jv + o.v[3] / e;
        const double x = e * z;
        stn(w + i, x);
        v[0] += x * x;
        v[1] += o.v[4] * x;
    });
    block_partial<2>(v, 0u, r);
}
void atimes(int64_t n, double *w, const double *fy, const double *V, const double *ewt, const double *V0,
            double ngamma, const double *ds, const Red &r, hipStream_t s) {
    LAUNCH_RED(k_atimes, r, s, n, w, fy, V, ewt, V0, ngamma, ds);
}

// SUNModifiedGS step: v[k] -= h[i-1] v[i-1] (N_VLinearSum -> Vaxpy), then h[i] = v[i].v[k] (or ||v[k]||^2).
template <int U>
__global__ void __launch_bounds__(kRedThreads) k_mgs(int64_t n, double *__restrict__ w, const double *__restrict__ Vprev,
                                                  const double *__restrict__ ds, int hslot,
                                                  const double *__restrict__ Vnext, Red r) {
    const double nh = Vprev ? -ds[hslot] : 0.0;
    double v[1] = {0.0};
    one<D3>(n, [&](int64_t i) {
        return D3{ldn(w + i), Vprev ? ldn(Vprev + i) : 0.0, Vnext ? ldn(Vnext + i) : 0.0};
    }, [&](int64_t i, const D3 &o) {
        double x = o.a;
        if (Vprev) {
            x = x + nh * o.b;
            stn(w + i, x);
        }
        v[0] += Vnext ? o.c * x : x * x;
    });
    block_partial<1>(v, 0u, r);
}
void mgs(int64_t n, double *w, const double *Vprev, const double *ds, int hslot, const double *Vnext, const Red &r,
         hipStream_t s) {
    LAUNCH_RED(k_mgs, r, s, n, w, Vprev, ds, hslot, Vnext);
}

// SPGMR: V[l+1] *= 1/h[l+1][l]; and the WRMS norm of V[l+1]/s2 for the next DQ perturbation.  24 B/entry.
template <int U>
__global__ void __launch_bounds__(kRedThreads) k_normalize(int64_t n, double *__restrict__ w, double c,
                                                        const double *__restrict__ ewt, Red r) {
    double v[1] = {0.0};
    one<D2>(n, [&](int64_t i) { return D2{ldn(w + i), ldn(ewt + i)}; }, [&](int64_t i, const D2 &o) {
        const double x = o.a * c;
        stn(w + i, x);
        const double e = o.b;
        const double p = (x / e) * e;
        v[0] += p * p;
    });
    block_partial<1>(v, 0u, r);
}
void normalize(int64_t n, double *w, double c, const double *ewt, const Red &r, hipStream_t s) {
    LAUNCH_RED(k_normalize, r, s, n, w, c, ewt);
}

// SPGMR solution xcor = sum_k yg[k] V[k] (N_VLinearCombination into xcor = 0), x = xcor/s2 (N_VDiv),
// cvLsSolve's b = x, Newton's ycor += delta, and the convergence test's two WRMS norms.
// (krydim <= kNuK here: SPGMR's maxl is 5; larger Krylov dimensions take the generic one-load-batch loop)
constexpr int kNuK = 8;
template <int U>
__global__ void __launch_bounds__(kRedThreads) k_newton_update(int64_t n, const double *__restrict__ V, int64_t vstride,
                                                            int krydim, Coefs yg, const double *__restrict__ dsrc,
                                                            const double *__restrict__ ewt,
                                                            double *__restrict__ ycor, int ycor_zero, Red r) {
    double v[2] = {0.0, 0.0};
    using T = DN<kNuK + 2>;               // [0] ewt, [1] ycor, [2] dsrc (krydim 0) or [2 + k] V[k]
    const bool small = krydim <= kNuK;
    one<T>(n, [&](int64_t i) {
        T a;
        a.v[0] = ldn(ewt + i);
        a.v[1] = ycor_zero ? 0.0 : ldn(ycor + i);          // ycor_zero: ycor is all +0.0 (lazy cvNls start)
        if (krydim == 0) {
            a.v[2] = dsrc ? ldn(dsrc + i) : 0.0;
        } else if (small) {
#pragma unroll
            for (int k = 0; k < kNuK; ++k)
                if (k < krydim) a.v[2 + k] = ldn(V + k * vstride + i);
        }
        return a;
    }, [&](int64_t i, const T &a) {
        const double e = a.v[0];
        double d;
        if (krydim > 0) {
            double xc = 0.0;
            if (small) {
#pragma unroll
                for (int k = 0; k < kNuK; ++k)
                    if (k < krydim) xc = xc + yg.c[k] * a.v[2 + k];
            } else {
                for (int k = 0; k < krydim; ++k) xc = xc + yg.c[k] * ldn(V + k * vstride + i);
            }
            d = xc / e;
        } else {
            d = a.v[2];
        }
        const double yc = a.v[1] + d;
        stn(ycor + i, yc);
        const double p = d * e, q = yc * e;
        v[0] += p * p;
        v[1] += q * q;
    });
    block_partial<2>(v, 0u, r);
}
void newton_update(int64_t n, const double *V, int64_t vstride, int krydim, const Coefs &yg, const double *dsrc,
                   const double *ewt, double *ycor, bool ycor_zero, const Red &r, hipStream_t s) {
    LAUNCH_RED(k_newton_update, r, s, n, V, vstride, krydim, yg, dsrc, ewt, ycor, (int)ycor_zero);
}

// cvCompleteStep: zn[j] = l[j]*acor + zn[j] (N_VScaleAddMulti) for j in [jlo, q], optional zn[qmax] = acor.
template <int U>
__global__ void __launch_bounds__(kThreads) k_complete(int64_t n, double *__restrict__ zn,
                                                       const double *__restrict__ acor, Coefs l, int jlo, int q,
                                                       int copy_to) {
    using T = DN<kQMax + 2>;              // [0] acor, [1 + j] zn[j], jlo <= j <= q
    one<T>(n, [&](int64_t i) {
        T a;
        a.v[0] = ldn(acor + i);
#pragma unroll
        for (int j = 0; j <= kQMax; ++j)
            if (j >= jlo && j <= q) a.v[1 + j] = ldn(zn + (int64_t)j * n + i);
        return a;
    }, [&](int64_t i, const T &a) {
#pragma unroll
        for (int j = 0; j <= kQMax; ++j)
            if (j >= jlo && j <= q) stn(zn + (int64_t)j * n + i, l.c[j] * a.v[0] + a.v[1 + j]);
        if (copy_to >= 0) stn(zn + (int64_t)copy_to * n + i, a.v[0]);
    });
}
void complete_step(int64_t n, double *zn, const double *acor, const Coefs &l, int jlo, int q, int copy_to,
                   hipStream_t s) {
    LAUNCH_EW(k_complete, n, s, zn, acor, l, jlo, q, copy_to);
}

// cvCompleteStep fused with the next step's cvEwtSetSS + N_VWrmsNorm(zn[0], ewt) (CVode's loop runs them back to
// back on the same zn[0]): the k_complete update, then k_ewt's arithmetic on the new zn[0] into ewt_next (a second
// buffer: cvPrepareNextStep still reads the current ewt).  Saves k_ewt's re-read of zn[0] and a launch.
template <int U>
__global__ void __launch_bounds__(kRedThreads) k_complete_ewt(int64_t n, double *__restrict__ zn,
                                                              const double *__restrict__ acor, Coefs l, int q,
                                                              int copy_to, int jst, double rtol, double atol,
                                                              double *__restrict__ ewt_next, Red r) {
    double v[2] = {INFINITY, 0.0};
    using T = DN<kQMax + 2>;
    one<T>(n, [&](int64_t i) {
        T a;
        a.v[0] = ldn(acor + i);
#pragma unroll
        for (int j = 0; j <= kQMax; ++j)
            if (j <= q) a.v[1 + j] = ldn(zn + (int64_t)j * n + i);
        return a;
    }, [&](int64_t i, const T &a) {
        double z0 = 0.0;
#pragma unroll
        for (int j = 0; j <= kQMax; ++j)
            if (j <= q) {
                const double z = l.c[j] * a.v[0] + a.v[1 + j];
                if (j >= jst) stn(zn + (int64_t)j * n + i, z);      // jst = 1: zn[0]'s completion stays pending
                if (j == 0) z0 = z;
            }
        if (copy_to >= 0) stn(zn + (int64_t)copy_to * n + i, a.v[0]);
        const double t = rtol * fabs(z0) + atol;                 // k_ewt
        const double w = 1.0 / t;
        stn(ewt_next + i, w);
        v[0] = fmin(v[0], t);
        const double p = z0 * w;
        v[1] += p * p;
    });
    block_partial<2>(v, 1u, r);
}
void complete_step_ewt(int64_t n, double *zn, const double *acor, const Coefs &l, int q, int copy_to, int jst,
                       double rtol, double atol, double *ewt_next, const Red &r, hipStream_t s) {
    LAUNCH_RED(k_complete_ewt, r, s, n, zn, acor, l, q, copy_to, jst, rtol, atol, ewt_next);
}

// cvComputeEtaqm1 / cvComputeEtaqp1 norms in one pass
template <int U>
__global__ void __launch_bounds__(kRedThreads) k_eta_norms(int64_t n, const double *__restrict__ znq,
                                                        const double *__restrict__ znqmax,
                                                        const double *__restrict__ acor, double ncquot,
                                                        const double *__restrict__ ewt, int pq, double lq, Red r) {
    double v[2] = {0.0, 0.0};
    const bool need_acor = znqmax || pq;
    one<D4>(n, [&](int64_t i) {
        return D4{ldn(ewt + i), znq ? ldn(znq + i) : 0.0, znqmax ? ldn(znqmax + i) : 0.0, need_acor ? ldn(acor + i) : 0.0};
    }, [&](int64_t, const D4 &o) {
        const double e = o.a;
        if (znq) {
            const double zq = pq ? lq * o.d + o.b : o.b;              // pending completion: k_complete's value
            const double p = zq * e;
            v[0] += p * p;
        }
        if (znqmax) {
            const double t = ncquot * o.c + o.d;
            const double p = t * e;
            v[1] += p * p;
        }
    });
    block_partial<2>(v, 0u, r);
}
void eta_norms(int64_t n, const double *zn_q, const double *zn_qmax, const double *acor, double ncquot,
               const double *ewt, int pend_q, double lq, const Red &r, hipStream_t s) {
    LAUNCH_RED(k_eta_norms, r, s, n, zn_q, zn_qmax, acor, ncquot, ewt, pend_q, lq);
}

// N_VLinearSum_Serial's case analysis for z distinct from x and y
__device__ inline double lin_sum2(double a, double x, double b, double y) {
    if (a == 1.0 && b == 1.0) return x + y;
    if (a == 1.0 && b == -1.0) return x - y;
    if (a == -1.0 && b == 1.0) return y - x;
    if (a == 1.0) return (b * y) + x;
    if (b == 1.0) return (a * x) + y;
    if (a == -1.0) return (b * y) - x;
    if (b == -1.0) return (a * x) - y;
    if (a == b) return a * (x + y);
    if (a == -b) return a * (x - y);
    return (a * x) + (b * y);
}

struct Js {
    int j[kQMax + 1];
};

// CVodeGetDky: N_VLinearCombination(nvec, c, zn[js], dky), then N_VScale(h^-k, dky, dky) for k > 0
__global__ void __launch_bounds__(kThreads) k_dky(int64_t n, const double *__restrict__ zn, int64_t stride, Js js,
                                                  Coefs c, int nvec, double rscale, double *__restrict__ out, Pend pd) {
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
        const double ac = pd.acor ? pd.acor[i] : 0.0;
        auto Zj = [&](int j) {            // zn[j] as completed (k_complete's value when its completion is pending)
            const double z = zn[j * stride + i];
            return (pd.acor && j >= pd.j0 && j <= pd.q) ? pd.l.c[j] * ac + z : z;
        };
        double z;
        if (nvec == 1) {
            z = c.c[0] * Zj(js.j[0]);
        } else if (nvec == 2) {
            z = lin_sum2(c.c[0], Zj(js.j[0]), c.c[1], Zj(js.j[1]));
        } else {
            z = c.c[0] * Zj(js.j[0]);
            for (int k = 1; k < nvec; ++k) z += c.c[k] * Zj(js.j[k]);
        }
        if (rscale != 0.0) z *= rscale;
        out[i] = z;
    }
}
void dky(int64_t n, const double *zn, int64_t stride, const int *jsv, const Coefs &c, int nvec, double rscale,
         double *out, const Pend &pd, hipStream_t s) {
    Js js{};
    for (int k = 0; k < nvec && k <= kQMax; ++k) js.j[k] = jsv[k];
    k_dky<<<ew_blocks(n), kThreads, 0, s>>>(n, zn, stride, js, c, nvec, rscale, out, pd);   // one entry per thread
}

}  // namespace ode
}  // namespace shud
