// shud_physics.h — device-side leaf physics shared by the element/river kernels (fp64, reference order).
// Every function restates a reference routine cited inline; NOT fmin/fmax anywhere (NaN behaviour of the
// reference's own min/max, functions.hpp:117-123, must be kept).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "shud_dev.h"

namespace shud {

// ---- constants: src/Model/Macros.hpp:46-77 ----
#define K_EPSILON 0.005
#define K_ZERO 1.0e-10
#define K_EPS_SLOPE 0.05e-6
#define K_FC_RATIO 0.75
#define K_PI 3.1415926
#define K_GRAV 9.8
#define K_MAXYSURF 0.5
#define K_NA_VALUE -9999.0

// functions.hpp:117-123 (NOT fmin/fmax: NaN behaviour must match)
__device__ __forceinline__ double rmin(double a, double b) { return (a > b ? b : a); }
__device__ __forceinline__ double rmax(double a, double b) { return (a < b ? b : a); }
__device__ __forceinline__ double pow23(double x) { double t = cbrt(x); return t * t; }

// Equations.hpp:54-63
__device__ __forceinline__ double manning(double A, double n, double R, double S) {
    if (S > 0) return sqrt(S) * A * pow23(R) / n;
    return -1.0 * sqrt(-S) * A * pow23(R) / n;
}
// Equations.cpp:116-134 (range check reported through *bad)
__device__ __forceinline__ double eff_kh(double ygw, double aq, double macd, double kmac, double af,
                                         double kmx) {
    double e;
    if (macd <= K_ZERO || ygw < aq - macd) e = kmx;
    else if (ygw > aq) e = (kmac * macd * af + kmx * (aq - macd * af)) / aq;
    else e = (kmac * (ygw - (aq - macd)) * af + kmx * (aq - macd + (ygw - (aq - macd)) * (1 - af))) / ygw;
    return e;
}
// MD_RiverFlux.cpp:65-98
__device__ __forceinline__ double weir_jtoi(double zi, double yi, double zj, double yj, double zbank,
                                            double cwr, double width, double thr) {
    double hi = yi + zi, hj = yj + zj, dh = hj - hi, y, Q;
    if (dh > 0.) {
        y = hi - zbank;
        if ((y > 0.) & (yj > thr)) {
            if (hi > zbank) y = dh;
            Q = cwr * sqrt(2. * K_GRAV * y) * width * y * 60.;
        } else Q = 0.;
    } else {
        y = hi - zbank;
        if (y > 0. && yi > thr) {
            if (hj > zbank) y = -dh;
            Q = -1. * cwr * sqrt(2. * K_GRAV * y) * width * y * 60.;
        } else Q = 0.;
    }
    return Q;
}
// Flux_RiverElement.cpp:11-55
__device__ __forceinline__ double r2e_gw(double yr, double zr, double ye, double ze, double kele,
                                         double kriv, double L, double D) {
    if (kele < K_ZERO || kriv < K_ZERO) return 0.;
    double K = (kele * 1. + kriv * 1.) / (1. + 1.);   // meanArithmetic(k1,k2,1,1) Equations.hpp:50-52
    double he = ye + ze, hr = yr + zr, dh = hr - he, A, Q = 0.;
    if (dh > K_ZERO) {
        A = (he > zr) ? (yr + (he - zr)) * .5 * L : yr * L;
        Q = (yr < K_EPSILON) ? 0. : A * K * (dh / D);
    } else if (dh < -K_ZERO) {
        if (ye > K_ZERO) { A = (yr + (he - zr)) * .5 * L; Q = A * K * (dh / D); }
    }
    return Q;
}

// single-use stream loads: non-temporal when the variant asks for it (VAR bit 1)
template <int VAR, class T>
__device__ __forceinline__ T ld1(const T *p) {
    if (VAR & 2) return __builtin_nontemporal_load(p);
    return *p;
}
template <int VAR, class T>
__device__ __forceinline__ void st1(T *p, T v) {
    if (VAR & 2) __builtin_nontemporal_store(v, p);
    else *p = v;
}
// minimum waves per SIMD requested by the variant (VAR bits 2-3)
template <int VAR> struct LB { static constexpr int w = ((VAR >> 2) & 3) == 1 ? 6 : ((VAR >> 2) & 3) == 2 ? 8 : 1; };
// workgroup -> element block: VAR bit 0 deals consecutive element blocks to the same XCD (blocks are
// dispatched round-robin over the 8 XCDs, so b and b+8 share an L2): the rows above/below an element
// block then sit in that XCD's L2.  Placement affects speed only, never results.
template <int VAR>
__device__ __forceinline__ int block_id() {
    if (VAR & 1) {
        const int per = gridDim.x >> 3;            // grid is padded to a multiple of 8 by the launcher
        return (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    }
    return blockIdx.x;
}

// record an error: bit in flags, lowest index per bit
__device__ __forceinline__ void report(DevErr *e, uint32_t bit, int slot, int idx) {
    atomicOr(&e->flags, bit);
    atomicMin(&e->first_index[slot], idx);
}

// uYgw after f_update's BC logic (MD_update.cpp:114-125 / MD_f_omp.cpp:119-128)
template <int MODE>
__device__ __forceinline__ double ugw_of(const DevMesh &m, const YView &Y, int i, int ibc) {
    if (ibc == 0) {
        double g = Y.gw(i);
        return MODE == 0 ? g : rmax(0.0, g);
    }
    if (ibc > 0) return m.eybc[ibc];
    return m.ugw_stale[i];
}
// uYriv after f_update's clamp + BC logic (MD_update.cpp:145-163 / MD_f_omp.cpp:152-167)
template <int MODE>
__device__ __forceinline__ double uriv_of(const DevMesh &m, const YView &Y, int r, double *yraw_geom) {
    double yr = Y.riv(r);
    if (MODE == 1) yr = (yr >= 0.) ? yr : 0.;
    *yraw_geom = yr;                                   // updateRiver() sees the pre-BC value
    int bc = m.riv_bc[r];
    if (bc > 0) yr = m.rybc[bc];
    return yr;
}

}  // namespace shud
