// shud_physics.h — device-side leaf physics shared by the element/river kernels (fp64, reference order).
// Every function restates a reference routine cited inline; NOT fmin/fmax anywhere (NaN behaviour of the
// reference's own min/max, functions.hpp:117-123, must be kept).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "shud_dev.h"
#include "shud_powtab.h"

namespace shud {

// a / b for a class-constant divisor b with its host-computed, correctly rounded reciprocal rb:
// q0 = a*rb is within 1 ulp of a/b, the residual a - q0*b is exact in one fma, and one fma correction then
// rounds to nearest exactly like IEEE division (Markstein's theorem; round-to-nearest, no under/overflow).
// Exact, zero, infinite and NaN residuals keep q0 (signed zeros and infinities as a/b gives them).
// Range: the handle admits a divisor only when it is 0, +-inf, NaN or 2^-20 <= |b| <= 2^20 (kCdivBmin/Bmax,
// checked at create); then for 2^-948 <= |a| <= 2^1000 neither q0 nor the residual leaves the normal range and
// the theorem holds.  Outside that numerator range (tiny non-zero or huge a: subnormal quotients, overflow of
// a*rb) the exec-masked cold path takes the IEEE division itself, so cdiv(a, b, RN(1/b)) == a / b for every a
// (tests/test_kat.py::test_cdiv_bit_identical on subnormal, near-overflow, signed-zero and special operands).
// Zero, infinite and NaN numerators and 0/inf/NaN divisors stay on the fast path: q0 is then already a / b.
__device__ __forceinline__ double cdiv(double a, double b, double rb) {
    const double q0 = a * rb;
    const double e = __builtin_fma(-q0, b, a);
    // e zero, infinite or NaN (one v_cmp_class): keep q0
    double q = __builtin_isfpclass(e, 0x0003 | 0x0204 | 0x0060) ? q0 : __builtin_fma(e, rb, q0);
    const double aa = __builtin_fabs(a);
    if (__builtin_expect((aa < 0x1p-948 && a != 0.) || aa > 0x1p1000, 0)) q = a / b;
    return q;
}

// ---- the compiler's correctly rounded f64 sqrt and division, without their range repairs on the common range ----
// sqrt: LLVM's gfx9 lowering is y = rsq(x'), g = x' y, h = y / 2, two Newton-Raphson steps on (g, h), where x' = x or,
// for x < 2^-767, x 2^256 (result scaled back by 2^-128), and a final select returns x itself for +-0 and +inf.  For x
// in [2^-767, DBL_MAX] neither repair changes anything, so the bare chain gives the same bits (tests/test_kat.py::
// test_fast_sqrt_div_bit_identical); any other x (zero, negative, tiny, inf, NaN) takes sqrt() on an exec-masked cold
// path.  Saves the scaling compare/ldexp pair and the zero/inf select (~7 VALU) per call.
__device__ __forceinline__ double sqrt_nr(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    h = __builtin_fma(h, r, h);
    g = __builtin_fma(g, r, g);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    if (__builtin_expect(!(x >= 0x1p-767 && x <= 0x1.fffffffffffffp+1023), 0)) g = sqrt(x);
    return g;
}
// division: LLVM's lowering is r = rcp(b') refined by two Newton steps, q = a' r, e = fma(-b', q, a'), q + e r (as
// v_div_fmas), then v_div_fixup for special operands, where v_div_scale rescales a, b (a' , b') only when 1/b, a/b or a
// would leave the normal range.  For |b| in [2^-100, 2^100] and |a| in [2^-900, 2^600] no operand is rescaled and
// the fixup returns the quotient as is, so the bare chain gives the same bits; and r depends on b alone, so two
// divisions by one divisor share it (Recip).  Other operands take the IEEE division on an exec-masked cold path.
// Element kernel with both (sqrt_nr in satKfun, Manning and the weir; the two Dist2Nabor divisions of an edge and the
// area divisions of the DY tail on shared reciprocals): wall per eval -0.5 % over 9 interleaved rounds, same bits
// (profiles/r06/rfold/abv_fold_sqrt_div_cbrt.log, lib:nr).
struct Recip {
    double b, r;
    bool ok;                 // |b| in [2^-100, 2^100]
};
__device__ __forceinline__ Recip recip_nr(double b) {
    Recip R;
    R.b = b;
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    R.r = __builtin_fma(r, e, r);
    const double bb = __builtin_fabs(b);
    R.ok = bb >= 0x1p-100 && bb <= 0x1p100;
    return R;
}
__device__ __forceinline__ double div_nr(double a, const Recip &R) {
    const double q0 = a * R.r;
    const double e = __builtin_fma(-R.b, q0, a);
    double q = __builtin_fma(e, R.r, q0);
    const double aa = __builtin_fabs(a);
    if (__builtin_expect(!(R.ok && aa >= 0x1p-900 && aa <= 0x1p600), 0)) q = a / R.b;
    return q;
}

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
// (glibc's cbrt restated for the device — bit-identical to the reference's libm, tests/test_kat.py — measured +1.9 %
// on the element kernel's wall per eval against OCML's cbrt, profiles/r06/rfold/abv_fold_sqrt_div_cbrt.log lib:nrcb:
// not used here; the restatement lives in the KAT library, shud_kat.hip cbrt_glibc)
__device__ __forceinline__ double pow23(double x) { const double t = cbrt(x); return t * t; }

// Equations.hpp:54-63.  The reference's two branches differ only in the sqrt argument (S or -S) and a leading
// -1.0 factor; IEEE multiplication and division round sign-symmetrically, so (-1.0*x)*A*p/n == -(x*A*p/n) bit
// for bit (zeros and NaNs included).  One sqrt of the selected argument, one chain, a final sign select —
// the compiler if-converted the two branches into two full sqrt sequences per call otherwise.
__device__ __forceinline__ double manning(double A, double n, double R, double S) {
    const bool pos = S > 0;
    const double t = sqrt_nr(pos ? S : -S) * A * pow23(R) / n;
    return pos ? t : -t;
}
// Equations.cpp:116-134 (range check reported by the caller).  The two macropore branches divide different
// numerators by different divisors; the numerator and divisor are selected per branch and ONE division follows
// the join, so a wave whose lanes take both branches runs one division sequence instead of two (same operations
// per lane, same bits).
__device__ __forceinline__ double eff_kh(double ygw, double aq, double macd, double kmac, double af,
                                         double kmx) {
    double e;
    if (macd <= K_ZERO || ygw < aq - macd) e = kmx;
    else {
        double num, den;
        if (ygw > aq) { num = kmac * macd * af + kmx * (aq - macd * af); den = aq; }
        else {
            const double t = ygw - (aq - macd);
            num = kmac * t * af + kmx * (aq - macd + t * (1 - af));
            den = ygw;
        }
        e = num / den;
    }
    return e;
}
// MD_RiverFlux.cpp:65-98
// Both branches evaluate cwr*sqrt(2g*y)*width*y*60 on their own y, the second with a leading -1.0 factor:
// as in manning() the negation is exact, so one sqrt chain on the selected y and a sign select give the same
// bits as the two branches (which the compiler otherwise if-converts into two sqrt sequences).
__device__ __forceinline__ double weir_jtoi(double zi, double yi, double zj, double yj, double zbank,
                                            double cwr, double width, double thr) {
    const double hi = yi + zi, hj = yj + zj, dh = hj - hi;
    const bool up = dh > 0.;                         // flow j -> i
    double y = hi - zbank;
    const bool on = up ? ((y > 0.) & (yj > thr)) : (y > 0. && yi > thr);
    if (up ? (hi > zbank) : (hj > zbank)) y = up ? dh : -dh;
    const double t = cwr * sqrt_nr(2. * K_GRAV * y) * width * y * 60.;
    return on ? (up ? t : -t) : 0.;
}
// Flux_RiverElement.cpp:11-55
__device__ __forceinline__ double r2e_gw(double yr, double zr, double ye, double ze, double kele, double kriv,
                                         double L, double D) {
    if (kele < K_ZERO || kriv < K_ZERO) return 0.;
    double K = (kele * 1. + kriv * 1.) / (1. + 1.);   // meanArithmetic(k1,k2,1,1) Equations.hpp:50-52
    // both flowing branches evaluate A * K * (dh / D) on their own A: one division, branch-selected A
    const double he = ye + ze, hr = yr + zr, dh = hr - he;
    const bool in = dh > K_ZERO;
    const double A = (in && !(he > zr)) ? yr * L : (yr + (he - zr)) * .5 * L;
    const bool on = in ? !(yr < K_EPSILON) : (dh < -K_ZERO && ye > K_ZERO);
    return on ? A * K * (dh / D) : 0.;
}
// x / a for x = 0.0 (QSS, never assigned by the reference): +-0 with a's sign for a non-zero a, NaN for a zero
// or NaN a — the IEEE quotient, without a division
__device__ __forceinline__ double zero_over(double a) {
    return (a != 0. && a == a) ? __builtin_copysign(0.0, a) : __builtin_nan("");
}

struct RivGeom { double csarea, csperem, topw, toparea; };
// _River::updateRiver (River.cpp:49-62) with fun_Cross* (River.hpp:115-127): geometry at stage y
__device__ __forceinline__ RivGeom riv_geom(double w0, double bs, double len, double y) {
    RivGeom g;
    const double topw = y * bs * 2.0 + w0;
    const double a = y * (w0 + y * bs);
    const double ys = y * bs;
    const double per = 2.0 * sqrt(y * y + ys * ys) + w0;
    const double eqw = 0.5 * ((y * bs * 2.0 + w0) + w0);
    const double ta = eqw * len;
    g.topw = (topw < 0.) ? 0. : topw;
    g.csarea = (a < 0.) ? 0. : a;
    g.csperem = (per < 0.) ? 0. : per;
    g.toparea = (ta < 0.) ? 0. : ta;
    return g;
}
// satKfun, Equations.cpp:136-141, with the class exponents ex1 = n/(n-1), ex2 = (n-1)/n precomputed.
// Both bases are positive here: satn in (ZERO, 0.99] (the callers' clamps), 1 - satn^ex1 in (0, 1];
// exponents are class constants of Beta > 1 (checked by the handle; the SoA kernel takes the full pow otherwise).
// pow is shud_pow_tab (shud_powtab.h: table-driven log/exp, ~60 VALU, within 0.51 ulp of x^y and equal to glibc's pow
// on 99.93 % of satKfun's domain, tests/test_kat.py).  lt / et: its log / exp tables (the packed element kernel passes
// its LDS copy; default: __constant__ memory)
__device__ __forceinline__ double sat_kfun(double satn, double ex1, double ex2, const double *lt, const double *et) {
    const double tmp = -1. + shud_pow_tab_t(1. - shud_pow_tab_t(satn, ex1, lt, et), ex2, lt, et);
    return sqrt_nr(satn) * tmp * tmp;
}
__device__ __forceinline__ double sat_kfun(double satn, double ex1, double ex2) {
    return sat_kfun(satn, ex1, ex2, SHUD_PT_LOGTAB, shud_pt_exptab);
}
// SoilMoistureStress, is_sm_et.cpp:131-140 (truncated PI), with dth = ThetaS - ThetaR and
// fcmr = ThetaS * 0.75 - ThetaR; b = (SatRatio * dth - ThetaR) / fcmr
//
// cos of K_PI * b for b in [0, 1] (the clamp also maps NaN to 0): the argument is finite and in [0, 3.1415926], so
// OCML's cos (__ocml_cos_f64: |x|, trigred = small or Payne-Hanek reduction by |x| < 2^30, sincosred2, quadrant
// selects, a non-finite select) reduces to its small-argument path; cos_small calls that path's own pieces in the
// same order and returns the same bits (tests/test_kat.py::test_cos_small_bit_identical) without the large-argument
// branch and the |x| / finiteness selects.
// fma(a, b, c) for a constant addend c: v_fma_f64 with c in an SGPR pair (one VALU + two SALU moves), where the
// compiler's v_fmac_f64 form needs c in a VGPR pair (two v_mov_b32 + the fmac: three VALU).  Same operation, same
// bits.  cos_small's nine constant-addend steps: -14 static VALU; element kernel 0.6017 vs 0.6012 ms, wall per eval
// 0.578 vs 0.580 ms (within noise, profiles/r05/tiles2/).
__device__ __forceinline__ double fma_sc(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}
// OCML's __ocmlpriv_trigredsmall_f64 + __ocmlpriv_sincosred2_f64 (ocml.bc, ROCm 7.2) restated operation for
// operation (their results come back in registers; a call to the bitcode's struct-returning functions went through
// scratch and cost the kernel 48 spill instructions)
__device__ __forceinline__ double cos_small(double x) {            // 0 <= x < 2^30, finite
    // Cody-Waite reduction by pi/2 in three parts (trigredsmall)
    const double q = __builtin_rint(x * 0x1.45f306dc9c883p-1);
    const double a = __builtin_fma(q, -0x1.921fb54442d18p+0, x);
    const double b = __builtin_fma(q, -0x1.1a62633145c00p-54, a);
    const double p = q * 0x1.1a62633145c00p-54;
    const double pe = __builtin_fma(q, 0x1.1a62633145c00p-54, -p);
    const double t = a - p;
    const double tl = ((t - b) + ((a - t) - p)) - pe;
    const double c2 = __builtin_fma(q, -0x1.b839a252049c0p-104, tl);
    const double hi = b + c2;
    const double lo = c2 - (hi - b);
    const int qi = (int)q & 3;
    // sincosred2(hi, lo)
    const double x2 = hi * hi;
    const double h = x2 * 0.5;
    const double w = 1.0 - h;
    const double wl = (1.0 - w) - h;
    const double x4 = x2 * x2;
    double pc = __builtin_fma(x2, -0x1.907db46cc5e42p-37, 0x1.1eeb69037ab78p-29);
    pc = fma_sc(x2, pc, -0x1.27e4fa17f65f6p-22);
    pc = fma_sc(x2, pc, 0x1.a01a019f4ec90p-16);
    pc = fma_sc(x2, pc, -0x1.6c16c16c16967p-10);
    pc = fma_sc(x2, pc, 0x1.5555555555555p-5);
    const double cs = w + __builtin_fma(x4, pc, __builtin_fma(hi, -lo, wl));
    double ps = __builtin_fma(x2, 0x1.5e0b2f9a43bb8p-33, -0x1.ae600b42fdfa7p-26);
    ps = fma_sc(x2, ps, 0x1.71de3796cde01p-19);
    ps = fma_sc(x2, ps, -0x1.a01a019e83e5cp-13);
    ps = fma_sc(x2, ps, 0x1.1111111110bb3p-7);
    const double x3 = hi * -x2;
    double sn = __builtin_fma(x3, ps, lo * 0.5);
    sn = __builtin_fma(x2, sn, -lo);
    sn = hi - __builtin_fma(x3, -0x1.5555555555555p-3, sn);
    const double c = (qi & 1) ? -sn : cs;
    return qi > 1 ? -c : c;
}
__device__ __forceinline__ double soil_moisture_stress(double b) {
    b = rmin(rmax(0., b), 1.);
    return 0.5 * (1 - cos_small(K_PI * b));
}
// fun_dAtodY + Quadratic, functions.hpp:125-153
__device__ __forceinline__ double da_to_dy(double dA, double w_top, double s) {
    if (dA == 0.) return 0.;
    if (fabs(s) < K_EPS_SLOPE) return dA / w_top;
    const double sa = fabs(s);
    const double cc = w_top * w_top + 4 * sa * dA;
    return (cc < K_ZERO) ? -1. * w_top / (2. * sa) : (-w_top + sqrt(cc)) / (2 * sa);
}


// record an error / warning, aggregated per wave: one lane (the lowest flagged lane = lowest element index
// of the wave, since lanes map to consecutive indices) does the atomics for the whole wave.  flags only gain
// bits and first_index only decreases, so a plain load that already shows the bit / a smaller index proves
// the atomic would change nothing (a stale load can only cost a redundant atomic): inputs that flag every
// element then issue ~no atomics on the shared word, and the warning count goes to one of kWarnSlots
// lines.  Must be reached by every active lane (it is a __ballot).
__device__ __forceinline__ void report_w(DevErr *e, bool c, uint32_t bit, int slot, int idx, bool count = false) {
    const unsigned long long mask = __builtin_amdgcn_ballot_w64(c);     // the compare's own lane mask
    if (mask == 0ULL) return;
    if ((int)__lane_id() == __ffsll((long long)mask) - 1) {
        if (!(__atomic_load_n(&e->flags, __ATOMIC_RELAXED) & bit)) atomicOr(&e->flags, bit);
        if (__atomic_load_n(&e->first_index[slot], __ATOMIC_RELAXED) > idx) atomicMin(&e->first_index[slot], idx);
        if (count) {
            unsigned long long *w = __atomic_load_n(&e->warn, __ATOMIC_RELAXED);
            atomicAdd(w + (blockIdx.x & (kWarnSlots - 1)) * kWarnStride, (unsigned long long)__popcll(mask));
        }
    }
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
