// shud_powtab.h — pow_tab(x, y): a table-driven pow for a positive finite base x and a finite exponent y, in C that
// compiles both as HIP device code (shud_physics.h: satKfun's two pow calls, Equations.cpp:136-141) and as host C
// (tests/pow_tab_emul.c: the CPU restatement the GPU is checked against bit for bit, and that is measured against
// glibc's pow and a high-precision reference).  Tables: shud_pow_tab.h (tools/gen_pow_tab.py).
//
// Why: OCML's pow core (pow_pos) costs ~180 VALU per call — an extended-precision log built from ~60 dependent
// two-sum steps and an extended exp — and satKfun's two calls were 314 of the element kernel's 1,409 VALU per wave
// (profiles/r05/ele_attr).  Here the log is a table + a degree-8 (compact: 10) polynomial in double-double and the exp a
// 128-entry table of 2^(i/128) + a degree-5 polynomial: ~60 VALU and 3 table loads per call, error within ~0.51 ulp
// of the true x^y (tests/test_kat.py measures it), where glibc's pow (the reference's) is within ~0.52 ulp too and
// OCML's within ~1 ulp.  The element kernel reads the tables from its LDS copy (the per-lane gathers from
// __constant__ memory measured 4 % slower than OCML's pow core: 10 divergent vector loads per element,
// profiles/r05/powtab/).
//
// log x = k ln2 + log c + log1p(z/c - 1) with x = 2^k z, z in [OFF, 2 OFF), invc = 1/c to 9 significant bits so
// r = z*invc - 1 is exact in one fma; exp(t) = 2^(j/128) 2^(k') exp(r) with r = t - (128 k' + j) ln2/128.
// Domain: x > 0 (subnormal x rescaled on a cold path), y finite, y log x < 709.78 (no overflow path: the callers'
// bases are in (0, 1] with positive exponents); underflow to subnormal / zero is rounded once (specialcase).
#pragma once
#include <stdint.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif
#include "shud_pow_tab.h"

#ifdef __HIPCC__
#define SHUD_PT_FN __device__ __forceinline__
#else
#define SHUD_PT_FN static inline
#endif

SHUD_PT_FN uint64_t shud_pt_asu(double x) { uint64_t u; __builtin_memcpy(&u, &x, 8); return u; }
SHUD_PT_FN double shud_pt_asd(uint64_t u) { double x; __builtin_memcpy(&x, &u, 8); return x; }
// two adjacent table doubles (16-B aligned): one 16-B load on the device (ds_read_b128 from the LDS copy)
SHUD_PT_FN void shud_pt_ld2(const double *p, double *a, double *b) {
#ifdef __HIPCC__
    typedef double shud_pt_v2 __attribute__((ext_vector_type(2)));
    const shud_pt_v2 v = *(const shud_pt_v2 *)p;
    *a = v.x;
    *b = v.y;
#else
    __builtin_memcpy(a, p, 8);                    // (the tables may hold integer bit patterns: no aliasing of types)
    __builtin_memcpy(b, p + 1, 8);
#endif
}
SHUD_PT_FN float shud_pt_asf(uint32_t u) { float x; __builtin_memcpy(&x, &u, 4); return x; }

// SHUD_PT_COMPACT (default): the 2.5-KiB log table (128 x {logc, logctail} + 128 float invc with 8 significant bits)
// and a degree-10 log1p polynomial instead of the 8-KiB one (256 x 32 B) and degree 8.  The tables are copied into
// every element workgroup's LDS, and that copy is not free: 10 KiB more per workgroup measured 3 % of the element
// kernel (pow_pos with and without the unused copy, profiles/r05/pow_ab/abl_compact.log); compact vs full tables
// 0.5768 vs 0.5902 ms per eval, the same accuracy (0.51 ulp, tests/test_kat.py).  0: the full tables (A/B).
#ifndef SHUD_PT_COMPACT
#define SHUD_PT_COMPACT 1
#endif

// log x as hi + *tail (|tail| <= 2^-60 |hi| or so); ix = bits of x, x normal and positive; lt = the log table
// (shud_pt_logtab or a copy of it)
SHUD_PT_FN double shud_pt_log(uint64_t ix, double *tail, const double *lt) {
    const uint64_t tmp = ix - SHUD_PT_OFF;
#if SHUD_PT_COMPACT
    const int i = (int)((tmp >> 45) & 127);
#else
    const int i = (int)((tmp >> 44) & 255);
#endif
    const int64_t k = (int64_t)tmp >> 52;                    // arithmetic shift: the exponent relative to OFF
    const uint64_t iz = ix - (tmp & (0xfffULL << 52));
    const double z = shud_pt_asd(iz);
    const double kd = (double)k;
#if SHUD_PT_COMPACT
    double logc, logctail;
    shud_pt_ld2(lt + 2 * i, &logc, &logctail);
#ifdef __HIPCC__
    const double invc = (double)((const float *)(lt + 2 * SHUD_PT_CLOG_N))[i];
#else
    float fi;
    __builtin_memcpy(&fi, (const char *)(lt + 2 * SHUD_PT_CLOG_N) + 4 * i, 4);
    const double invc = (double)fi;
#endif
#else
    double invc, logc;
    shud_pt_ld2(lt + 4 * i, &invc, &logc);
    const double logctail = lt[4 * i + 2];
#endif
    const double r = __builtin_fma(z, invc, -1.0);           // exact: invc has 9 (compact: 8) significant bits
    // k ln2 + log c + r, in double-double
    const double t1 = kd * SHUD_PT_LN2HI + logc;
    const double t2 = t1 + r;
    const double lo1 = kd * SHUD_PT_LN2LO + logctail;
    const double lo2 = t1 - t2 + r;
    // log1p(r) = r - r^2/2 + p(r)
    const double ar = -0.5 * r;
    const double ar2 = r * ar;
    const double ar3 = r * ar2;
    const double hi = t2 + ar2;
    const double lo3 = __builtin_fma(ar, r, -ar2);
    const double lo4 = t2 - hi + ar2;
    // p = r^3/3 - r^4/4 + r^5/5 - r^6/6 + r^7/7 - r^8/8 = ar3 (A1 + r A2 + ar2 (A3 + r A4 + ar2 (A5 + r A6)))
    const double A1 = -0x1.5555555555555p-1;                 // -2/3
    const double A2 = 0.5;
    const double A3 = 0x1.999999999999ap-1;                  // 4/5
    const double A4 = -0x1.5555555555555p-1;                 // -2/3
    const double A5 = -0x1.2492492492492p+0;                 // -8/7
    const double A6 = 1.0;
#if SHUD_PT_COMPACT
    // ... + r^9/9 - r^10/10 (|r| < 2^-8 + 2^-9: degree 8 would leave ~2^-62 |r|)
    const double A7 = 0x1.c71c71c71c71cp+0;                  // 16/9
    const double A8 = -0x1.999999999999ap+0;                 // -8/5
    const double p = ar3 * (A1 + r * A2 + ar2 * (A3 + r * A4 + ar2 * (A5 + r * A6 + ar2 * (A7 + r * A8))));
#else
    const double p = ar3 * (A1 + r * A2 + ar2 * (A3 + r * A4 + ar2 * (A5 + r * A6)));
#endif
    const double lo = lo1 + lo2 + lo3 + lo4 + p;
    const double y = hi + lo;
    *tail = hi - y + lo;
    return y;
}

// exp of a result below 2^-1022 (k < 0): rounded once into the subnormal range (no double rounding)
SHUD_PT_FN double shud_pt_exp_special(double tmp, uint64_t sbits) {
    sbits += 1022ULL << 52;
    const double scale = shud_pt_asd(sbits);
    double y = scale + scale * tmp;
    if (y < 1.0) {
        const double one = 1.0;
        double lo = scale - y + scale * tmp;
        const double hi = one + y;
        lo = one - hi + y + lo;
        y = (hi + lo) - one;
        if (y == 0.) y = 0.;                                 // +0 (the result is positive)
    }
    return 0x1p-1022 * y;
}

// exp(x + xtail), |xtail| <= 2^-50 |x| or so; x <= 709 (no overflow path); et = the exp table
SHUD_PT_FN double shud_pt_exp(double x, double xtail, const double *et) {
    const uint32_t abstop = (uint32_t)(shud_pt_asu(x) >> 52) & 0x7ff;
    bool special = false;
    if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {               // |x| < 2^-54 or |x| >= 512 (0x3c9 = top12(2^-54))
        if (abstop - 0x3c9u >= 0x80000000u) return 1.0 + x;  // tiny: exp(x) rounds as 1 + x
        if (abstop >= 0x409u) return x < 0. ? 0. : __builtin_inf();  // |x| >= 1024: underflow to 0 (overflow: unused)
        special = true;                                      // 512 <= |x| < 1024: the scale may leave the normal range
    }
    const double shift = 0x1.8p52;
    double kd = x * SHUD_PT_INVLN2N + shift;                 // round to nearest integer
    const uint64_t ki = shud_pt_asu(kd);
    kd -= shift;
    double r = x + kd * SHUD_PT_NEGLN2HIN + kd * SHUD_PT_NEGLN2LON;
    r += xtail;
    const int idx = 2 * (int)(ki & 127);
    const uint64_t top = ki << 45;
    double tl, sb;
    shud_pt_ld2(et + idx, &tl, &sb);
    const uint64_t sbits = shud_pt_asu(sb) + top;
    const double r2 = r * r;
    const double C2 = 0.5, C3 = 0x1.5555555555555p-3, C4 = 0x1.5555555555555p-5, C5 = 0x1.1111111111111p-7;
    const double tmp = tl + r + r2 * (C2 + r * C3) + r2 * r2 * (C4 + r * C5);
    if (special && (ki & 0x80000000ULL)) return shud_pt_exp_special(tmp, sbits);
    const double scale = shud_pt_asd(sbits);
    return scale + scale * tmp;
}

SHUD_PT_FN double shud_pow_tab_t(double x, double y, const double *lt, const double *et) {
    uint64_t ix = shud_pt_asu(x);
    if (ix < 0x0010000000000000ULL) {                        // subnormal base (cold): normalise
        ix = shud_pt_asu(x * 0x1p52);
        ix -= 52ULL << 52;
    }
    double lo;
    const double hi = shud_pt_log(ix, &lo, lt);
    const double ehi = y * hi;
    const double elo = y * lo + __builtin_fma(y, hi, -ehi);
    return shud_pt_exp(ehi, elo, et);
}
// with the tables in __constant__ memory (device) / static arrays (host)
#if SHUD_PT_COMPACT
#define SHUD_PT_LOGTAB ((const double *)shud_pt_clogtab)
#define SHUD_PT_LOG_DOUBLES (2 * SHUD_PT_CLOG_N + SHUD_PT_CLOG_N / 2)
#else
#define SHUD_PT_LOGTAB shud_pt_logtab
#define SHUD_PT_LOG_DOUBLES (4 * SHUD_PT_LOG_N)
#endif
SHUD_PT_FN double shud_pow_tab(double x, double y) { return shud_pow_tab_t(x, y, SHUD_PT_LOGTAB, shud_pt_exptab); }
