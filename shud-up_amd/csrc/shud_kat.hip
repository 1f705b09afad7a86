// shud_kat.hip — known-answer harness (test infrastructure; not part of the RHS C-ABI):
// evaluates the element/river kernels' own device leaf functions (shud_physics.h) on host-given input
// tuples, ids and argument order as oracle_kat() (oracle/shud_oracle.c).  tests/test_kat.py compares.
#include <hip/hip_runtime.h>
#include <vector>
#include "shud_physics.h"

using namespace shud;

// glibc's cbrt (sysdeps/ieee754/dbl-64/s_cbrt.c, glibc 2.35: the reference's libm for pow23's cbrt,
// Equations.hpp:36-39) restated operation for operation: x = xm 2^xe with xm in [0.5, 1), a degree-6 polynomial u ~
// xm^(1/3), one Halley step u (u^3 + 2 xm) / (2 u^3 + xm), times 2^((xe mod 3) / 3) from a 5-entry table, scaled by
// 2^(xe / 3).  2 xm and 2 u^3 are exact, so t2 + 2 xm and 2 t2 + xm are single fmas with the same rounding; the Halley
// quotient has numerator and denominator in [0.7, 3], where the bare division chain (div_nr's, without v_div_scale /
// v_div_fixup) is the IEEE quotient.  Zero, infinite and NaN x return x + x, as glibc does.  Bit-identical to glibc's
// cbrt (tests/test_kat.py::test_cbrt_glibc_bit_identical).  Not in the kernels: +1.9 % wall per eval against OCML's cbrt
// in the element kernel (profiles/r06/rfold/abv_fold_sqrt_div_cbrt.log, lib:nrcb), so Manning keeps OCML's cbrt (within the parity tolerance).
__device__ __forceinline__ double cbrt_glibc(double x) {
    constexpr double kC2 = 1.2599210498948731648, kSqC2 = 1.5874010519681994748;   // 2^(1/3), 2^(2/3)
    int xe;
    const double xm = __builtin_frexp(__builtin_fabs(x), &xe);
    double p = 0.784932344976639262 - 0.145263899385486377 * xm;
    p = -1.83469277483613086 + p * xm;
    p = 2.44693122563534430 + p * xm;
    p = -2.11499494167371287 + p * xm;
    p = 1.50819193781584896 + p * xm;
    const double u = 0.354895765043919860 + p * xm;
    const double t2 = u * u * u;
    const double num = u * __builtin_fma(xm, 2.0, t2), den = __builtin_fma(t2, 2.0, xm);
    double r = __builtin_amdgcn_rcp(den);                       // num / den: the division chain, no repairs
    double e = __builtin_fma(-den, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-den, r, 1.0);
    r = __builtin_fma(r, e, r);
    double q = num * r;
    e = __builtin_fma(-den, q, num);
    q = __builtin_fma(e, r, q);
    const int q3 = xe / 3, rem = xe - 3 * q3;                   // C's truncating / and %
    const double f = rem == 0 ? 1.0 : rem == 1 ? kC2 : rem == 2 ? kSqC2 : rem == -1 ? 1.0 / kC2 : 1.0 / kSqC2;
    const double ym = q * f;
    const double res = __builtin_ldexp(x > 0.0 ? ym : -ym, q3);
    return __builtin_isfpclass(x, 0x0003 | 0x0204 | 0x0060) ? x + x : res;    // NaN, +-inf, +-0
}

enum { KAT_MANNING, KAT_EFFKH, KAT_WEIR, KAT_R2E, KAT_SATK, KAT_SMS, KAT_DADY, KAT_AREA, KAT_PEREM, KAT_TOPW,
       KAT_TOPAREA, KAT_COUNT };
static const int kat_nin_tab[KAT_COUNT] = {4, 6, 8, 8, 2, 3, 3, 4, 4, 4, 4};

__global__ void kat_kernel(int fn, int k, const double *__restrict__ in, int n, double *__restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const double *x = in + (size_t)t * k;
    double r = 0.;
    switch (fn) {
        case KAT_MANNING: r = manning(x[0], x[1], x[2], x[3]); break;
        case KAT_EFFKH: r = eff_kh(x[0], x[1], x[2], x[3], x[4], x[5]); break;
        case KAT_WEIR: r = weir_jtoi(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]); break;
        case KAT_R2E: r = r2e_gw(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]); break;
        case KAT_SATK: {                       // class exponents as the handle derives them (shud_rhs.cpp)
            const double nb = x[1];
            r = sat_kfun(x[0], nb / (nb - 1.), (nb - 1.) / nb);
            break;
        }
        case KAT_SMS: {                        // dth and fcmr as the handle derives them
            const double ths = x[0], thr = x[1];
            r = soil_moisture_stress((x[2] * (ths - thr) - thr) / (ths * 0.75 - thr));
            break;
        }
        case KAT_DADY: r = da_to_dy(x[0], x[1], x[2]); break;
        case KAT_AREA: r = riv_geom(x[0], x[1], x[2], x[3]).csarea; break;
        case KAT_PEREM: r = riv_geom(x[0], x[1], x[2], x[3]).csperem; break;
        case KAT_TOPW: r = riv_geom(x[0], x[1], x[2], x[3]).topw; break;
        case KAT_TOPAREA: r = riv_geom(x[0], x[1], x[2], x[3]).toparea; break;
    }
    out[t] = r;
}

// pow_tab (shud_powtab.h) next to OCML's full pow on the same (x, y) pairs: which = 0 pow, 2 pow_tab
__global__ void kat_pow_kernel(int which, const double *__restrict__ xy, int n, double *__restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const double x = xy[2 * t], y = xy[2 * t + 1];
    out[t] = which == 2 ? shud_pow_tab(x, y) : pow(x, y);
}
extern "C" int shud_kat_pow(int which, const double *h_xy, int n, double *h_out) {
    if (n <= 0) return -1;
    double *d_xy = nullptr, *d_out = nullptr;
    if (hipMalloc(&d_xy, sizeof(double) * 2 * (size_t)n) != hipSuccess) return -3;
    if (hipMalloc(&d_out, sizeof(double) * (size_t)n) != hipSuccess) { (void)hipFree(d_xy); return -3; }
    int rc = 0;
    if (hipMemcpy(d_xy, h_xy, sizeof(double) * 2 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess) rc = -3;
    if (!rc) {
        hipLaunchKernelGGL(kat_pow_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, which, d_xy, n, d_out);
        if (hipGetLastError() != hipSuccess) rc = -3;
    }
    if (!rc && hipMemcpy(h_out, d_out, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) rc = -3;
    (void)hipFree(d_xy);
    (void)hipFree(d_out);
    return rc;
}

// cos_small (shud_physics.h: OCML's small-argument cos path) next to OCML's full cos: which = 0 cos, 1 cos_small
__global__ void kat_cos_kernel(int which, const double *__restrict__ x, int n, double *__restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    out[t] = which ? cos_small(x[t]) : cos(x[t]);
}
extern "C" int shud_kat_cos(int which, const double *h_x, int n, double *h_out) {
    if (n <= 0) return -1;
    double *d = nullptr;
    const size_t bytes = sizeof(double) * (size_t)n;
    if (hipMalloc(&d, 2 * bytes) != hipSuccess) return -3;
    int rc = 0;
    if (hipMemcpy(d, h_x, bytes, hipMemcpyHostToDevice) != hipSuccess) rc = -3;
    if (!rc) {
        hipLaunchKernelGGL(kat_cos_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, which, d, n, d + n);
        if (hipGetLastError() != hipSuccess) rc = -3;
    }
    if (!rc && hipMemcpy(h_out, d + n, bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = -3;
    (void)hipFree(d);
    return rc;
}

extern "C" int shud_kat_nin(int fn) { return (fn >= 0 && fn < KAT_COUNT) ? kat_nin_tab[fn] : -1; }

extern "C" int shud_kat_eval(int fn, const double *h_in, int n, double *h_out) {
    if (fn < 0 || fn >= KAT_COUNT || n <= 0) return -1;
    const int k = kat_nin_tab[fn];
    double *d_in = nullptr, *d_out = nullptr;
    if (hipMalloc(&d_in, sizeof(double) * k * (size_t)n) != hipSuccess) return -3;
    if (hipMalloc(&d_out, sizeof(double) * (size_t)n) != hipSuccess) { (void)hipFree(d_in); return -3; }
    int rc = 0;
    if (hipMemcpy(d_in, h_in, sizeof(double) * k * (size_t)n, hipMemcpyHostToDevice) != hipSuccess) rc = -3;
    if (!rc) {
        hipLaunchKernelGGL(kat_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, fn, k, d_in, n, d_out);
        if (hipGetLastError() != hipSuccess) rc = -3;
    }
    if (!rc && hipMemcpy(h_out, d_out, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) rc = -3;
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return rc;
}

// ---- published ODE test problems on the device, for the integrator (tests/test_gpu_ode.py) ----
// Same expressions, same order as oracle/shud_oracle_ode.c (robertson_rhs, decay_rhs, decayn_rhs).
struct KatOde {
    int problem;
    hipStream_t s;
};
__constant__ double kat_decay_lam[3] = {1.0, 10.0, 1000.0};
__constant__ double kat_decayn_lam[7] = {0.01, 0.1, 1.0, 10.0, 100.0, 1000.0, 10000.0};

__global__ void kat_ode_kernel(int problem, int64_t n, const double *__restrict__ y, double *__restrict__ yd) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (problem == 1) {                                          // Robertson (1966)
        if (i != 0) return;
        const double y1 = y[0], y2 = y[1], y3 = y[2];
        const double a = -0.04 * y1 + 1.0e4 * y2 * y3;
        const double c = 3.0e7 * y2 * y2;
        yd[0] = a;
        yd[2] = c;
        yd[1] = -a - c;
    } else if (problem == 2) {
        if (i < 3) yd[i] = -kat_decay_lam[i] * y[i];
    } else if (i < n) {
        yd[i] = -kat_decayn_lam[i % 7] * y[i];
    }
}

extern "C" void *shud_kat_ode_user(int problem) {
    KatOde *u = new KatOde{problem, nullptr};
    if (hipStreamCreate(&u->s) != hipSuccess) { delete u; return nullptr; }
    return u;
}
extern "C" void *shud_kat_ode_stream(void *u) { return u ? ((KatOde *)u)->s : nullptr; }
static int64_t kat_ode_n = 0;
extern "C" void shud_kat_ode_set_n(int64_t n) { kat_ode_n = n; }
extern "C" int shud_kat_ode_rhs(double t, const double *y, double *yd, void *user) {
    (void)t;
    KatOde *u = (KatOde *)user;
    const int64_t n = u->problem == 3 ? kat_ode_n : 3;
    hipLaunchKernelGGL(kat_ode_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, u->s, u->problem, n, y, yd);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" void shud_kat_ode_free(void *user) {
    KatOde *u = (KatOde *)user;
    if (!u) return;
    (void)hipStreamSynchronize(u->s);
    (void)hipStreamDestroy(u->s);
    delete u;
}

// sqrt_nr / div_nr (shud_physics.h) next to the device's own sqrt and IEEE division on the same operands: which = 0
// sqrt_nr(a), 1 sqrt(a), 2 div_nr(a, recip_nr(b)), 3 a / b, 4 cbrt_glibc(a)
__global__ void kat_fast_kernel(int which, const double *__restrict__ a, const double *__restrict__ b, int n,
                                double *__restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    double r;
    switch (which) {
        case 0: r = sqrt_nr(a[t]); break;
        case 1: r = sqrt(a[t]); break;
        case 2: r = div_nr(a[t], recip_nr(b[t])); break;
        case 4: r = cbrt_glibc(a[t]); break;
        default: r = a[t] / b[t]; break;
    }
    out[t] = r;
}
extern "C" int shud_kat_fast(int which, const double *h_a, const double *h_b, int n, double *h_out) {
    if (n <= 0) return -1;
    double *d = nullptr;
    const size_t bytes = sizeof(double) * (size_t)n;
    if (hipMalloc(&d, 3 * bytes) != hipSuccess) return -3;
    int rc = 0;
    if (hipMemcpy(d, h_a, bytes, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d + n, h_b, bytes, hipMemcpyHostToDevice) != hipSuccess)
        rc = -3;
    if (!rc) {
        hipLaunchKernelGGL(kat_fast_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, which, d, d + n, n, d + 2 * (size_t)n);
        if (hipGetLastError() != hipSuccess) rc = -3;
    }
    if (!rc && hipMemcpy(h_out, d + 2 * (size_t)n, bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = -3;
    (void)hipFree(d);
    return rc;
}

// cdiv (shud_physics.h) on host-given (a, b) pairs with the host's correctly rounded rb = 1/b, as the handle
// supplies it (tests/test_kat.py::test_cdiv_bit_identical compares against IEEE a / b)
__global__ void kat_cdiv_kernel(const double *__restrict__ a, const double *__restrict__ b,
                                const double *__restrict__ rb, int n, double *__restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) out[t] = cdiv(a[t], b[t], rb[t]);
}
extern "C" int shud_kat_cdiv(const double *h_a, const double *h_b, int n, double *h_out) {
    if (n <= 0) return -1;
    std::vector<double> rb(n);
    for (int k = 0; k < n; k++) rb[k] = 1. / h_b[k];
    double *d = nullptr;
    const size_t bytes = sizeof(double) * (size_t)n;
    if (hipMalloc(&d, 4 * bytes) != hipSuccess) return -3;
    int rc = 0;
    if (hipMemcpy(d, h_a, bytes, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d + n, h_b, bytes, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d + 2 * (size_t)n, rb.data(), bytes, hipMemcpyHostToDevice) != hipSuccess)
        rc = -3;
    if (!rc) {
        hipLaunchKernelGGL(kat_cdiv_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, d, d + n, d + 2 * (size_t)n, n,
                           d + 3 * (size_t)n);
        if (hipGetLastError() != hipSuccess) rc = -3;
    }
    if (!rc && hipMemcpy(h_out, d + 3 * (size_t)n, bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = -3;
    (void)hipFree(d);
    return rc;
}
