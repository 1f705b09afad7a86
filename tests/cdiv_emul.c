/* tests/cdiv_emul.c — test infrastructure: the device cdiv (shud-up_amd/csrc/shud_physics.h) restated in C with
 * glibc's correctly rounded fma, so tests/test_kat.py can check the reciprocal-division algorithm itself against
 * IEEE division on the CPU (built with -ffp-contract=off; no GPU). */
#include <math.h>

static double cdiv(double a, double b, double rb) {
    const double q0 = a * rb;
    const double e = fma(-q0, b, a);
    double q = (e == 0. || !isfinite(e)) ? q0 : fma(e, rb, q0);
    const double aa = fabs(a);
    if ((aa < 0x1p-948 && a != 0.) || aa > 0x1p1000) q = a / b;
    return q;
}

/* unguarded: the pre-round-3 form, to show what the guard changes */
static double cdiv_raw(double a, double b, double rb) {
    const double q0 = a * rb;
    const double e = fma(-q0, b, a);
    return (e == 0. || !isfinite(e)) ? q0 : fma(e, rb, q0);
}

void cdiv_eval(const double *a, const double *b, int n, int guarded, double *out) {
    for (int k = 0; k < n; k++) {
        const double rb = 1. / b[k];
        out[k] = guarded ? cdiv(a[k], b[k], rb) : cdiv_raw(a[k], b[k], rb);
    }
}
