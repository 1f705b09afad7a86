/* tests/pow_tab_emul.c — test infrastructure: pow_tab (shud-up_amd/csrc/shud_powtab.h, the element kernel's pow for
 * satKfun) compiled as host C from the same header the HIP kernels use, with glibc's correctly rounded fma; built with
 * -ffp-contract=off by tests/test_kat.py, which checks it against glibc's pow and a high-precision reference (CPU) and
 * the device build against it bit for bit (GPU). */
#include <math.h>
#include "shud_powtab.h"

void pow_tab_eval(const double *x, const double *y, long n, double *out) {
    for (long k = 0; k < n; k++) out[k] = shud_pow_tab(x[k], y[k]);
}
void pow_glibc_eval(const double *x, const double *y, long n, double *out) {
    for (long k = 0; k < n; k++) out[k] = pow(x[k], y[k]);
}
