// calibrate_pmc.hip — known-byte kernels to calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the
// access widths the SHUD kernels use (MI355X_MICROARCH.md §HBM: FETCH_SIZE is exact only after a
// per-pattern calibration; 16 B/lane streaming reads report 1/2).  Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./calibrate_pmc      (and separately --pmc WRITE_SIZE)
// and divide each kernel's counter by the bytes printed here.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void rd_x2(const double *__restrict__ a, size_t n, double *out) {   // 8 B / lane
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    double s = 0;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.678) out[0] = s;
}
__global__ void rd_x4(const double2 *__restrict__ a, size_t n2, double *out) { // 16 B / lane
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    double s = 0;
    for (; i < n2; i += (size_t)gridDim.x * blockDim.x) { double2 v = a[i]; s += v.x + v.y; }
    if (s == 12345.678) out[0] = s;
}
__global__ void rd_x1(const int *__restrict__ a, size_t n, double *out) {       // 4 B / lane
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    int s = 0;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 123456789) out[0] = s;
}
__global__ void wr_x2(double *__restrict__ a, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}
// one lane per element reading 12 separate SoA double arrays (the element kernel's pattern)
__global__ void rd_soa12(const double *__restrict__ a, size_t n, double *out) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) s += a[k * n + i];
    if (s == 12345.678) out[0] = s;
}

// scattered patterns of the river kernel: a bijective odd-multiplier hash of the lane index picks the target, so
// every record / word is read exactly once and consecutive lanes land far apart (no coalescing, no reuse)
__device__ __forceinline__ size_t scat(size_t i, size_t n) { return (i * 0x9E3779B1ull) & (n - 1); }   // n: power of 2
__global__ void rd_rec64_scat(const double2 *__restrict__ a, size_t nrec, double *out) {   // 4 x 16 B, one 64-B record
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    const double2 *q = a + 4 * scat(i, nrec);
    const double2 x = q[0], y = q[1], z = q[2], w = q[3];
    const double s = x.x + x.y + y.x + y.y + z.x + z.y + w.x + w.y;
    if (s == 12345.678) out[0] = s;
}
__global__ void rd_rec64_seq(const double2 *__restrict__ a, size_t nrec, double *out) {    // lane r: record r
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    const double2 *q = a + 4 * i;
    const double2 x = q[0], y = q[1], z = q[2], w = q[3];
    const double s = x.x + x.y + y.x + y.y + z.x + z.y + w.x + w.y;
    if (s == 12345.678) out[0] = s;
}
__global__ void rd_16_scat(const double2 *__restrict__ a, size_t n2, double *out) {       // one random 16-B pair
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n2) return;
    const double2 v = a[scat(i, n2)];
    if (v.x + v.y == 12345.678) out[0] = v.x;
}
__global__ void rd_8_scat(const double *__restrict__ a, size_t n, double *out) {          // one random 8-B word
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = a[scat(i, n)];
    if (v == 12345.678) out[0] = v;
}

int main() {
    const size_t bytes = 2ull << 30;            // 2 GiB: far beyond the 256 MiB Infinity Cache
    double *a, *o;
    (void)hipMalloc(&a, bytes);
    (void)hipMalloc(&o, 64);
    (void)hipMemset(a, 0, bytes);
    (void)hipDeviceSynchronize();
    const size_t n = bytes / 8;
    for (int rep = 0; rep < 2; rep++) {
        rd_x2<<<2048, 256>>>(a, n, o);
        rd_x4<<<2048, 256>>>((const double2 *)a, n / 2, o);
        rd_x1<<<2048, 256>>>((const int *)a, bytes / 4, o);
        wr_x2<<<2048, 256>>>(a, n);
        rd_soa12<<<(n / 12 + 255) / 256, 256>>>(a, n / 12, o);
        rd_rec64_scat<<<(bytes / 64 + 255) / 256, 256>>>((const double2 *)a, bytes / 64, o);
        rd_rec64_seq<<<(bytes / 64 + 255) / 256, 256>>>((const double2 *)a, bytes / 64, o);
        rd_16_scat<<<(bytes / 16 + 255) / 256, 256>>>((const double2 *)a, bytes / 16, o);
        rd_8_scat<<<(bytes / 8 + 255) / 256, 256>>>(a, bytes / 8, o);
    }
    (void)hipDeviceSynchronize();
    printf("bytes per kernel: %zu (rd_soa12: %zu; the scattered kernels read every byte once)\n", bytes,
           (n / 12) * 12 * 8);
    return 0;
}
