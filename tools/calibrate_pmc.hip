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

int main() {
    const size_t bytes = 2ull << 30;            // 2 GiB: far beyond the 256 MiB Infinity Cache
    double *a, *o;
    hipMalloc(&a, bytes);
    hipMalloc(&o, 64);
    hipMemset(a, 0, bytes);
    hipDeviceSynchronize();
    const size_t n = bytes / 8;
    for (int rep = 0; rep < 2; rep++) {
        rd_x2<<<2048, 256>>>(a, n, o);
        rd_x4<<<2048, 256>>>((const double2 *)a, n / 2, o);
        rd_x1<<<2048, 256>>>((const int *)a, bytes / 4, o);
        wr_x2<<<2048, 256>>>(a, n);
        rd_soa12<<<(n / 12 + 255) / 256, 256>>>(a, n / 12, o);
    }
    hipDeviceSynchronize();
    printf("bytes per kernel: %zu (rd_soa12: %zu)\n", bytes, (n / 12) * 12 * 8);
    return 0;
}
