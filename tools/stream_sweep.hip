// tools/stream_sweep.hip — sweep of STREAM-copy / read kernels to find this box's practical HBM ceiling
// (bench.py's stream_probe reports the best configuration of libshud_stream.so).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/stream_sweep tools/stream_sweep.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef double v2d __attribute__((ext_vector_type(2)));

template <int U, bool NTL, bool NTS>
__global__ void copy_k(const v2d *__restrict__ s, v2d *__restrict__ d, size_t n) {
    const size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x;
    v2d v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * blockDim.x;
        if (i < n) v[u] = NTL ? __builtin_nontemporal_load(&s[i]) : s[i];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * blockDim.x;
        if (i < n) {
            if (NTS) __builtin_nontemporal_store(v[u], &d[i]);
            else d[i] = v[u];
        }
    }
}

template <int U, bool NTL>
__global__ void read_k(const v2d *__restrict__ s, double *sink, size_t n) {
    const size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x;
    double acc = 0.;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * blockDim.x;
        if (i < n) {
            const v2d v = NTL ? __builtin_nontemporal_load(&s[i]) : s[i];
            acc += v.x + v.y;
        }
    }
    if (acc == 12345.678) sink[threadIdx.x] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1); } } while (0)

template <class F>
static double timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) f();
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; i++) f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

template <int U, bool NTL, bool NTS>
static void run_copy(const v2d *s, v2d *d, size_t n, int blk) {
    const size_t nb = (n + (size_t)blk * U - 1) / ((size_t)blk * U);
    const double ms = timeit([&] { hipLaunchKernelGGL((copy_k<U, NTL, NTS>), dim3(nb), dim3(blk), 0, 0, s, d, n); }, 20);
    printf("copy U=%d blk=%4d ntl=%d nts=%d bytes=%zu  %.1f GB/s\n", U, blk, NTL, NTS, n * 16, 2.0 * n * 16 / ms / 1e6);
}
template <int U, bool NTL>
static void run_read(const v2d *s, double *k, size_t n, int blk) {
    const size_t nb = (n + (size_t)blk * U - 1) / ((size_t)blk * U);
    const double ms = timeit([&] { hipLaunchKernelGGL((read_k<U, NTL>), dim3(nb), dim3(blk), 0, 0, s, k, n); }, 20);
    printf("read U=%d blk=%4d ntl=%d bytes=%zu  %.1f GB/s\n", U, blk, NTL, n * 16, 1.0 * n * 16 / ms / 1e6);
}

int main() {
    for (size_t gib : {1, 4}) {
        const size_t n = (gib << 30) / 16;
        v2d *s, *d;
        CK(hipMalloc(&s, n * 16));
        CK(hipMalloc(&d, n * 16));
        CK(hipMemset(s, 0, n * 16));
        CK(hipMemset(d, 0, n * 16));
        for (int blk : {256, 512, 1024}) {
            run_copy<1, false, false>(s, d, n, blk);
            run_copy<2, false, false>(s, d, n, blk);
            run_copy<4, false, false>(s, d, n, blk);
            run_copy<8, false, false>(s, d, n, blk);
            run_copy<4, true, false>(s, d, n, blk);
            run_copy<4, false, true>(s, d, n, blk);
            run_copy<4, true, true>(s, d, n, blk);
            run_copy<8, false, true>(s, d, n, blk);
            run_copy<2, false, true>(s, d, n, blk);
            run_copy<1, false, true>(s, d, n, blk);
            run_read<4, false>(s, (double *)d, n, blk);
            run_read<8, false>(s, (double *)d, n, blk);
            run_read<4, true>(s, (double *)d, n, blk);
        }
        const double ms = timeit([&] { CK(hipMemcpyAsync(d, s, n * 16, hipMemcpyDeviceToDevice, 0)); }, 20);
        printf("hipMemcpy D2D bytes=%zu  %.1f GB/s\n", n * 16, 2.0 * n * 16 / ms / 1e6);
        CK(hipFree(s));
        CK(hipFree(d));
    }
    return 0;
}
