// tools/ode_red_bench.hip — measurement only: variants of the integrator's five-operand reduction pass
// (k_atimes shape: read ewt, w, fy, V, V0; write w; two sums) on NY = 31M fp64 entries (syn-10M's state), to
// find the streaming form that gets closest to the box's copy ceiling.  Every variant computes the same
// per-entry values; the sums differ only in order (not compared).  Build: hipcc --offload-arch=gfx950 -O3.
// usage: ode_red_bench [n] [reps]   -> one line per variant: us per pass, GB/s (48 B/entry)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int T = 256;
typedef double v2d __attribute__((ext_vector_type(2)));

__device__ inline void block_sum2(double a, double b, double *part, int nblk_stride) {
    __shared__ double sm[2][T / 64];
    for (int off = 32; off >= 1; off >>= 1) { a += __shfl_xor(a, off, 64); b += __shfl_xor(b, off, 64); }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { sm[0][w] = a; sm[1][w] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s0 = sm[0][0], s1 = sm[1][0];
        for (int k = 1; k < T / 64; ++k) { s0 += sm[0][k]; s1 += sm[1][k]; }
        part[blockIdx.x] = s0;
        part[nblk_stride + blockIdx.x] = s1;
    }
}

__device__ inline double op(double e, double w, double f, double v, double ng, double siginv, double &z) {
    const double jv = siginv * (w - f);
    z = e * (ng * jv + v / e);
    return z;
}

// A: grid-stride, fixed grid (production form)
template <bool NT>
__global__ void __launch_bounds__(T) kA(int64_t n, double *w, const double *fy, const double *V, const double *ewt,
                                        const double *V0, double *part, int ps) {
    double a = 0, b = 0;
    const int64_t st = (int64_t)gridDim.x * T;
    for (int64_t i = (int64_t)blockIdx.x * T + threadIdx.x; i < n; i += st) {
        double e, ww, f, v, v0;
        if (NT) { e = __builtin_nontemporal_load(ewt + i); ww = __builtin_nontemporal_load(w + i);
                  f = __builtin_nontemporal_load(fy + i); v = __builtin_nontemporal_load(V + i);
                  v0 = __builtin_nontemporal_load(V0 + i); }
        else { e = ewt[i]; ww = w[i]; f = fy[i]; v = V[i]; v0 = V0[i]; }
        double x;
        op(e, ww, f, v, -0.5, 2.0, x);
        if (NT) __builtin_nontemporal_store(x, w + i); else w[i] = x;
        a += x * x;
        b += v0 * x;
    }
    block_sum2(a, b, part, ps);
}

// B: one entry per thread, full grid (block partials: n/256 of them)
__global__ void __launch_bounds__(T) kB(int64_t n, double *w, const double *fy, const double *V, const double *ewt,
                                        const double *V0, double *part, int ps) {
    double a = 0, b = 0;
    const int64_t i = (int64_t)blockIdx.x * T + threadIdx.x;
    if (i < n) {
        const double e = ewt[i], ww = w[i], f = fy[i], v = V[i], v0 = V0[i];
        double x;
        op(e, ww, f, v, -0.5, 2.0, x);
        w[i] = x;
        a = x * x;
        b = v0 * x;
    }
    block_sum2(a, b, part, ps);
}

// C: K consecutive tiles of 256 per block (one-shot, K loads per stream in flight per thread)
template <int K>
__global__ void __launch_bounds__(T) kC(int64_t n, double *w, const double *fy, const double *V, const double *ewt,
                                        const double *V0, double *part, int ps) {
    double a = 0, b = 0;
    const int64_t base = (int64_t)blockIdx.x * T * K + threadIdx.x;
    double e[K], ww[K], f[K], v[K], v0[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t i = base + k * T;
        const bool ok = i < n;
        e[k] = ok ? ewt[i] : 1.0; ww[k] = ok ? w[i] : 0.0; f[k] = ok ? fy[i] : 0.0; v[k] = ok ? V[i] : 0.0;
        v0[k] = ok ? V0[i] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t i = base + k * T;
        double x;
        op(e[k], ww[k], f[k], v[k], -0.5, 2.0, x);
        if (i < n) { w[i] = x; a += x * x; b += v0[k] * x; }
    }
    block_sum2(a, b, part, ps);
}

// D: grid-stride with 16-B loads (2 consecutive entries per thread per iteration)
__global__ void __launch_bounds__(T) kD(int64_t n, double *w, const double *fy, const double *V, const double *ewt,
                                        const double *V0, double *part, int ps) {
    double a = 0, b = 0;
    const int64_t n2 = n / 2;
    const int64_t st = (int64_t)gridDim.x * T;
    for (int64_t j = (int64_t)blockIdx.x * T + threadIdx.x; j < n2; j += st) {
        const v2d e = ((const v2d *)ewt)[j], ww = ((const v2d *)w)[j], f = ((const v2d *)fy)[j],
                  v = ((const v2d *)V)[j], v0 = ((const v2d *)V0)[j];
        double x0, x1;
        op(e.x, ww.x, f.x, v.x, -0.5, 2.0, x0);
        op(e.y, ww.y, f.y, v.y, -0.5, 2.0, x1);
        v2d x;
        x.x = x0;
        x.y = x1;
        ((v2d *)w)[j] = x;
        a += x.x * x.x; a += x.y * x.y;
        b += v0.x * x.x; b += v0.y * x.y;
    }
    block_sum2(a, b, part, ps);
}

// finalize over nb partials (one block)
__global__ void kFin(const double *part, int nb, int ps, double *out) {
    __shared__ double sm[T / 64];
    for (int q = 0; q < 2; ++q) {
        double x = 0;
        for (int k = threadIdx.x; k < nb; k += T) x += part[q * ps + k];
        for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
        if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = x;
        __syncthreads();
        if (threadIdx.x == 0) out[q] = sm[0] + sm[1] + sm[2] + sm[3];
        __syncthreads();
    }
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 31000000;
    const int reps = argc > 2 ? atoi(argv[2]) : 30;
    double *buf[5], *part, *out;
    for (auto &b : buf) { CK(hipMalloc(&b, n * sizeof(double))); }
    const int ps = (int)((n + T - 1) / T) + 16;
    CK(hipMalloc(&part, 2 * (size_t)ps * sizeof(double)));
    CK(hipMalloc(&out, 16));
    std::vector<double> h(n);
    for (int k = 0; k < 5; ++k) {
        for (int64_t i = 0; i < n; ++i) h[i] = 1.0 + 1e-3 * ((i * 7 + k) % 1000);
        CK(hipMemcpy(buf[k], h.data(), n * sizeof(double), hipMemcpyHostToDevice));
    }
    double *ewt = buf[0], *w = buf[1], *fy = buf[2], *V = buf[3], *V0 = buf[4];
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto launch) {
        for (int r = 0; r < 3; ++r) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        printf("%-36s %8.1f us  %7.0f GB/s (48 B/entry)\n", name, us, 48.0 * n / (us * 1e-6) / 1e9);
        fflush(stdout);
    };
    const int nbB = (int)((n + T - 1) / T);
    timeit("A grid-stride 2048 blk (prod)", [&] { kA<false><<<2048, T>>>(n, w, fy, V, ewt, V0, part, ps); kFin<<<1, T>>>(part, 2048, ps, out); });
    timeit("A grid-stride 2048 blk + nt", [&] { kA<true><<<2048, T>>>(n, w, fy, V, ewt, V0, part, ps); kFin<<<1, T>>>(part, 2048, ps, out); });
    timeit("A grid-stride 4096 blk", [&] { kA<false><<<4096, T>>>(n, w, fy, V, ewt, V0, part, ps); kFin<<<1, T>>>(part, 4096, ps, out); });
    timeit("A grid-stride 1024 blk", [&] { kA<false><<<1024, T>>>(n, w, fy, V, ewt, V0, part, ps); kFin<<<1, T>>>(part, 1024, ps, out); });
    timeit("B one entry/thread + fin(n/256)", [&] { kB<<<nbB, T>>>(n, w, fy, V, ewt, V0, part, ps); kFin<<<1, T>>>(part, nbB, ps, out); });
    timeit("B kernel only", [&] { kB<<<nbB, T>>>(n, w, fy, V, ewt, V0, part, ps); });
    const int nb4 = (int)((n + 4 * T - 1) / (4 * T)), nb8 = (int)((n + 8 * T - 1) / (8 * T)), nb16 = (int)((n + 16 * T - 1) / (16 * T));
    timeit("C K=4 tiles/blk + fin", [&] { kC<4><<<nb4, T>>>(n, w, fy, V, ewt, V0, part, ps); kFin<<<1, T>>>(part, nb4, ps, out); });
    timeit("C K=8 tiles/blk + fin", [&] { kC<8><<<nb8, T>>>(n, w, fy, V, ewt, V0, part, ps); kFin<<<1, T>>>(part, nb8, ps, out); });
    timeit("C K=16 tiles/blk + fin", [&] { kC<16><<<nb16, T>>>(n, w, fy, V, ewt, V0, part, ps); kFin<<<1, T>>>(part, nb16, ps, out); });
    timeit("D grid-stride 16-B 2048 blk", [&] { kD<<<2048, T>>>(n, w, fy, V, ewt, V0, part, ps); kFin<<<1, T>>>(part, 2048, ps, out); });
    timeit("fin(2048) alone", [&] { kFin<<<1, T>>>(part, 2048, ps, out); });
    timeit("fin(n/256) alone", [&] { kFin<<<1, T>>>(part, nbB, ps, out); });
    timeit("fin(n/4096) alone", [&] { kFin<<<1, T>>>(part, nb16, ps, out); });
    return 0;
}
