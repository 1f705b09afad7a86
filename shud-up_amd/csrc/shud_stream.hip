// shud_stream.hip — STREAM probes of the practical HBM ceiling (bench.py reports it beside the roofline
// peak).  Not part of the RHS C-ABI: a separate libshud_stream.so.
//
// Variants (shud_stream_copy's `variant`):
//   0  grid-stride copy, 16-B non-temporal loads/stores, 32 workgroups per CU
//   1  one-shot copy, every lane moves UNROLL=4 16-B records spaced one workgroup apart (no grid-stride
//      loop), non-temporal loads and stores: the fastest copy of tools/stream_sweep.hip on MI355X
//   2  one-shot copy, one 16-B record per lane, plain loads, non-temporal stores
//   3  one-shot read-only sweep (16-B non-temporal loads, 512-lane workgroups, a per-lane xor kept live by one
//      conditional store): the read-side ceiling, which is what a read-dominated kernel such as the element
//      kernel meets
// and a pure fp64-VALU probe (shud_valu_probe): what the box's vector ALUs sustain and the clock they hold under a
// dense fp64 load, so a bench line can say what kind of box it ran on (the element kernel's VALU issue floor is
// ~0.67 of its cycles: its time follows the clock as well as the HBM rate).
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

typedef double v2d __attribute__((ext_vector_type(2)));
typedef unsigned long long v2u __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) stream_copy_gs(const v2d *__restrict__ src, v2d *__restrict__ dst,
                                                      size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}

constexpr int UNROLL = 4;

// block b covers records [b*256*UNROLL, (b+1)*256*UNROLL); lane t of iteration u reads record
// base + u*256 + t, so each wave-instruction is one contiguous 1 KiB
template <int U, bool NT_LD>
__global__ void __launch_bounds__(256) stream_copy_1shot(const v2d *__restrict__ src, v2d *__restrict__ dst,
                                                         size_t n) {
    const size_t base = (size_t)blockIdx.x * (256 * U) + threadIdx.x;
    v2d v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) v[u] = NT_LD ? __builtin_nontemporal_load(&src[i]) : src[i];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * 256;
        if (i < n) __builtin_nontemporal_store(v[u], &dst[i]);
    }
}

__global__ void __launch_bounds__(512) stream_read_1shot(const v2u *__restrict__ src, unsigned long long *sink,
                                                         size_t n) {
    const size_t base = (size_t)blockIdx.x * (512 * UNROLL) + threadIdx.x;
    unsigned long long acc = 0;
    v2u v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
        const size_t i = base + (size_t)u * 512;
        v[u] = i < n ? __builtin_nontemporal_load(&src[i]) : (v2u){0ull, 0ull};
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) acc ^= v[u].x ^ v[u].y;
    if (acc == 0x5a5a5a5a5a5a5a5aull) sink[threadIdx.x] = acc;     // practically never taken
}

extern "C" int shud_stream_copy_v(const void *src, void *dst, size_t bytes, void *stream, int variant) {
    const size_t n = bytes / sizeof(v2d);
    if (!n) return 0;
    hipStream_t s = (hipStream_t)stream;
    const unsigned nb = (unsigned)((n + 256 * UNROLL - 1) / (256 * UNROLL));
    const unsigned nb1 = (unsigned)((n + 255) / 256);
    const unsigned nbr = (unsigned)((n + 512 * UNROLL - 1) / (512 * UNROLL));
    switch (variant) {
    case 0:
        hipLaunchKernelGGL(stream_copy_gs, dim3(256 * 32), dim3(256), 0, s, (const v2d *)src, (v2d *)dst, n);
        break;
    case 1:
        hipLaunchKernelGGL((stream_copy_1shot<UNROLL, true>), dim3(nb), dim3(256), 0, s, (const v2d *)src, (v2d *)dst,
                           n);
        break;
    case 2:
        hipLaunchKernelGGL((stream_copy_1shot<1, false>), dim3(nb1), dim3(256), 0, s, (const v2d *)src, (v2d *)dst, n);
        break;
    case 3:
        hipLaunchKernelGGL(stream_read_1shot, dim3(nbr), dim3(512), 0, s, (const v2u *)src,
                           (unsigned long long *)dst, n);
        break;
    default:
        return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int shud_stream_copy(const void *src, void *dst, size_t bytes, void *stream) {
    return shud_stream_copy_v(src, dst, bytes, stream, 0);
}

// fp64 VALU probe: 8 independent fma chains per lane (a[k] = a[k] * m + c, bounded: the fixed point is c / (1 - m)),
// 2,048 workgroups of 256 lanes (8 waves per SIMD on 256 CUs), non-trivial operands (zero operands clock higher).
// Lane 0 of every workgroup stamps s_memtime (shader clock) and s_memrealtime (100 MHz constant clock) around its
// loop: the in-kernel clock is the ratio (MI355X_MICROARCH.md, DVFS give-back item 6).
__global__ void __launch_bounds__(256) valu_probe_kernel(int iters, double m, double c, double *sink,
                                                         unsigned long long *stamps) {
    double a[8];
    const double x0 = 0.5 + 1e-9 * (double)threadIdx.x + 1e-6 * (double)blockIdx.x;
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = x0 + 0.125 * k;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 16; u++)
#pragma unroll
            for (int k = 0; k < 8; k++) a[k] = __builtin_fma(a[k], m, c);
    }
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    double sum = 0.;
#pragma unroll
    for (int k = 0; k < 8; k++) sum += a[k];
    if (sum == 12345.678) sink[threadIdx.x] = sum;                  // keeps the chains live; never taken
}
// fp64 FMAs per launch = blocks x 256 x iters x 128; stamps: [2 * blocks] (shader cycles, 100 MHz ticks) per block
extern "C" int shud_valu_probe(int blocks, int iters, double *sink, unsigned long long *stamps, void *stream) {
    if (blocks <= 0 || iters <= 0) return -2;
    hipLaunchKernelGGL(valu_probe_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, iters, 0.9999999999, 1e-12,
                       sink, stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
