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
