// shud_stream.hip — STREAM-copy probe of the practical HBM ceiling (bench.py reports it beside the
// roofline peak).  Not part of the RHS C-ABI: a separate libshud_stream.so.
#include <hip/hip_runtime.h>
#include <stddef.h>

typedef double v2d __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) stream_copy_kernel(const v2d *__restrict__ src, v2d *__restrict__ dst,
                                                          size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}

extern "C" int shud_stream_copy(const void *src, void *dst, size_t bytes, void *stream) {
    const size_t n = bytes / sizeof(v2d);
    if (!n) return 0;
    const int grid = 256 * 32;            // 32 workgroups per CU, grid-stride over 16-B records
    hipLaunchKernelGGL(stream_copy_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const v2d *)src,
                       (v2d *)dst, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
