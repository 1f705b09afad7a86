// Workgroups of 256 threads per CU that the runtime admits for a given dynamic LDS size (gfx950 LDS allocation
// granularity probe): prints "bytes blocks" rows.  hipcc --offload-arch=gfx950 -O2 tools/lds_occ.hip -o tools/lds_occ
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(256) k_dummy(double *p) {
    extern __shared__ double s[];
    s[threadIdx.x] = p[threadIdx.x];
    __syncthreads();
    p[threadIdx.x] = s[255 - threadIdx.x];
}
int main() {
    const int sizes[] = {16384, 20480, 22528, 23000, 23008, 23040, 23100, 23296, 23406, 23424, 23552, 24576, 27306, 32768};
    for (int b : sizes) {
        int n = -1;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void *)k_dummy, 256, b);
        printf("%d %d\n", b, n);
    }
    return 0;
}
