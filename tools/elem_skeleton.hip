// tools/elem_skeleton.hip — the element kernel's memory traffic without its physics: what the access pattern alone
// costs on this box, for the production layout (16 separate element streams) and for record layouts that merge the
// static and per-step streams into one line per element.  Timing only (not part of the product).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/elem_skeleton tools/elem_skeleton.hip
// usage: tools/elem_skeleton [NE]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef double v2d __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ v2d ldnt(const v2d *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ int tile_of(int per8) { return (int)(blockIdx.x & 7) * per8 + (int)(blockIdx.x >> 3); }

// neighbours of a jittered-grid triangle strip: left / right in the row, and the row above or below
__device__ __forceinline__ int nbr(int i, int j, int ne, int row) {
    int n = j == 0 ? i - 1 : j == 1 ? i + 1 : ((i & 1) ? i + row : i - row);
    return (n < 0 || n >= ne) ? -1 : n;
}

// production layout: meta, zz, 3 y blocks, snp, stl, csv, sfl, area, ged[3][NE]; writes cs, 3 dy blocks
struct Prod {
    const v4i *meta; const v2d *zz; const double *y; const v2d *snp, *stl, *csv; const int *sfl; const double *area;
    const v2d *ged; v2d *cs; double *dy;
};
__global__ void __launch_bounds__(256, 5) k_prod(Prod P, int ne, int row, int per8) {
    const int i = tile_of(per8) * 256 + (int)threadIdx.x;
    if (i >= ne) return;
    const v4i mt = P.meta[i];
    const v2d zz = P.zz[i];
    const double ys = P.y[i], yu = P.y[ne + i], yg = P.y[2 * (size_t)ne + i];
    const v2d snp = ldnt(P.snp + i), stl = ldnt(P.stl + i), csv = ldnt(P.csv + i);
    const int sfl = P.sfl[i];
    const double area = __builtin_nontemporal_load(P.area + i);
    double acc = zz.x + zz.y + ys + yu + yg + snp.x + snp.y + stl.x + stl.y + csv.x + csv.y + sfl + mt.w;
    for (int j = 0; j < 3; j++) {
        const int nb = nbr(i, j, ne, row);
        const int nc = nb >= 0 ? nb : i;
        const v2d g = ldnt(P.ged + (size_t)j * ne + i);
        const v2d nz = P.zz[nc];
        const int ncf = ((const int *)(P.meta + nc))[3];
        acc += g.x * g.y + nz.x + nz.y + ncf + P.y[nc] + P.y[2 * (size_t)ne + nc];
    }
    v2d o; o.x = acc; o.y = area;
    __builtin_nontemporal_store(o, P.cs + i);
    __builtin_nontemporal_store(acc * 2., P.dy + i);
    __builtin_nontemporal_store(acc * 3., P.dy + ne + i);
    __builtin_nontemporal_store(acc * 4., P.dy + 2 * (size_t)ne + i);
}

// the production skeleton plus synthetic fp64 VALU work (NV dependent FMAs in 4 independent chains: ~60 % after
// the own record, the rest spread over the edge iterations) — how much VALU the access pattern hides
__device__ __forceinline__ void burn(double (&c)[4], int n) {
    for (int k = 0; k < n; k++) {
#pragma unroll
        for (int t = 0; t < 4; t++) c[t] = __builtin_fma(c[t], 1.0000001, 1e-9);
    }
}
__global__ void __launch_bounds__(256, 5) k_prod_v(Prod P, int ne, int row, int per8, int nv) {
    extern __shared__ double pad[];
    const int i = tile_of(per8) * 256 + (int)threadIdx.x;
    if (i >= ne) return;
    const v4i mt = P.meta[i];
    const v2d zz = P.zz[i];
    const double ys = P.y[i], yu = P.y[ne + i], yg = P.y[2 * (size_t)ne + i];
    const v2d snp = ldnt(P.snp + i), stl = ldnt(P.stl + i), csv = ldnt(P.csv + i);
    const int sfl = P.sfl[i];
    const double area = __builtin_nontemporal_load(P.area + i);
    double c[4] = {zz.x + ys, zz.y + yu, yg + snp.x + snp.y, stl.x + stl.y + csv.x + csv.y + sfl + mt.w};
    burn(c, (nv * 3 / 5) / 4);
    double acc = c[0] + c[1] + c[2] + c[3];
    for (int j = 0; j < 3; j++) {
        const int nb = nbr(i, j, ne, row);
        const int nc = nb >= 0 ? nb : i;
        const v2d g = ldnt(P.ged + (size_t)j * ne + i);
        const v2d nz = P.zz[nc];
        const int ncf = ((const int *)(P.meta + nc))[3];
        double d[4] = {g.x * g.y + acc, nz.x + nz.y, ncf + P.y[nc], P.y[2 * (size_t)ne + nc]};
        burn(d, (nv * 2 / 15) / 4);
        acc += d[0] + d[1] + d[2] + d[3];
    }
    if (acc == 1234.5) pad[threadIdx.x] = acc;
    v2d o; o.x = acc; o.y = area;
    __builtin_nontemporal_store(o, P.cs + i);
    __builtin_nontemporal_store(acc * 2., P.dy + i);
    __builtin_nontemporal_store(acc * 3., P.dy + ne + i);
    __builtin_nontemporal_store(acc * 4., P.dy + 2 * (size_t)ne + i);
}

// two tiles per workgroup: the second tile's own streams are loaded while the first tile computes (software
// prefetch into registers) — does a wave that always has loads in flight fix the few-rounds case?
struct Own { v4i mt; v2d zz, snp, stl, csv; double ys, yu, yg, area; int sfl; };
__device__ __forceinline__ Own own_load(const Prod &P, int ne, int i) {
    Own o;
    o.mt = P.meta[i]; o.zz = P.zz[i];
    o.ys = P.y[i]; o.yu = P.y[ne + i]; o.yg = P.y[2 * (size_t)ne + i];
    o.snp = ldnt(P.snp + i); o.stl = ldnt(P.stl + i); o.csv = ldnt(P.csv + i);
    o.sfl = P.sfl[i]; o.area = __builtin_nontemporal_load(P.area + i);
    return o;
}
__device__ __forceinline__ void own_body(const Prod &P, int ne, int row, int i, const Own &o, int nv) {
    double c[4] = {o.zz.x + o.ys, o.zz.y + o.yu, o.yg + o.snp.x + o.snp.y,
                   o.stl.x + o.stl.y + o.csv.x + o.csv.y + o.sfl + o.mt.w};
    burn(c, (nv * 3 / 5) / 4);
    double acc = c[0] + c[1] + c[2] + c[3];
    for (int j = 0; j < 3; j++) {
        const int nb = nbr(i, j, ne, row);
        const int nc = nb >= 0 ? nb : i;
        const v2d g = ldnt(P.ged + (size_t)j * ne + i);
        const v2d nz = P.zz[nc];
        const int ncf = ((const int *)(P.meta + nc))[3];
        double d[4] = {g.x * g.y + acc, nz.x + nz.y, ncf + P.y[nc], P.y[2 * (size_t)ne + nc]};
        burn(d, (nv * 2 / 15) / 4);
        acc += d[0] + d[1] + d[2] + d[3];
    }
    v2d ov; ov.x = acc; ov.y = o.area;
    __builtin_nontemporal_store(ov, P.cs + i);
    __builtin_nontemporal_store(acc * 2., P.dy + i);
    __builtin_nontemporal_store(acc * 3., P.dy + ne + i);
    __builtin_nontemporal_store(acc * 4., P.dy + 2 * (size_t)ne + i);
}
__global__ void __launch_bounds__(256, 4) k_prod_2t(Prod P, int ne, int row, int per8, int nv, int half) {
    extern __shared__ double pad[];
    const int t0 = tile_of(per8);
    const int ia = t0 * 256 + (int)threadIdx.x, ib = (t0 + half) * 256 + (int)threadIdx.x;
    Own a, b;
    if (ia < ne) a = own_load(P, ne, ia);
    if (ib < ne) b = own_load(P, ne, ib);
    if (ia < ne) own_body(P, ne, row, ia, a, nv);
    if (ib < ne) own_body(P, ne, row, ib, b, nv);
    if (nv == -1) pad[threadIdx.x] = 0.;
}

// record layout: one 128-B line per element {meta | zz | snp | stl | ged0 | ged1 | ged2 | area, sfl, pad}; y and dy
// stay the ABI's blocks, the carried state its ping-pong pair
struct Rec {
    const v2d *rec; const double *y; const v2d *csv; v2d *cs; double *dy;
};
__global__ void __launch_bounds__(256, 5) k_rec(Rec P, int ne, int row, int per8) {
    const int i = tile_of(per8) * 256 + (int)threadIdx.x;
    if (i >= ne) return;
    const v2d *r = P.rec + 8 * (size_t)i;
    const v2d m0 = r[0], zz = r[1], snp = ldnt(r + 2), stl = ldnt(r + 3), tail = r[7];
    const double ys = P.y[i], yu = P.y[ne + i], yg = P.y[2 * (size_t)ne + i];
    const v2d csv = ldnt(P.csv + i);
    const v4i mt = __builtin_bit_cast(v4i, m0);
    double acc = zz.x + zz.y + ys + yu + yg + snp.x + snp.y + stl.x + stl.y + csv.x + csv.y + tail.y + mt.w;
    for (int j = 0; j < 3; j++) {
        const int nb = nbr(i, j, ne, row);
        const int nc = nb >= 0 ? nb : i;
        const v2d g = r[4 + j];
        const v2d *rn = P.rec + 8 * (size_t)nc;
        const v2d nm = rn[0], nz = rn[1];
        const int ncf = __builtin_bit_cast(v4i, nm).w;
        acc += g.x * g.y + nz.x + nz.y + ncf + P.y[nc] + P.y[2 * (size_t)ne + nc];
    }
    v2d o; o.x = acc; o.y = tail.x;
    __builtin_nontemporal_store(o, P.cs + i);
    __builtin_nontemporal_store(acc * 2., P.dy + i);
    __builtin_nontemporal_store(acc * 3., P.dy + ne + i);
    __builtin_nontemporal_store(acc * 4., P.dy + 2 * (size_t)ne + i);
}

template <class F>
static double timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 5; i++) f();
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; i++) f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int ne = argc > 1 ? atoi(argv[1]) : 10001406;
    const int row = 4472;
    void *buf;
    const size_t per = 16 + 16 + 24 + 16 + 16 + 16 + 4 + 8 + 48 + 16 + 24 + 128 + 16;
    CK(hipMalloc(&buf, per * (size_t)ne + (1 << 20)));
    CK(hipMemset(buf, 0, per * (size_t)ne + (1 << 20)));
    char *b = (char *)buf;
    auto take = [&](size_t bytes) { char *p = b; b += (bytes + 255) & ~(size_t)255; return p; };
    Prod P;
    P.meta = (const v4i *)take(16ull * ne); P.zz = (const v2d *)take(16ull * ne); P.y = (const double *)take(24ull * ne);
    P.snp = (const v2d *)take(16ull * ne); P.stl = (const v2d *)take(16ull * ne); P.csv = (const v2d *)take(16ull * ne);
    P.sfl = (const int *)take(4ull * ne); P.area = (const double *)take(8ull * ne); P.ged = (const v2d *)take(48ull * ne);
    P.cs = (v2d *)take(16ull * ne); P.dy = (double *)take(24ull * ne);
    Rec R;
    R.rec = (const v2d *)take(128ull * ne); R.y = P.y; R.csv = P.csv; R.cs = P.cs; R.dy = P.dy;
    const int nb = ((ne + 255) / 256 + 7) / 8 * 8;
    const double tp = timeit([&] { hipLaunchKernelGGL(k_prod, dim3(nb), dim3(256), 0, 0, P, ne, row, nb / 8); }, 50);
    const double tr = timeit([&] { hipLaunchKernelGGL(k_rec, dim3(nb), dim3(256), 0, 0, R, ne, row, nb / 8); }, 50);
    const double bp = (double)ne * (164 + 40), br = (double)ne * (168 + 40);
    // synthetic VALU per element nv (the element kernel issues ~1,380 VALU per wave = per element), LDS padding to
    // hold 6 (lds 26 KiB) or 5 workgroups per CU like the element kernel
    {   // two tiles per workgroup (half the grid), loads of the second tile in flight during the first
        const int ntile = (ne + 255) / 256, half = (ntile + 1) / 2;
        const int nb2 = (half + 7) / 8 * 8;
        for (int nv : {0, 1200, 1600}) {
            const double tv = timeit([&] { hipLaunchKernelGGL(k_prod_2t, dim3(nb2), dim3(256), 0, 0, P, ne, row, nb2 / 8, nv, half); }, 30);
            printf("{\"num_ele\": %d, \"two_tiles\": 1, \"valu_per_element\": %d, \"ms\": %.4f}\n", ne, nv, tv);
        }
    }
    for (int lds : {0, 26 * 1024}) {
        for (int nv : {0, 400, 800, 1200, 1600}) {
            const double tv = timeit([&] { hipLaunchKernelGGL(k_prod_v, dim3(nb), dim3(256), lds, 0, P, ne, row, nb / 8, nv); }, 30);
            printf("{\"num_ele\": %d, \"lds\": %d, \"valu_per_element\": %d, \"ms\": %.4f}\n", ne, lds, nv, tv);
        }
    }
    printf("{\"num_ele\": %d, \"prod_ms\": %.4f, \"prod_GBs_unique\": %.0f, \"rec_ms\": %.4f, \"rec_GBs_unique\": %.0f}\n", ne,
           tp, bp / tp / 1e6, tr, br / tr / 1e6);
    return 0;
}
