// shud_ele_packed.hip — production element kernel on the packed class layout (shud_dev.h DevPacked).
//
// Same physics, same fp64 operation order as shud_ele_kernel (shud_kernels.hip) — which restates
// f_etFlux (MD_ET.cpp:343-404), updateElement/Flux_Infiltration/Flux_Recharge (Element.cpp:271-384),
// fun_Ele_surface/fun_Ele_sub (MD_ElementFlux.cpp:35-156), fun_Seg_surface/fun_Seg_sub
// (MD_RiverFlux.cpp:100-126), PassValue's Qe2r sums (MD_f.cpp:228-235) and f_applyDY (MD_f.cpp:65-156).
// What differs is only how the operands reach the registers:
//   * loads are unconditional (neighbour indices clamped to the element itself on a boundary edge), so
//     they never queue behind branches; the element's own records are issued up front, each edge's
//     neighbour data at the top of its (rolled) iteration — at <= 96 VGPRs five waves per SIMD hide the
//     latency that three waves holding everything up front could not;
//   * errors/warnings are aggregated per wave (one atomic per wave, shud_physics.h report_w);
//   * the element's own streams arrive as 16-byte records (global_load_dwordx4), per-element hydraulic
//     parameters through a class id into a table that stays in L1/L2;
//   * single-use streams are loaded/stored non-temporally and workgroups are dealt to XCDs in
//     contiguous chunks so the neighbour rows an element block gathers are in its own XCD's L2.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "shud_dev.h"
#include "shud_physics.h"

namespace shud {

typedef double v2d __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
template <class T>
__device__ __forceinline__ T ldnt(const T *p) { return __builtin_nontemporal_load(p); }
// one 16-byte non-temporal load (global_load_dwordx4 nt)
__device__ __forceinline__ double2 ldnt2(const double2 *p) {
    const v2d v = __builtin_nontemporal_load((const v2d *)p);
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ int4 ldnt4(const int4 *p) {
    const v4i v = __builtin_nontemporal_load((const v4i *)p);
    return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stnt2(double2 *p, double a, double b) {
    v2d v;
    v.x = a;
    v.y = b;
    __builtin_nontemporal_store(v, (v2d *)p);
}
// element / segment streams are addressed as a wave-uniform base + a 32-bit byte offset, which the compiler
// emits as global_load/store v, vOff, s[base] (saddr form): one 32-bit shift per record size shared by every
// stream of that size, instead of a sign extension and a 64-bit address add per stream.  The handle keeps
// every such array below 4 GiB (build_packed: 48 B x NE and 16 B x NS).
template <class T>
__device__ __forceinline__ const T *at(const T *b, uint32_t off) { return (const T *)((const char *)b + off); }
template <class T>
__device__ __forceinline__ T *atw(T *b, uint32_t off) { return (T *)((char *)b + off); }

// IEEE class tests (one v_cmp_class_f64 each): NaN | +-inf, and NaN | +-inf | negative (not -0.0)
__device__ __forceinline__ bool nan_or_inf(double x) { return __builtin_isfpclass(x, 0x0003 | 0x0004 | 0x0200); }
__device__ __forceinline__ bool bad_nonneg(double x) {
    return __builtin_isfpclass(x, 0x0003 | 0x0004 | 0x0008 | 0x0010 | 0x0200);
}

// stage of an owned or ghost reach: the address is selected, so one load and no branch
__device__ __forceinline__ const double *riv_y_at(const YView &Y, int r) {
    return r < Y.n_own_riv ? Y.y + 3 * (size_t)Y.n_own + r : Y.griv + (r - Y.n_own_riv);
}

// packed cf word (DevPacked::meta.w)
__device__ __forceinline__ int cf_ibc(int cf) { return (int)(int8_t)(cf & 0xff); }
__device__ __forceinline__ int cf_iss(int cf) { return (cf >> 8) & 3; }
__device__ __forceinline__ int cf_nseg(int cf) { return (cf >> 10) & 63; }
__device__ __forceinline__ int cf_class(int cf) { return (int)(((unsigned)cf >> 16) & 0x7fffu); }   // bit 31: lake

// uYgw of element j (MD_update.cpp:114-125 / MD_f_omp.cpp:119-128)
template <int MODE>
__device__ __forceinline__ double ugw_pk(const DevMesh &m, double ygw_raw, int ibc, int j) {
    if (ibc == 0) return MODE == 0 ? ygw_raw : rmax(0.0, ygw_raw);
    if (ibc > 0) return m.eybc[ibc];
    return m.ugw_stale[j];
}

// class table staged in LDS (record-major [class][field]) when it has <= LDS_CLS_MAX classes: the 18 + 3x5
// class lookups per element become LDS reads with immediate offsets instead of dependent L2 trips
constexpr int LDS_CLS_MAX = kLdsClassMax;
constexpr int CF_LDS_STRIDE = CF_STRIDE;   // the HBM table's record layout, copied linearly into LDS

// LAKE: the model has lakes.  Lake elements (cf bit 31) follow updateLakeElement /
// fun_Ele_lakeVertical / fun_Ele_lakeHorizon (Element.cpp:336-346, MD_ElementFlux.cpp:2-23) and get zero DY
// (MD_f.cpp:146-150); bank edges of other elements exchange with the lake (MD_ElementFlux.cpp:46-53,107-121)
// and leave their fluxes in DevLake for the lake kernel.  LAKE = false compiles all of it away.
constexpr int kEleWaves = 5;      // min waves per SIMD: <= 96 VGPRs (rolled edge loop, no spills)
constexpr int kEleWavesSh = 7;    // the edge-sharing instantiations with the parked DY tail (kEleWavesOf)
// in-tile edge sharing (ele_body, SH): the ghost-free, lake-free, non-hybrid, non-diagnostic instantiations with the
// class table in LDS (the 256-thread ones; the 1024-thread table kernel passes BS = 1024)
constexpr bool kShareOn(bool lct, bool gh, bool lake, int hyb, bool diag) {
    return lct && !gh && !lake && hyb == 0 && !diag;
}
// min waves per SIMD of an instantiation: with sharing and the parked DY tail 7 (72 VGPRs, no spills with FU1; 6
// without FU1, where 7 would spill); the plain LDS-table one (36..~128 classes) 6 on closed boundaries (80 VGPRs, no
// spills; its unbounded allocation drifts between 80 and 86 with unrelated code), others 5
constexpr int kEleWavesOf(bool lct, int lspk, bool gh, bool lake, int hyb, bool diag, bool fu1, bool open) {
    return (kShareOn(lct, gh, lake, hyb, diag) && lspk) ? (fu1 ? kEleWavesSh : 6)
           : (kShareOn(lct, gh, lake, hyb, diag) && !open) ? 6 : kEleWaves;
}
constexpr int kEleBS = 256;       // elements per workgroup
static_assert(kEleBS == kShareTile, "edge sharing pairs elements within one workgroup's tile");
static_assert(2 * kEleBS <= kPowTabDoubles, "edge-sharing slots fit the pow tables' LDS region");
// an edge-sharing slot's "evaluate it yourself" mark: a signalling NaN, which no arithmetic result is
constexpr uint64_t kShareVoid = 0x7ff0000000000001ull;
// f_etFlux's three conditions (negative flux, NaN, eta > 2 ETP) are collected in a lane bit mask and reported together —
// one ballot per wave when none fired (the common case) instead of three; the same flags, first indices and warning
// count (atomics commute).  (Deferring all five conditions to the end of the body kept the mask live across the edge
// loop: 85 VGPRs, 5 waves/SIMD.)
// One 256-element tile per workgroup.  (Persistent workgroups — one per resident slot looping over XCD-chunked
// tiles, the class table copied to LDS once per workgroup — measured 0.735 vs 0.657 ms in round 3: the tile loop
// took the kernel to 96 VGPRs with spills, profiles/r03/ab_persist/.  Round 5 (a persistent kernel, commit a4b4e96):
// the spills were machine-LICM hoisting the polynomial constants out of the tile loop; with -mllvm -disable-machine-licm the loop
// fits 82 VGPRs without spills, bit-identical, and is still slower: 0.682 / 0.671 ms at 5 / 6 waves per SIMD vs
// 0.608 ms, profiles/r05/persist/.  Other workgroup sizes: 384 / 512 / 768 threads 0.672 / 0.615 / 0.666 ms,
// profiles/r05/ele_bs/.  In-tile neighbours from LDS — each lane staging {z_surf, z_bottom, isf, uYgw, effKH,
// roughness} after updateElement with a per-wave ready flag, edges to a same-tile neighbour reading them instead of
// four gathers, two class lookups and eff_kh — bit-identical and neutral (0.605 vs 0.599 ms, wall 0.582 vs 0.583);
// gathering the one out-of-tile neighbour before the loop took 94 VGPRs and was slower, profiles/r05/nb_lds/.  Two tiles
// per workgroup sharing one table copy: 83 VGPRs / 5 waves 0.628 ms, forced to 6 waves 0.606 vs 0.602 ms,
// profiles/r05/tiles2/.  Round-5 A/B switches that measured slower were removed in round 6; commit a4b4e96 holds them.)
// the element's own records, loaded before the workgroup's class-table barrier so both round trips overlap
struct OwnRec {
    int4 mt;
    double2 zz, snp, stl, fu, csv;
    double ysf, yus, ygw;
    int sfl;                                              // seg_first word (bit 31: LAI on)
};
template <bool FU1, bool GH>
__device__ __forceinline__ OwnRec load_own(const DevPacked &p, const YView &Y, int i, int cur) {
    const int nown = Y.n_own;
    const uint32_t o16 = (uint32_t)i << 4, o8 = (uint32_t)i << 3;
    OwnRec o;
    o.mt = *at(p.meta, o16);
    o.zz = *at(p.zz, o16);
    o.ysf = GH ? Y.sf(i) : *at(Y.y, o8);
    o.yus = GH ? Y.us(i) : *at(Y.y + nown, o8);
    o.ygw = GH ? Y.gw(i) : *at(Y.y + 2 * (size_t)nown, o8);
    o.snp = ldnt2(at(p.s_np, o16));
    o.stl = ldnt2(at(p.s_tl, o16));                       // {pot_tran, ETP}
    if (FU1) { o.fu.x = 1.0; o.fu.y = 1.0; } else o.fu = ldnt2(at(p.s_fu, o16));
    o.csv = ldnt2(at(p.cs[cur], o16));
    o.sfl = *at(p.seg_first, (uint32_t)i << 2);
    return o;
}

// class table global -> LDS by BS threads: the first kTabBatch loads of every thread are issued together (and
// before the caller's own-record loads, which they overlap), then stored; a longer table continues in a loop.
// (A load -> wait -> ds_write per iteration cost one L2 round trip per 256 table words at every workgroup start.)
// The copy runs in 16-B words (global_load_dwordx4 / ds_write_b128; the table is an even number of 16-B aligned
// words): half the load / LDS-write instructions of 8-B words for the same bytes — the per-workgroup copy is a
// measurable share of the kernel (10 KiB more of it cost 3 %, profiles/r05/pow_ab/abl_compact.log).
constexpr int kTabBatch = 8;                             // 8-B words per thread in the first batch
template <int BS>
__device__ __forceinline__ void tab_issue(const DevPacked &p, double (&tv)[kTabBatch]) {
    const int nt2 = (p.ntab + 1) >> 1;
#pragma unroll
    for (int k = 0; k < kTabBatch / 2; k++) {
        const int t = (int)threadIdx.x + k * BS;
        const double2 v = t < nt2 ? ((const double2 *)p.ctab)[t] : make_double2(0., 0.);
        tv[2 * k] = v.x;
        tv[2 * k + 1] = v.y;
    }
}
template <int BS>
__device__ __forceinline__ void tab_store(const DevPacked &p, const double (&tv)[kTabBatch], double *lct) {
    const int nt2 = (p.ntab + 1) >> 1;
#pragma unroll
    for (int k = 0; k < kTabBatch / 2; k++) {
        const int t = (int)threadIdx.x + k * BS;
        if (t < nt2) ((double2 *)lct)[t] = make_double2(tv[2 * k], tv[2 * k + 1]);
    }
    for (int t = (int)threadIdx.x + kTabBatch / 2 * BS; t < nt2; t += BS)
        ((double2 *)lct)[t] = ((const double2 *)p.ctab)[t];
}
// workgroup -> tile: XCD-contiguous chunks (block_id<1>, shud_physics.h) with the chunk length per8 = grid/8
// passed by the launcher, so no workgroup reads the grid size from the dispatch packet at its start
__device__ __forceinline__ int tile_of(int per8, int b) { return (b & 7) * per8 + (b >> 3); }
__device__ __forceinline__ int tile_of(int per8) { return tile_of(per8, (int)blockIdx.x); }

// QrivDown pre-pass (DevPacked::qdown): nb_q workgroups of the last element launch of an eval compute every local
// reach's QrivDown (MD_RiverFlux.cpp:5-63; a function of y only, computed once per reach as MD_f.cpp:41-43 does)
// into an 8-B slot, so the river kernel reads its own and its upstream reaches' values (MD_f.cpp:236-240) instead
// of recomputing each from a 64-B reach record and two stages.  They occupy blocks [q0, q0 + nb_q) of the launch,
// among the element tiles (q0 from DevPacked::qd_pm): late enough that the slots are still in L2 when the river
// kernel reads them, early enough that their dependent loads overlap element work instead of forming the launch's
// tail.  q0 and nb_q are multiples of 8, so the element tiles keep their XCD chunks.
struct HaloWait;
template <int MODE, bool HALO>
__device__ __forceinline__ void qd_pre(const DevMesh &m, const DevPacked &p, const YView &Y, int r, int n_int,
                                       const HaloWait *hw);
// block b -> QrivDown block (>= 0, *e untouched) or -1 with *e = the element block ordinal
__device__ __forceinline__ int qd_split(int b, int nb_q, int q0, int *e) {
    if (nb_q && b >= q0 && b < q0 + nb_q) return b - q0;
    *e = b < q0 ? b : b - nb_q;
    return -1;
}

template <int MODE, bool OPEN, bool DIAG, bool FU1, bool LCT, bool LAKE, bool GH, int HYB = 0, int LSP = 0, int BS = 256>
__device__ __forceinline__ void ele_body(const DevMesh &m, const DevPacked &p, const YView &Y, double *__restrict__ dy,
                                         int i, int cur, const DevDiag &dg, const DevLake &lk, const double *lct,
                                         const OwnRec &own);
// LSP: the values the DY tail needs from the vertical part (Es, Eg, Tg, the two DY heads and the
// cf word) are parked in per-thread LDS slots across the segment and edge loops (ds_write / ds_read on the LDS
// address space; a volatile generic pointer became flat loads with a wait each) instead of ~11 VGPRs: 80 -> 72 VGPRs,
// 7 waves per SIMD without scratch spills, element kernel -0.9 / -1.1 % in two interleaved A/Bs, same bits
// (profiles/r05/lsp/).  Forcing 7 waves without it spills 20 VGPRs to scratch: 0.788 vs 0.608 ms.  The slots add
// 11 KiB of LDS per workgroup, so the handle takes this instantiation only while 7 workgroups still fit in a CU's
// 160 KiB (kLspLdsMax: 23,296 B per workgroup, the runtime's occupancy answer on gfx950, tools/lds_occ.hip), i.e. up
// to ~35 parameter classes, and never for the diagnostic, lake or hybrid instantiations.
// (kLspN, kLspLdsMax, lsp_lds_bytes: shud_dev.h, shared with the host's edge-sharing assignment)

// HYB: the hybrid layout (DevPacked::hv): the streamed class fields come from the element's (and its neighbours')
// per-element record, the rest from the LDS class table; 1 = one streamed field (one 8-B value per element, held in
// one register pair), 2 = two to four
template <int MODE, bool OPEN, bool DIAG, bool FU1, bool LCT, bool LAKE, bool GH, int HYB = 0, int LSPK = 0>
__global__ void __launch_bounds__(kEleBS, kEleWavesOf(LCT, LSPK, GH, LAKE, HYB, DIAG, FU1, OPEN))
shud_ele_kernel_packed(DevMesh m, DevPacked p, YView Y, double *__restrict__ dy, int i0, int n_compute, int cur,
                       DevDiag dg, DevLake lk, int per8, int nb_q, int q0) {
    extern __shared__ double lct[];                       // ntab doubles (class table + pow tables) when LCT
    int eb = (int)blockIdx.x;
    const int qb = qd_split((int)blockIdx.x, nb_q, q0, &eb);
    if (qb >= 0) {
        const int r = qb * kEleBS + (int)threadIdx.x;
        if (r < p.nqd) qd_pre<MODE, false>(m, p, Y, r, 0, nullptr);
        return;
    }
    const int i = i0 + tile_of(per8, eb) * kEleBS + (int)threadIdx.x;   // elements [i0, n_compute)
    const bool act = i < n_compute;
    double tv[kTabBatch];
    if (LCT) tab_issue<kEleBS>(p, tv);
    OwnRec own;
    if (act) own = load_own<FU1, GH>(p, Y, i, cur);
    if (LCT) {
        tab_store<kEleBS>(p, tv, lct);
        __syncthreads();
    }
    if (act) ele_body<MODE, OPEN, DIAG, FU1, LCT, LAKE, GH, HYB, LCT ? LSPK : 0>(m, p, Y, dy, i, cur, dg, lk, lct, own);
}

// 129..kLdsClassMaxBig classes: the same body with the class table in LDS, staged by 1024-thread workgroups (one
// per CU, 4 waves/SIMD) — instead of dependent L2 trips per class field (the L2 table) or the SoA layout
template <int MODE, bool OPEN, bool DIAG, bool FU1, bool GH>
__global__ void __launch_bounds__(1024, 4)
shud_ele_kernel_packed_big(DevMesh m, DevPacked p, YView Y, double *__restrict__ dy, int i0, int n_compute, int cur,
                           DevDiag dg, DevLake lk, int per8) {
    extern __shared__ double lct[];
    const int i = i0 + tile_of(per8) * 1024 + (int)threadIdx.x;
    const bool act = i < n_compute;
    double tv[kTabBatch];
    tab_issue<1024>(p, tv);
    OwnRec own;
    if (act) own = load_own<FU1, GH>(p, Y, i, cur);
    tab_store<1024>(p, tv, lct);
    __syncthreads();
    if (act) ele_body<MODE, OPEN, DIAG, FU1, true, false, GH, 0, 0, 1024>(m, p, Y, dy, i, cur, dg, lk, lct, own);
}

// Partitioned handles: one launch for the interior elements [0, n_int) (ghost-free instantiation, XCD-chunked
// tiles, blocks [0, nb_int)) and, in the blocks after them, the boundary + ghost elements [n_int, n_all), which read
// halo data.  A boundary workgroup is dispatched after every interior one, so by then the halo exchange on the comm
// stream has normally long finished; each of its waves still checks the comm stream's flag (one lane polls, agent
// scope) and takes an agent-scope acquire before its first halo read.  The comm stream's work never waits for this
// kernel (the flag is enqueued before it), so the poll ends once the peers have sent; it is bounded by wall-clock
// time anyway (hw.timeout ticks of the 100 MHz constant clock, SHUD_HALO_TIMEOUT_MS, default 5 s; then the fatal
// SHUD_EF_HALO_WAIT).  An RCCL handle's first exchange (lazy connection setup) takes the split path instead.
// Consumer form (MI355X guide, "Valid forms", Consumer bullet): one relaxed agent-scope poll by lane 0, then ONE
// agent-scope acquire by the wave, whose own loads follow (no other wave of the workgroup reads halo data before it
// has polled and acquired itself).  Saves the boundary launch (~12 us at 8 ranks) and its cross-queue wait.
__device__ __forceinline__ void halo_wait(const DevMesh &m, const HaloWait &hw, int i) {
    if (hw.epoch == 0) return;
    bool late = false;
    if (__lane_id() == 0) {
        const unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load(hw.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < hw.epoch) {
            __builtin_amdgcn_s_sleep(8);
            if (wall_clock64() - t0 > hw.timeout) { late = true; break; }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    report_w(m.err, late, 0x80u, 7, i);                      // SHUD_EF_HALO_WAIT
}
template <int MODE, bool OPEN, bool FU1, int LSPK = 0>
__global__ void __launch_bounds__(256, kEleWaves)
shud_ele_kernel_packed_fold(DevMesh m, DevPacked p, YView Y, double *__restrict__ dy, int n_int, int n_all, int cur,
                            DevDiag dg, int per8, int nb_int, HaloWait hw, int nb_q, int q0) {
    extern __shared__ double lct[];
    const DevLake lk{};
    int b = (int)blockIdx.x;
    const int qb = qd_split((int)blockIdx.x, nb_q, q0, &b);
    if (qb >= 0) {                                            // QrivDown blocks: only ghost-touching waves wait
        const int r = qb * 256 + (int)threadIdx.x;
        qd_pre<MODE, true>(m, p, Y, r < p.nqd ? r : -1, n_int, &hw);
        return;
    }
    if (b < nb_int) {
        const int i = tile_of(per8, b) * 256 + (int)threadIdx.x;
        const bool act = i < n_int;
        double tv[kTabBatch];
        tab_issue<256>(p, tv);
        OwnRec own;
        if (act) own = load_own<FU1, false>(p, Y, i, cur);
        tab_store<256>(p, tv, lct);
        __syncthreads();
        if (act) ele_body<MODE, OPEN, false, FU1, true, false, false, 0, LSPK>(m, p, Y, dy, i, cur, dg, lk, lct, own);
        return;
    }
    const int i = n_int + (b - nb_int) * 256 + (int)threadIdx.x;
    const bool act = i < n_all;
    double tv[kTabBatch];
    tab_issue<256>(p, tv);
    halo_wait(m, hw, act ? i : n_int);
    OwnRec own;
    if (act) own = load_own<FU1, true>(p, Y, i, cur);
    tab_store<256>(p, tv, lct);
    __syncthreads();
    if (act) ele_body<MODE, OPEN, false, FU1, true, false, true, 0, LSPK>(m, p, Y, dy, i, cur, dg, lk, lct, own);
}
// Producer: the halo's bytes were written by earlier kernels of the comm stream (pack + RCCL, or the test's copy
// kernel), complete before this one starts; the flag store follows an agent-scope release with an explicit
// vmcnt(0) wait between them (MI355X guide, "Compiler hazard": with an empty scoreboard the compiler may drop the
// wait after the L2 write-back, letting the flag overtake it).
__global__ void shud_halo_flag_kernel(unsigned long long *flag, unsigned long long epoch) {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__global__ void shud_spin_kernel(unsigned long long ticks) {
    if (threadIdx.x == 0) {
        const unsigned long long t0 = wall_clock64();
        while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
    }
}
__global__ void shud_copy_f64_kernel(double *__restrict__ dst, const double *__restrict__ src, size_t n) {
    for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x)
        dst[k] = src[k];
}

// the streamed value of field slot k (1-based, wave-uniform) from a per-element record of up to 4 doubles: a uniform
// branch per read (a branch-free select chain on the uniform slot measured slower, profiles/r05/hybrid/)
__device__ __forceinline__ double hsel(const double (&v)[4], int k) {
    return k == 1 ? v[0] : k == 2 ? v[1] : k == 3 ? v[2] : v[3];
}
// the element's streamed record: hs = 1 (one field), 2 or 4 doubles
__device__ __forceinline__ void hload(const DevPacked &p, int i, double (&v)[4]) {
    v[1] = 0.; v[2] = 0.; v[3] = 0.;
    if (p.hs == 1) {
        v[0] = p.hv[i];
        return;
    }
    const double2 a = *(const double2 *)(p.hv + (size_t)p.hs * i);
    v[0] = a.x; v[1] = a.y;
    if (p.hs == 4) {
        const double2 b = *(const double2 *)(p.hv + (size_t)p.hs * i + 2);
        v[2] = b.x; v[3] = b.y;
    }
}

// (Edge j+1's neighbour gathers issued at the top of edge j's iteration, or edge 0's before the segment loop: 92 / 94
// VGPRs, 5 waves per SIMD, element kernel 0.620 / 0.627 vs 0.600 ms; forced to 6 waves it spills (0.752).  Occupancy
// hides the gathers' latency better than the extra loads in flight per wave, profiles/r05/edge_pf/.)
template <int MODE, bool OPEN, bool DIAG, bool FU1, bool LCT, bool LAKE, bool GH, int HYB, int LSP, int BS>
__device__ __forceinline__ void ele_body(const DevMesh &m, const DevPacked &p, const YView &Y, double *__restrict__ dy,
                                         int i, int cur, const DevDiag &dg, const DevLake &lk, const double *lct,
                                         const OwnRec &own) {
    const int NEl = m.num_ele;
    const int nown = Y.n_own;
    // ---------------- own records (loaded by the caller); saturation (its two pow calls are the register peak) is
    // computed while little else is live ----------------
    const uint32_t o16 = (uint32_t)i << 4, o8 = (uint32_t)i << 3;
    (void)o16;
    const int4 mt = own.mt;
    const double2 zz = own.zz;
    const double ysf_raw = own.ysf, yus_raw = own.yus, ygw_raw = own.ygw;
    const int cf = mt.w;
    const int cid = cf_class(cf), ibc = cf_ibc(cf);
    const bool is_lake = LAKE && cf < 0;
    const double2 snp = own.snp, stl = own.stl;            // stl = {pot_tran, ETP}
    const double etp = stl.y;
    const double2 fu = own.fu;
    const double2 csv = own.csv;
    // REPORT: an error / warning condition, reported now; REPORT_ET: one of f_etFlux's, collected in `rep`
#define REPORT(c, bit, slot, cnt) report_w(m.err, (c), (bit), (slot), i, (cnt))
#define REPORT_ET(c, bit) (rep |= (c) ? (uint32_t)(bit) : 0u)
#define CL(f) (LCT ? lct[cid * CF_LDS_STRIDE + CfPos<CF_##f>::v] : p.ctab[cid * CF_STRIDE + CfPos<CF_##f>::v])
#define CDIV(a, F) cdiv(a, CL(F), CL(r_##F))
    // HYB: CLH(f) for a field the hybrid layout may stream (uniform test of its slot), CDIV_SY: a / Sy with Sy
    // streamed takes the IEEE division (the class reciprocal would be another class's)
    double hvo[4] = {0., 0., 0., 0.};
    if (HYB == 1) hvo[0] = p.hv[i];
    else if (HYB == 2) hload(p, i, hvo);
#define CLH(f) ((HYB && p.hslot1[CF_##f]) ? (HYB == 1 ? hvo[0] : hsel(hvo, p.hslot1[CF_##f])) : CL(f))
#define CDIV_SY(a) ((HYB && p.hslot1[CF_Sy]) ? (a) / (HYB == 1 ? hvo[0] : hsel(hvo, p.hslot1[CF_Sy])) : CDIV(a, Sy))

    // ---- f_update ----
    double usf = ysf_raw, uus = yus_raw;
    if (MODE == 1) { usf = (usf >= 0.) ? usf : 0.; uus = (uus >= 0.) ? uus : 0.; }
    const double ugw = ugw_pk<MODE>(m, ygw_raw, ibc, i);
    const double zs = zz.x, zb = zz.y;
    const double aq = zs - zb;                    // InitElement after rmSinks (Model_Data.cpp:262-264)

    // ---- updateElement (Element.cpp:347-384); pure function of the state, hoisted above f_etFlux ----
    double ekh, deficit, theta, satn, satkr;
    if (is_lake) {                                // updateLakeElement (Element.cpp:336-346)
        ekh = CLH(KsatH); deficit = 0.; satn = 1.; theta = CL(ThetaS); satkr = 1.0;
    } else {
        ekh = eff_kh(ugw, aq, CLH(macD), CLH(macKsatH), CLH(vAreaF), CLH(KsatH));
        REPORT(ekh < 0. || ekh > 1e9, 0x02u, 1, false);
        deficit = aq - ugw;
        const double ThS = CL(ThetaS), ThR = CL(ThetaR);
        if (deficit <= 0.) { deficit = 0.; satn = 1.; theta = ThS; }
        else { theta = uus / deficit * ThS; satn = CDIV(theta - ThR, dTh); }
        if (satn > 0.99) { satn = 1.0; satkr = 1.0; theta = ThS; }
        else if (satn <= K_ZERO) { satn = 0.; satkr = 0.; theta = ThR; }
        else {   // satKfun, Equations.cpp:136-141
            // n/(n-1), (n-1)/n; pow_tab's tables from the workgroup's LDS copy (or the L2 class table's buffer)
            const double *pt = (LCT ? lct : p.ctab) + p.pt_off;
            satkr = sat_kfun(satn, CL(ex1), CL(ex2), pt, pt + kPowTabLogDoubles);
        }
    }

    const int sfl = own.sfl;
    // bits 26-29: edge sharing (SH), 31: LAI.  The host assigns sharing bits only to handles that take the LSP
    // instantiations (lsp_lds_bytes), without lakes or the hybrid layout, so the plain LDS-table, big-table, lake and
    // hybrid instantiations never see them and keep the 31-bit mask (the 26-bit one costs the plain LDS-table
    // kernel 6 VGPRs: 80 -> 86, 6 -> 5 waves)
    const int sfirst = sfl & ((LSP || DIAG || !LCT) ? 0x03ffffff : 0x7fffffff);
    const bool lai_on = sfl < 0;                       // bit 31: t_lai > ZERO (set with the step inputs)
    const int iss = cf_iss(cf), nseg = cf_nseg(cf);
    const double infD = CL(infD), ThR = CL(ThetaR);
    const double infK = CL(infKsatV);
    const double fu_surf = fu.x, fu_sub = fu.y;

    // ---- f_etFlux (MD_ET.cpp:343-404), serial semantics only (reads the previous call's u_satn) ----
    double Es = 0., Eu = 0., Eg = 0., Tu = 0., Tg = 0., eic = csv.y, ibeta = 0.;
    if (is_lake) {
        eic = 0.;                                 // fun_Ele_lakeVertical: qEleE_IC = 0 (carried)
        if (DIAG) { dg.q_es[i] = 0.; dg.q_eu[i] = 0.; dg.q_eg[i] = 0.; dg.q_tu[i] = 0.; dg.q_tg[i] = 0.;
                    dg.q_eta[i] = 0. + snp.y + 0.; }
    } else if (MODE == 0) {
        const double satn_prev = csv.x;
        const double va = CL(VegFrac), vb = 1. - va, pj = CL(pj);   // vb as the host derived it
        const double pet = snp.y, ptr = stl.x;
        ibeta = soil_moisture_stress(CDIV(satn_prev * CL(dTh) - ThR, fcmr));   // fc = ThS * 0.75
        Es = rmin(rmax(0., usf), pet) * vb;
        if (Es < pet) {
            if (ugw > aq - infD) { Eg = rmin(rmax(0., ugw), pet - Es) * pj * vb; Eu = 0.; }
            else { Eg = 0.; Eu = rmin(rmax(0., uus), ibeta * (pet - Es)) * pj * vb; }
        }
        if (lai_on) {                                                // LAI > ZERO
            if (eic >= ptr) { Tg = Tu = 0.; eic = ptr * pj * va; }
            else if (ugw > aq - CLH(RzD)) { Tg = rmin(rmax(0., ugw), (ptr - eic)) * pj * va; Tu = 0.; }
            else { Tg = 0.; Tu = rmin(rmax(0., uus), ibeta * (ptr - eic)) * pj * va; }
        } else { Tg = Tu = eic = 0.; }
        const double trans = Tg + Tu, evapo = Eu + Eg + Es, eta = eic + evapo + trans;
        uint32_t rep = 0;
        REPORT_ET(eta > etp * 2., 0x10u);        // printf warning, MD_ET.cpp:391-393
        // CheckNonNegative (functions.cpp:148-154): x < 0 || isnan || isinf || |x - NA| < ZERO is exactly
        // "NaN, an infinity, or a negative normal/subnormal" (-0.0 passes; x ~ -9999 is negative): one
        // v_cmp_class per value
        const bool neg = bad_nonneg(Es) || bad_nonneg(Eu) || bad_nonneg(Eg) || bad_nonneg(Tu) || bad_nonneg(Tg);
        REPORT_ET(neg, 0x04u);
        REPORT_ET(!neg && (nan_or_inf(eta) || nan_or_inf(evapo) || nan_or_inf(trans)), 0x08u);
        if (__builtin_amdgcn_ballot_w64(rep != 0)) {
            report_w(m.err, rep & 0x04u, 0x04u, 2, i);
            report_w(m.err, rep & 0x08u, 0x08u, 3, i);
            report_w(m.err, rep & 0x10u, 0x10u, 4, i, true);
        }
        if (DIAG) { dg.q_es[i] = Es; dg.q_eu[i] = Eu; dg.q_eg[i] = Eg; dg.q_tu[i] = Tu; dg.q_tg[i] = Tg;
                    dg.q_eta[i] = eta; dg.i_beta[i] = ibeta; }
    }
    stnt2(atw(p.cs[cur ^ 1], o16), satn, eic);

    // ---- Flux_Infiltration (Element.cpp:271-303) and Flux_Recharge (:304-335); zero on lake elements ----
    double qi = 0., qex = 0., qr = 0.;
    if (!is_lake) {
        const double kmax = CL(kmax);
        const double av = usf + snp.x;
        if (ugw + uus > aq || deficit < uus) {
            qex = fabs(ugw + uus - aq) / aq * kmax;
        } else if (av > 0. && deficit > infD) {
            const double grad = 1. + CDIV(av, infD);
            double ek;
            if (av > kmax) ek = CL(ekA) + CL(ekB) * satn;
            else if (av > infK) ek = satkr * infK * CL(omh) + CL(ekB) * satn;
            else ek = satkr * infK * CL(omh);
            qi = rmin(av, rmax(0., grad * ek));
        }
        const double KV = CLH(KsatV);                              // meanHarmonic, Equations.hpp:45-48
        if (!(ugw > aq - infD && uus < deficit)) {
            double grad = 0.;
            if (theta > ThR && !(uus <= K_EPSILON)) {
                grad = CDIV(theta - ThR, fcmr);
                grad = rmax(grad, 0.);
            }
            if (!(infK <= 0. || KV <= 0.)) {
                const double ku = infK * satkr;
                qr = grad * ((ku * KV) * (deficit + ugw) / (deficit * KV + ugw * ku));
            }
        }
    }
    const double q_infil = qi * fu_surf, q_exfil = qex * fu_surf;
    const double q_rech = is_lake ? 0. : qr * fu_sub;

    // DY terms that do not depend on the lateral fluxes, in the reference's left-to-right order
    // (MD_f.cpp:88-90): dsf = ((net_prep - infil) + exfil) - Qsurf/area - Es,  dus complete,
    // dgw = (recharge - exfil) - Qsub/area - Eg - Tg.  Ends the ET/vertical live ranges early.
    const double dsf_head = snp.x - q_infil + q_exfil;
    const double dgw_head = q_rech - q_exfil;
    typedef __attribute__((address_space(3))) volatile double lds_vd;        // ds_write / ds_read, not flat
    lds_vd *lsp = LSP ? (lds_vd *)(lct + p.ntab) + threadIdx.x : nullptr;
    typedef __attribute__((address_space(3))) volatile int lds_vi;
    lds_vi *lspi = LSP ? (lds_vi *)(lct + p.ntab + kLspN * kEleBS) + threadIdx.x : nullptr;   // + the cf word
    if (LSP) {
        lsp[0] = Es; lsp[kEleBS] = Eg; lsp[2 * kEleBS] = Tg; lsp[3 * kEleBS] = dsf_head; lsp[4 * kEleBS] = dgw_head;
        lspi[0] = cf;
    }
    if (i < nown) __builtin_nontemporal_store(is_lake ? 0. : CDIV_SY(q_infil - q_rech - Eu - Tu), atw(dy + nown, o8));

    // ---- own river segments (fun_Seg_surface / fun_Seg_sub) and Qe2r (PassValue) ----
    const double dep = CLH(depression), rgh = CLH(rough);
    double qe2r_surf = 0., qe2r_sub = 0.;
    if (nseg) {
        const double isf_seg = rmax(0., usf - q_infil + q_exfil);
        for (int k = sfirst, k1 = k + nseg; k < k1; k++) {
            // 20 B per segment streamed ({length, Cwr} + its reach); the reach's {depth, KsatH | BedThick, BC} is one
            // 32-B record shared by the reach's ~5 segments (a gather beside the stage gather, mostly cache hits).
            // (A 48-B segment record with the reach statics copied in, rounds 1-3: +153 MB of HBM per launch.)
            const uint32_t k16 = (uint32_t)k << 4;
            const double2 lc = *at(p.sg_lc, k16);
            const int rr = *at(p.sg_r, (uint32_t)k << 2);
            const double2 dk = p.rrec[2 * (size_t)rr], rx = p.rrec[2 * (size_t)rr + 1];
            const int rbc = __builtin_bit_cast(int2, rx.y).x;
            const double bt = rx.x;
            // (the first segment's reach index + stage loaded at the top of the body instead, in flight across the
            // vertical physics: 88 VGPRs, 0.625 vs 0.623 ms — not kept, profiles/r03/ab_river2/)
            double yr = GH ? Y.riv(rr) : *at(Y.y + 3 * (size_t)nown, (uint32_t)rr << 3);   // uriv_of, BC below
            if (MODE == 1) yr = (yr >= 0.) ? yr : 0.;
            if (rbc > 0) yr = m.rybc[rbc];
            const double rdep = dk.x, L = lc.x;
            const double qs = weir_jtoi(zs, isf_seg, zs - rdep, yr, zs + 0.0, lc.y, L, dep);
            const double qg = r2e_gw(yr, zs - rdep, ugw, zb, ekh, dk.y, L, bt) * fu_sub;
            *atw(p.qseg2, k16) = make_double2(qs, qg);                  // element-sorted
            qe2r_surf += -qs;
            qe2r_sub += -qg;
        }
    }
    if (DIAG) {
        dg.q_infil[i] = q_infil; dg.q_exfil[i] = q_exfil; dg.q_recharge[i] = q_rech;
        dg.e_ic[i] = eic; dg.u_satn[i] = satn; dg.eff_kh[i] = ekh;
        dg.qe2r_surf[i] = qe2r_surf; dg.qe2r_sub[i] = qe2r_sub;
    }
    if (i >= nown) return;    // ghost element of a partition: vertical + segments only

    // ---- fun_Ele_surface / fun_Ele_sub (MD_ElementFlux.cpp:35-156) ----
    // edge(j): edge j's QeleSurf (qsf) and QeleSub before fu_Sub (q).  Its neighbour data is loaded at the top of
    // each evaluation and the callers keep their loops rolled (<= 96 VGPRs = 5 waves/SIMD; all three edges in flight
    // at once needs ~145 = 3 waves: slower).  sh (interior edges, SH below): bit 0 the neighbour's QeleSurf for this
    // edge is -qsf (else qsf), bit 1 its QeleSub before fu_Sub is -q (else q), bit 2 neither head difference is NaN.
    bool nan_q = false;
    const double isf = usf < 0. ? 0. : usf;
    const double area = ldnt(at(p.area, o8));          // in flight across the edge loop
    const int n_edges = is_lake ? 0 : 3;               // lake elements: fun_Ele_lakeHorizon, all zero
    constexpr bool SH = kShareOn(LCT, GH, LAKE, HYB, DIAG) && LSP != 0 && BS == kEleBS;   // edge sharing, below
    auto edge = [&](int j, double &qsf, double &q, uint32_t &sh) __attribute__((always_inline)) {
        const int nb = j == 0 ? mt.x : j == 1 ? mt.y : mt.z;
        const int nc = nb >= 0 ? nb : i;                  // boundary edge: harmless in-bounds loads
        // (edge 0's loads issued right after the own record instead — held through the vertical physics — took
        // the kernel to 96 VGPRs with spills and measured 0.707 vs 0.617 ms, profiles/r03/ab_prologue/)
        const uint32_t n16 = (uint32_t)nc << 4, n8 = (uint32_t)nc << 3;
        // (a 32-bit byte offset: j is per lane under SH, and a 64-bit pointer per lane cost a spilled VGPR and +3 %)
        const double2 g = ldnt2(at(p.ged, o16 + (uint32_t)j * ((uint32_t)NEl << 4)));
        const double2 nzz = *at(p.zz, n16);
        const int ncf = *at((const int *)p.meta + 3, n16);
        const double nsf_raw = GH ? Y.sf(nc) : *at(Y.y, n8);
        const double ngw_raw = GH ? Y.gw(nc) : *at(Y.y + 2 * (size_t)nown, n8);
        const double B = g.x, d2n = g.y;
        const Recip R2 = recip_nr(d2n);                   // both Dist2Nabor divisions of the edge share 1/d2n
        qsf = 0.; q = 0.; sh = 0u;
        // (SH: the own depression and roughness re-read from the LDS class table per edge instead of held in four
        // VGPRs across the edge section)
        const double dep_e = SH ? (double)((lds_vd *)lct)[cid * CF_LDS_STRIDE + CfPos<CF_depression>::v] : dep;
        const double rgh_e = SH ? (double)((lds_vd *)lct)[cid * CF_LDS_STRIDE + CfPos<CF_rough>::v] : rgh;
        const int cn = cf_class(ncf);
#define CN(f) (LCT ? lct[cn * CF_LDS_STRIDE + CfPos<CF_##f>::v] : p.ctab[cn * CF_STRIDE + CfPos<CF_##f>::v])
        double hvn[4] = {0., 0., 0., 0.};                 // HYB: the neighbour's streamed fields (if it reads any)
        if (HYB == 1 && p.hnb) hvn[0] = p.hv[nc];
        else if (HYB == 2 && p.hnb) hload(p, nc, hvn);
#define CNH(f) ((HYB && p.hslot1[CF_##f]) ? (HYB == 1 ? hvn[0] : hsel(hvn, p.hslot1[CF_##f])) : CN(f))
        if (LAKE && nb >= 0 && ncf < 0) {                 // bank edge: the neighbour is a lake element
            const int l = lk.lake_of[nb];
            const double zl = lk.bathy_y[lk.bathy_off[l]];               // lake[l].zmin = bathymetry.yi[0]
            const double yl = Y.y[lk.y_off + l];                         // yLakeStg (serial: unclamped)
            const double nsf = yl < 0. ? 0. : yl;
            qsf = weir_jtoi(zl, nsf, zs, isf, zs, 0.6, B, 0.01);          // MD_ElementFlux.cpp:46-53
            const double dhg = (ugw + zb) - (yl + zl);                   // MD_ElementFlux.cpp:107-121
            if (dhg > 0. && ugw <= 0.02) q = 0.;
            else if (dhg < 0. && yl <= 0.02) q = 0.;
            else {
                const double ymg = (rmax(ugw, 0.) + rmax(yl, 0.)) * .5;
                const double grad = div_nr(dhg, R2);
                const double kmean = 0.5 * (ekh + CNH(KsatH));           // the lake element's u_effKH = KsatH
                q = kmean * grad * ymg * B;
            }
            lk.bank_qs[(size_t)j * NEl + i] = qsf;
            lk.bank_qg[(size_t)j * NEl + i] = q;
        } else if (nb >= 0) {
            double nsf = nsf_raw;
            if (MODE == 1) nsf = (nsf >= 0.) ? nsf : 0.;
            nsf = nsf < 0. ? 0. : nsf;
            const double zsn = nzz.x;
            const double dh = (isf + zs) - (nsf + zsn);
            [[maybe_unused]] const bool dh_nz = dh != 0., dh_ok = dh == dh;
            double ym = ((isf + zs) > (nsf + zsn)) ? ((isf > dep_e) ? isf : 0.) : ((nsf > dep_e) ? nsf : 0.);
            ym = rmin(ym, K_MAXYSURF);
            bool mu = false;                              // Manning evaluated
            if (ym > 0.) {
                const double s = div_nr(dh, R2);
                if (s > 0 && isf <= 0) qsf = 0.;
                else if (s < 0 && nsf <= 0) qsf = 0.;
                else { qsf = manning(ym * B, 0.5 * (rgh_e + CNH(rough)), ym, s); mu = true; }  // avgRough, Element.cpp:253
            }
            const double ugn = ugw_pk<MODE>(m, ngw_raw, cf_ibc(ncf), nb);
            const double zbn = nzz.y;
            const double dhg = (ugw + zb) - (ugn + zbn);
            [[maybe_unused]] const bool dhg_nz = dhg != 0., dhg_ok = dhg == dhg;
            bool zq = true;                               // one of the two zero branches
            if (dhg > 0. && ugw <= 0.02) q = 0.;
            else if (dhg < 0. && ugn <= 0.02) q = 0.;
            else {
                const double ekn = eff_kh(ugn, zsn - zbn, CNH(macD), CNH(macKsatH), CNH(vAreaF), CNH(KsatH));
                const double ymg = (rmax(ugw, 0.) + rmax(ugn, 0.)) * .5;
                const double grad = div_nr(dhg, R2);
                const double kmean = 0.5 * (ekh + ekn);
                q = kmean * grad * ymg * B;
                zq = false;
            }
            if constexpr (SH) sh = (mu && dh_nz ? 1u : 0u) | (!zq && dhg_nz ? 2u : 0u) | (dh_ok && dhg_ok ? 4u : 0u);
        } else if (OPEN) {
            const double d2e = m.dist2edge[j * NEl + i];
            if (isf > dep_e) {
                const double s = isf / d2e * 0.5;
                if (s > 0.) qsf = sqrt(s) * cbrt(isf * isf * isf * isf * isf) * B / rgh_e;
            }
            if (ugw > dep_e * 10.) {
                const double grad = ugw / d2e * 0.5;
                if (grad > 0.) q = ekh * grad;
            }
        }                                                 // closed boundary: Q = 0, times fu_Sub
#undef CN
#undef CNH
    };
    double sumsurf = qe2r_surf, sumsub = qe2r_sub;     // QeleSurfTot = Qe2r + sum_j QeleSurf[j]
    auto add = [&](int j, double qsf, double q) __attribute__((always_inline)) {
        const double qsb = q * fu_sub;
        if (MODE == 0) nan_q |= nan_or_inf(qsf) || nan_or_inf(qsb);
        sumsurf += qsf;
        sumsub += qsb;
        if (DIAG) { dg.qele_surf[j * NEl + i] = qsf; dg.qele_sub[j * NEl + i] = qsb; }
    };
    // SH: in-tile edge sharing.  The host marks (seg_first bits 26-29) interior edges between two elements of one
    // 256-element tile whose fluxes are exactly antisymmetric — the same edge length and Dist2Nabor bits on both sides,
    // the same depression, a positive avgRough, no lake — and orients them so that every element publishes at most one
    // edge and receives at most one.  From both sides the edge evaluates the same operands with dh, dhg (and the
    // Manning slope) negated exactly, the same ym, kmean, ymg and zero-branch choices, so the neighbour's values are
    // the publisher's negated — except where the negation would turn a +0 into -0: no Manning / a zero branch (both
    // sides +0), dh == +0 or dhg == +0 (both sides compute the same +-0 operands).  The publisher evaluates its edge
    // first and leaves the receiver's values in the LDS slot of its thread (the pow tables' region, dead once every
    // wave is past satKfun), keeping the two sign bits to recover its own; the receiver takes them after a barrier, or
    // evaluates the edge itself when the slot holds kShareVoid (a NaN head difference).  A lane without a publication
    // evaluates one of its own edges in that first pass instead.  The remaining edges are then evaluated one per
    // iteration with a per-lane slot (a paired element: one), so a wave makes two edge-evaluation passes instead of
    // three unless it holds the one element per tile path that must evaluate three; the sums keep the reference's
    // slot order.  syn-10M: 99.6 % of the elements receive an edge (profiles/r06/share/).
    if constexpr (!SH) {
#pragma unroll 1
        for (int j = 0; j < n_edges; j++) {
            double qsf, q;
            uint32_t sh;
            edge(j, qsf, q, sh);
            add(j, qsf, q);
        }
    } else {
        // xq[t], xq[kEleBS + t]: the receiver's {QeleSurf, QeleSub before fu_Sub} of thread t's published edge, or
        // kShareVoid in the first when a head difference was NaN (the receiver then evaluates the edge itself)
        lds_vd *xq = (lds_vd *)(lct + p.pt_off);
        const int tid = (int)threadIdx.x;
        // st: bits 0-1 the published slot + 1, 2-3 the received slot + 1, 4-5 the sh signs of the thread's own LDS
        // slot (own values = the LDS values with these signs undone), 8-10 the slots still to be taken from LDS, 12-13
        // the first pass's slot + 1 — one register for all of it: the loop below runs at the kernel's VGPR peak
        uint32_t st = ((uint32_t)sfl >> 26) & 15u;
        // first pass, every lane: its published edge, or else its lowest slot that is not the received one, whose
        // values then wait in the thread's own (unpublished) LDS slot — so an element that only receives (a tile's
        // first) makes its two evaluations in the two passes the wave makes anyway
        const int jr0 = (int)((st >> 2) & 3u) - 1;
        const int j1 = (st & 3u) ? (int)(st & 3u) - 1 : (jr0 == 0 ? 1 : 0);
        st |= (uint32_t)(j1 + 1) << 12;
        __syncthreads();                                  // every wave is past satKfun's pow-table reads
        {
            double qsf, q;
            uint32_t sh;
            edge(j1, qsf, q, sh);
            if (!(st & 3u)) sh = 4u;                      // not a publication: raw values, always taken back
            xq[tid] = (sh & 4u) ? ((sh & 1u) ? -qsf : qsf) : __builtin_bit_cast(double, kShareVoid);
            xq[kEleBS + tid] = (sh & 2u) ? -q : q;
            st |= (sh & 3u) << 4 | ((sh & 4u) ? 1u << (8 + j1) : 0u);   // void: evaluated again below
        }
        __syncthreads();                                  // the published edges are in LDS
        auto rthread = [&]() __attribute__((always_inline)) {   // the publisher of the received edge
            const int jr = (int)((st >> 2) & 3u) - 1;
            return (jr == 0 ? mt.x : jr == 1 ? mt.y : mt.z) - (i - tid);
        };
        if (st & 12u) {
            const int rt = rthread();
            if (rt >= 0 && rt < kEleBS && __builtin_bit_cast(uint64_t, (double)xq[rt]) != kShareVoid)
                st |= 1u << (8 + ((st >> 2) & 3u) - 1);
        }
        auto take = [&](int mm) __attribute__((always_inline)) {
            double qsf, q;
            if (mm == (int)((st >> 12) & 3u) - 1) {       // the thread's own slot: undo the receiver's signs
                const double a = xq[tid], b = xq[kEleBS + tid];
                qsf = (st & 16u) ? -a : a;
                q = (st & 32u) ? -b : b;
            } else {
                const int rt = rthread();
                qsf = xq[rt];
                q = xq[kEleBS + rt];
            }
            add(mm, qsf, q);
        };
#pragma unroll 1
        for (uint32_t om = 7u & ~(st >> 8); om; om &= om - 1) {
            const int j = __builtin_ctz(om);
            double qsf, q;
            uint32_t sh;
            edge(j, qsf, q, sh);
#pragma unroll
            for (int mm = 0; mm < 2; mm++)
                if ((st >> (8 + mm) & 1u) && mm < j) { take(mm); st &= ~(1u << (8 + mm)); }
            add(j, qsf, q);
        }
#pragma unroll
        for (int mm = 0; mm < 3; mm++)
            if (st >> (8 + mm) & 1u) take(mm);
    }
    if (DIAG && is_lake)
        for (int j = 0; j < 3; j++) { dg.qele_surf[j * NEl + i] = 0.; dg.qele_sub[j * NEl + i] = 0.; }
    if (MODE == 0) REPORT(nan_q, 0x01u, 0, false);         // CheckNANij, MD_f.cpp:73-74

    // ---- f_applyDY element part (MD_f.cpp:88-150 / MD_f_omp.cpp:26-46) ----
    double dsf, dgw;
    const Recip RA = recip_nr(area);                          // the area divisions share 1/area
    if (LSP) {
        const double es = lsp[0], eg = lsp[kEleBS], tg = lsp[2 * kEleBS], dsh = lsp[3 * kEleBS], dgh = lsp[4 * kEleBS];
        dsf = dsh - div_nr(sumsurf, RA) - es;
        dgw = dgh - div_nr(sumsub, RA) - eg - tg;
    } else {
        dsf = dsf_head - div_nr(sumsurf, RA) - Es;
        dgw = dgw_head - div_nr(sumsub, RA) - Eg - Tg;
    }
    const int cf_t = LSP ? lspi[0] : cf;                      // (LSP: the cf word back from LDS)
    const int ibc_t = LSP ? cf_ibc(cf_t) : ibc, iss_t = LSP ? cf_iss(cf_t) : iss;
    if (ibc_t > 0) dgw = 0;
    else if (ibc_t < 0) dgw += div_nr(m.eqbc[-ibc_t], RA);
    if (iss_t == 1) dsf += zero_over(area);                   // QSS is never assigned: 0.0 / area
    else if (iss_t == 2) dgw += zero_over(area);
    dgw = CDIV_SY(dgw);
    if (LSP ? (LAKE && cf_t < 0) : is_lake) { dsf = 0.; dgw = 0.; }   // MD_f.cpp:146-150
#undef CL
#undef CLH
#undef CDIV_SY
    __builtin_nontemporal_store(dsf, atw(dy, o8));
    __builtin_nontemporal_store(dgw, atw(dy + 2 * (size_t)nown, o8));
    if (DIAG) { dg.qele_surf_tot[i] = sumsurf; dg.qele_sub_tot[i] = sumsub; }
#undef REPORT
#undef REPORT_ET
}

// ===================================================================================
// river kernel on 16-byte reach records (same physics and order as shud_riv_kernel, shud_kernels.hip)
// ===================================================================================
struct RivP {
    double w0, bs, len, slope, d2d, n, depth;
    int down, bc;
};
__device__ __forceinline__ int2 rv_ib(double x) { return __builtin_bit_cast(int2, x); }   // (down, BC)
__device__ __forceinline__ RivP riv_load(const DevPacked &p, int r) {
    const double2 *q = p.rv + 4 * (size_t)r;                  // one 64-B record: a single cache line
    const double2 a = q[0], b = q[1], c = q[2], d = q[3];
    const int2 ib = rv_ib(d.y);
    RivP o;
    o.w0 = a.x; o.bs = a.y; o.len = b.x; o.slope = b.y; o.d2d = c.x; o.n = c.y; o.depth = d.x;
    o.down = ib.x; o.bc = ib.y;
    return o;
}
__device__ __forceinline__ RivGeom riv_geom_p(const RivP &q, double y) { return riv_geom(q.w0, q.bs, q.len, y); }
// stage after f_update's clamp + BC override; *yg = the value updateRiver() saw
template <int MODE>
__device__ __forceinline__ double riv_stage_p(const DevMesh &m, const YView &Y, int r, int bc, double *yg) {
    double yr = Y.riv(r);
    if (MODE == 1) yr = (yr >= 0.) ? yr : 0.;
    *yg = yr;
    return bc > 0 ? m.rybc[bc] : yr;
}
// MD_RiverFlux.cpp:5-63: reach q with stage uq and geometry g; its downstream has stage ud, depth, slope
__device__ __forceinline__ double riv_down_p(const RivP &q, double uq, const RivGeom &g, double ud, double ddepth,
                                             double dslope) {
    if (q.down >= 0) {
        const double smean = (q.slope + dslope) * 0.5;
        const double s = ((uq - q.depth) - (ud - ddepth)) / q.d2d + smean;
        const double R = (g.csperem <= K_ZERO) ? 0. : (g.csarea / g.csperem);
        return manning(g.csarea, q.n, R, s);
    } else if (q.down >= -3) {
        const double s = q.slope + uq * 2. / q.len;
        const double R = (g.csperem <= 0.) ? 0. : (g.csarea / g.csperem);
        return manning(g.csarea, q.n, R, s);
    }
    return g.csarea * sqrt(K_GRAV * uq) * 60.;
}
// outlet form only (a reach flowing into a lake, the lake kernel's QLakeRivIn: down = -3 on the record)
__device__ __forceinline__ double riv_down_outlet(const RivP &q, double uq, const RivGeom &g) {
    return riv_down_p(q, uq, g, 0., 0., 0.);
}
// QrivDown of local reach r (owned or ghost) into its slot: the river kernel's own-reach term, operand for operand
// (a ghost reach whose downstream is not local carries the outlet code on its record; its slot is never read).
// HALO (the folded partition launch): a wave with a lane whose reach or downstream is a ghost takes the halo
// wait (poll + agent acquire, which invalidates the CU's L1) before its stage loads; the others — nearly all —
// read only owned stages and skip it.  r < 0: an idle lane (still reaches the wave-wide ballot).
template <int MODE, bool HALO>
__device__ __forceinline__ void qd_pre(const DevMesh &m, const DevPacked &p, const YView &Y, int r, int n_int,
                                       const HaloWait *hw) {
    const int rr = r < 0 ? 0 : r;
    const RivP q = riv_load(p, rr);
    const int d = q.down >= 0 ? q.down : rr;                    // clamped: unconditional loads
    if (HALO) {
        const bool ghost = r >= 0 && (r >= Y.n_own_riv || d >= Y.n_own_riv);
        if (__builtin_amdgcn_ballot_w64(ghost)) halo_wait(m, *hw, n_int);
    }
    if (r < 0) return;
    double yg;
    const double ur = riv_stage_p<MODE>(m, Y, r, q.bc, &yg);
    const RivGeom g = riv_geom_p(q, yg);
    const double2 bd = p.rv[4 * (size_t)d + 1], dd = p.rv[4 * (size_t)d + 3];
    double ydg;
    const double ud = riv_stage_p<MODE>(m, Y, d, rv_ib(dd.y).y, &ydg);
    p.qdown[r] = riv_down_p(q, ur, g, ud, dd.x, bd.y);
}

// dword-aligned 16-B / 8-B loads of index words (gfx950 global loads need only 4-B alignment for dwordx4)
struct __attribute__((packed, aligned(4))) Int4u { int x, y, z, w; };
struct __attribute__((packed, aligned(4))) Int2u { int x, y; };

// The kernel is bound by its load-instruction count per wave, not by bytes (227 MB per launch is 1.07x its unique
// footprint) nor by neighbour locality (profiles/r04/ab_riv/riv_order*.log): round 4 cut the per-reach loads —
// one 16-B index word per reach (rv_u, shud_dev.h) instead of two; a many-upstream reach's up_idx slots loaded
// together from the offset in that word (no up_off load, no index load per upstream reach); a segment batch's
// flux positions as 16-B (+ 8-B) loads instead of one 4-B load each; SB segments per batch, chosen by the host
// from the reaches' segment counts (choose_riv_sb, shud_rhs.cpp).  0.0709 -> 0.0605 ms at syn-10M, same bits.
template <int MODE, bool DIAG, int SB, bool QD>
__device__ __forceinline__ void riv_body(const DevMesh &m, const DevPacked &p, const YView &Y, double *__restrict__ dy,
                                         const DevDiag &dg, int r) {
    const RivP q = riv_load(p, r);
    const int4 ru = p.rv_u[r];                  // {first segment, #segments | code << 16, w2, w3}
    const int seg0 = ru.x, nseg = ru.y & 0xffff, upc = ru.y >> 16;
    double yg;
    const double ur = riv_stage_p<MODE>(m, Y, r, q.bc, &yg);
    const RivGeom g = riv_geom_p(q, yg);
    double qdown = 0.;
    if (QD) {
        qdown = p.qdown[r];                                     // this eval's pre-pass (qd_pre), same operands
    } else {
        const int d = q.down >= 0 ? q.down : r;                 // clamped: unconditional loads
        const double2 bd = p.rv[4 * (size_t)d + 1], dd = p.rv[4 * (size_t)d + 3];   // same line of d's record
        const int bcd = rv_ib(dd.y).y;
        double ydg;
        const double ud = riv_stage_p<MODE>(m, Y, d, bcd, &ydg);
        qdown = riv_down_p(q, ur, g, ud, dd.x, bd.y);
    }
    // junction: QrivUp[down] += -QrivDown[i], i ascending (MD_f.cpp:236-240).  An upstream reach u's QrivDown is
    // the same expression on the same operands (its downstream is r: stage ur, r's depth and slope) whether read
    // from u's pre-pass slot or recomputed from u's record
    auto up_term = [&](int u) {
        if (QD) return -p.qdown[u];
        const RivP qu = riv_load(p, u);
        double yu;
        const double uu = riv_stage_p<MODE>(m, Y, u, qu.bc, &yu);
        return -riv_down_p(qu, uu, riv_geom_p(qu, yu), ur, q.depth, q.slope);
    };
    double qup = 0.;
    if (upc < 3) {                                       // 0..2 upstream reaches in w2, w3
        if (upc > 0) qup += up_term(ru.z);
        if (upc > 1) qup += up_term(ru.w);
    } else {                                                    // more: up_idx[w2 .. w2 + w3), 8 indices at a time
        for (int k0 = ru.z, k1 = ru.z + ru.w; k0 < k1; k0 += 8) {
            int uv[8];
#pragma unroll
            for (int j = 0; j < 8; j++) uv[j] = m.up_idx[k0 + j < k1 ? k0 + j : k0];
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (k0 + j < k1) qup += up_term(uv[j]);
        }
    }
    // segment sums, ascending reference segment order (MD_f.cpp:228-235), gathered from the element-sorted
    // fluxes (scattered 8-B writes from the element kernel cost more than these gathers).  Batches of SB:
    // the positions (16-B loads; rseg_pos is padded by 8 words), then all gathers, are in flight together;
    // positions past the reach's last segment are replaced by its first (the same line); the adds stay in order
    double qsurf = 0., qsub = 0.;
    for (int k0 = seg0, k1 = seg0 + nseg; k0 < k1; k0 += SB) {
        int raw[SB], ps[SB];
#pragma unroll
        for (int c = 0; c + 4 <= SB; c += 4) {
            const Int4u v = *reinterpret_cast<const Int4u *>(m.rseg_pos + k0 + c);
            raw[c] = v.x; raw[c + 1] = v.y; raw[c + 2] = v.z; raw[c + 3] = v.w;
        }
        if constexpr (SB % 4 == 2) {
            const Int2u v = *reinterpret_cast<const Int2u *>(m.rseg_pos + k0 + SB - 2);
            raw[SB - 2] = v.x; raw[SB - 1] = v.y;
        }
#pragma unroll
        for (int j = 0; j < SB; j++) ps[j] = k0 + j < k1 ? raw[j] : raw[0];
        double2 qv[SB];
#pragma unroll
        for (int j = 0; j < SB; j++) qv[j] = p.qseg2[ps[j]];
#pragma unroll
        for (int j = 0; j < SB; j++)
            if (k0 + j < k1) { qsurf += qv[j].x; qsub += qv[j].y; }
    }
    const double qbc = (q.bc < 0) ? m.rqbc[-q.bc] : 0.0;
    double dv;
    if (q.bc > 0) dv = 0.;
    else if (MODE == 0) {   // MD_f.cpp:162-166
        dv = (-qup - qsurf - qsub - qdown + qbc) / q.len;
        if (dv < -1. * g.csarea) dv = -1. * g.csarea;
        dv = da_to_dy(dv, g.topw, q.bs);                              // fun_dAtodY functions.hpp:125-153
    } else {                // MD_f_omp.cpp:59
        dv = (-qup - qsurf - qsub - qdown + qbc) / g.toparea;
    }
    dy[3 * Y.n_own + r] = dv;
    if (DIAG) { dg.qriv_down[r] = qdown; dg.qriv_up[r] = qup; dg.qriv_surf[r] = qsurf; dg.qriv_sub[r] = qsub; }
}
template <int MODE, bool DIAG, int SB, bool QD>
__global__ void __launch_bounds__(256)
shud_riv_kernel_packed(DevMesh m, DevPacked p, YView Y, double *__restrict__ dy, DevDiag dg, int per8) {
    // XCD-chunked workgroup order: a reach's up/downstream records sit a few blocks away in index space,
    // so they are L2 hits on the same XCD instead of fabric round trips (speed only)
    const int r = tile_of(per8) * 256 + (int)threadIdx.x;
    if (r >= Y.n_own_riv) return;
    riv_body<MODE, DIAG, SB, QD>(m, p, Y, dy, dg, r);
}

template <int SB, bool QD>
static void launch_riv_sb(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int mode, bool diag,
                          const DevDiag &dg, hipStream_t s) {
    const dim3 grid(((Y.n_own_riv + 255) / 256 + 7) / 8 * 8), blk(256);
    const int per8 = (int)grid.x / 8;
    if (mode == 0) {
        if (diag) hipLaunchKernelGGL((shud_riv_kernel_packed<0, true, SB, QD>), grid, blk, 0, s, m, p, Y, dy, dg, per8);
        else hipLaunchKernelGGL((shud_riv_kernel_packed<0, false, SB, QD>), grid, blk, 0, s, m, p, Y, dy, dg, per8);
    } else {
        if (diag) hipLaunchKernelGGL((shud_riv_kernel_packed<1, true, SB, QD>), grid, blk, 0, s, m, p, Y, dy, dg, per8);
        else hipLaunchKernelGGL((shud_riv_kernel_packed<1, false, SB, QD>), grid, blk, 0, s, m, p, Y, dy, dg, per8);
    }
}

void launch_river_kernel_packed(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int mode,
                                bool diag, const DevDiag &dg, hipStream_t s, bool qd) {
    if (Y.n_own_riv <= 0) return;
    const int sb = p.riv_sb;
    if (qd && p.qdown) {
        if (sb == 6) launch_riv_sb<6, true>(m, p, Y, dy, mode, diag, dg, s);
        else launch_riv_sb<8, true>(m, p, Y, dy, mode, diag, dg, s);
    } else {
        if (sb == 6) launch_riv_sb<6, false>(m, p, Y, dy, mode, diag, dg, s);
        else launch_riv_sb<8, false>(m, p, Y, dy, mode, diag, dg, s);
    }
}

// ===================================================================================
// lakes: one workgroup per lake.  Every lake sum keeps the reference's order — lake elements
// ascending (MD_f.cpp:16-17), bank edges by element then edge (MD_ElementFlux.cpp:52,121), inflowing reaches
// ascending (MD_RiverFlux.cpp:24) — by staging each 256-wide chunk of terms in LDS (parallel loads) and
// adding them on one lane.  A lake has O(1e3) terms: the kernel is latency-bound and tiny.
// ===================================================================================
// Lake.cpp:59-79 LakeBathymetry::toparea, the reference's own interpolation as written
__device__ double lake_toparea(const DevLake &L, int l, double y) {
    const double *yi = L.bathy_y + L.bathy_off[l], *ai = L.bathy_a + L.bathy_off[l];
    const int nvalue = L.bathy_off[l + 1] - L.bathy_off[l];
    double ta = ai[0];
    if (y <= yi[0]) {
        ta = ai[0];
    } else {
        for (int k = 1; k < nvalue; k++) {
            if (y < yi[k]) {
                const double da = (ai[k] - ta), dyy = yi[k] - y;
                ta = da / dyy * (y - yi[k - 1]) + ta;
                break;
            }
            ta = ai[k];
        }
    }
    return ta;
}

// ordered sum of f(k) for k in [k0, k1): chunks of blockDim.x loaded in parallel, added in order by lane 0
template <class F>
__device__ double ordered_sum(int k0, int k1, F f, double *buf) {
    double acc = 0.;
    for (int b = k0; b < k1; b += blockDim.x) {
        const int k = b + (int)threadIdx.x;
        if (k < k1) buf[threadIdx.x] = f(k);
        __syncthreads();
        if (threadIdx.x == 0) {
            const int n = min((int)blockDim.x, k1 - b);
            for (int t = 0; t < n; t++) acc += buf[t];
        }
        __syncthreads();
    }
    return acc;                                  // valid on lane 0
}

__global__ void __launch_bounds__(256)
shud_lake_kernel(DevMesh m, DevPacked p, DevLake L, YView Y, double *__restrict__ dy, int diag, DevDiag dg) {
    __shared__ double buf[256];
    const int l = blockIdx.x;
    const double yl = Y.y[L.y_off + l];                                   // yLakeStg (MD_update.cpp:175)
    const int e0 = L.ele_off[l], e1 = L.ele_off[l + 1];
    const double n_ele = (double)(e1 - e0);                               // lake[l].NumEleLake
    // qLakeEvap += qEleEvapo / NumEleLake (qEleEvapo = qPotEvap, fun_Ele_lakeVertical); qLakePrcp likewise
    const double qevap = ordered_sum(e0, e1, [&](int k) { return m.pot_evap[L.ele_idx[k]] / n_ele; }, buf);
    const double qprcp = ordered_sum(e0, e1, [&](int k) { return m.prcp[L.ele_idx[k]] / n_ele; }, buf);
    const double qsurf = ordered_sum(L.bank_off[l], L.bank_off[l + 1],
                                     [&](int k) { return L.bank_qs[L.bank_pos[k]]; }, buf);
    const double qsub = ordered_sum(L.bank_off[l], L.bank_off[l + 1],
                                    [&](int k) { return L.bank_qg[L.bank_pos[k]]; }, buf);
    // QLakeRivIn += QrivDown of each inflowing reach (zero-depth-gradient Manning, MD_RiverFlux.cpp:17-25),
    // recomputed here from the reach's own stage with the river kernel's functions
    const double qin = ordered_sum(L.rin_off[l], L.rin_off[l + 1], [&](int k) {
        const int r = L.rin_idx[k];
        const RivP q = riv_load(p, r);
        double yg;
        const double ur = riv_stage_p<0>(m, Y, r, q.bc, &yg);
        return riv_down_outlet(q, ur, riv_geom_p(q, yg));                // q.down = -3: outlet formula
    }, buf);
    if (threadIdx.x == 0) {
        const double zmin = L.bathy_y[L.bathy_off[l]];
        const double area = lake_toparea(L, l, yl + zmin);                // _Lake::update (Lake.cpp:104-107)
        double qe = rmin(qevap, qprcp + yl);                              // MD_f.cpp:44-47
        qe = rmax(0, qe);
        dy[L.y_off + l] = qprcp - qe + (qin - 0. + qsub + qsurf) / area;  // MD_f.cpp:180-183 (QLakeRivOut = 0)
        if (diag) {
            dg.q_lake_surf[l] = qsurf; dg.q_lake_sub[l] = qsub; dg.q_lake_rivin[l] = qin;
            dg.q_lake_evap[l] = qe; dg.q_lake_prcp[l] = qprcp; dg.lake_toparea[l] = area;
        }
    }
}

void launch_lake_kernel(const DevMesh &m, const DevPacked &p, const DevLake &L, const YView &Y, double *dy,
                        bool diag, const DevDiag &dg, hipStream_t s) {
    if (L.nl <= 0) return;
    hipLaunchKernelGGL(shud_lake_kernel, dim3(L.nl), dim3(256), 0, s, m, p, L, Y, dy, diag ? 1 : 0, dg);
}

// step inputs (SoA staging in DevMesh) -> packed records; `what` bits: 1 np, 2 tl, 4 fu, 8 u_satn, 16 e_ic
__global__ void __launch_bounds__(256)
shud_pack_step_kernel(DevMesh m, DevPacked p, int n, int cur, unsigned what) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (what & 1) p.s_np[i] = make_double2(m.net_prep[i], m.pot_evap[i]);
    if (what & 2) {
        p.s_tl[i] = make_double2(m.pot_tran[i], m.etp[i]);
        p.seg_first[i] = (p.seg_first[i] & 0x7fffffff) | (m.lai[i] > K_ZERO ? (int)0x80000000u : 0);
    }
    if (what & 4) p.s_fu[i] = make_double2(m.fu_surf[i], m.fu_sub[i]);
    if (what & 8) p.cs[cur][i].x = m.u_satn[0][i];
    if (what & 16) p.cs[cur][i].y = m.e_ic[0][i];
}

template <int MODE, bool OPEN, bool DIAG, bool FU1, bool GH>
static void launch_big(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int i0, int i1, int cur,
                       const DevDiag &dg, const DevLake &lk, hipStream_t s) {
    int nb = (i1 - i0 + 1023) / 1024;
    nb = (nb + 7) / 8 * 8;                  // block_id<1> deals blocks to XCDs in contiguous chunks
    const size_t lds = (size_t)p.ntab * sizeof(double);
    auto *fn = shud_ele_kernel_packed_big<MODE, OPEN, DIAG, FU1, GH>;
    static bool attr = false;               // dynamic LDS above 64 KiB must be allowed per kernel
    if (!attr) {
        (void)hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)((kLdsClassMaxBig * CF_LDS_STRIDE + 1 + kPowTabDoubles) * sizeof(double)));
        attr = true;
    }
    hipLaunchKernelGGL(fn, dim3(nb), dim3(1024), lds, s, m, p, Y, dy, i0, i1, cur, dg, lk, nb / 8);
}

// first block of the QrivDown workgroups: pm permille of the nb element blocks before them, rounded down to 8
static int qd_start(int nb, int pm) {
    const long long q = (long long)nb * std::min(std::max(pm, 0), 1000) / 1000;
    return (int)(q / 8 * 8);
}
// dynamic LDS of the 256-thread packed kernel: the class + pow tables, and with LSPK the parked DY-tail slots
static size_t lds_bytes(const DevPacked &p, bool lct, bool lspk) {
    if (!lct) return 0;
    return lspk ? lsp_lds_bytes(p.ntab) : (size_t)p.ntab * sizeof(double);
}
template <int MODE, bool OPEN, bool DIAG, bool FU1, bool LCT, bool LAKE, bool GH, int HYB = 0, int LSPK = 0>
static void launch_p(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int i0, int i1, int cur,
                     const DevDiag &dg, const DevLake &lk, hipStream_t s, int nq = 0) {
    int nb = (i1 - i0 + kEleBS - 1) / kEleBS;
    nb = (nb + 7) / 8 * 8;                  // block_id<1> deals blocks to XCDs in contiguous chunks
    const int nbq = nq > 0 ? ((nq + kEleBS - 1) / kEleBS + 7) / 8 * 8 : 0;
    const int q0 = qd_start(nb, p.qd_pm);
    const size_t lds = lds_bytes(p, LCT, LSPK != 0);
    hipLaunchKernelGGL((shud_ele_kernel_packed<MODE, OPEN, DIAG, FU1, LCT, LAKE, GH, HYB, LSPK>), dim3(nb + nbq), dim3(kEleBS),
                       lds, s,
                       m, p, Y, dy, i0, i1, cur, dg, lk, nb / 8, nbq, q0);
}

// the plain LDS-table instantiation, with the DY-tail values parked in LDS when 7 workgroups still fit (LSP)
template <int MO, bool OP, bool DI, bool FU, bool GH>
static void launch_plain(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int i0, int i1, int cur,
                         const DevDiag &dg, const DevLake &lk, hipStream_t s, int nq) {
    if constexpr (!DI) {
        if (lds_bytes(p, true, true) <= kLspLdsMax) {
            launch_p<MO, OP, DI, FU, true, false, GH, 0, 1>(m, p, Y, dy, i0, i1, cur, dg, lk, s, nq);
            return;
        }
    }
    launch_p<MO, OP, DI, FU, true, false, GH>(m, p, Y, dy, i0, i1, cur, dg, lk, s, nq);
}
bool launch_element_kernel_packed(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int i0, int i1,
                                  int cur, int mode, bool open, bool diag, bool fu_unit, const DevDiag &dg,
                                  hipStream_t s, const DevLake *lake, bool interior, bool with_qd) {
    if (i1 <= i0) return false;
    DevLake lk{};
    if (lake) lk = *lake;
    // the QrivDown pre-pass rides in the 256-thread launches (not the 1024-thread big-class one)
    const int nq = (with_qd && p.qdown && p.nqd > 0 && (lake || p.ncls <= LDS_CLS_MAX)) ? p.nqd : 0;
    // lakes: serial semantics only (the handle rejects OMP + lakes), class table in LDS, with or without ghosts.
    // A partitioned handle's interior elements (interior = true: every lateral neighbour and every segment's
    // reach owned) read only owned state, so they take the ghost-free instantiation (direct y addressing).
    const bool gh = !interior && (Y.gele != nullptr || Y.griv != nullptr);
#define LP(MO, OP, DI, FU) do {                                                                            \
        if (lake && MO == 0) {                                                                            \
            if (gh) launch_p<MO, OP, DI, FU, true, true, true>(m, p, Y, dy, i0, i1, cur, dg, lk, s, nq);  \
            else launch_p<MO, OP, DI, FU, true, true, false>(m, p, Y, dy, i0, i1, cur, dg, lk, s, nq);    \
        }                                                                                                 \
        else if (p.ncls > LDS_CLS_MAX && p.ncls <= kLdsClassMaxBig && p.lds_big) {                        \
            if (gh) launch_big<MO, OP, DI, FU, true>(m, p, Y, dy, i0, i1, cur, dg, lk, s);                 \
            else launch_big<MO, OP, DI, FU, false>(m, p, Y, dy, i0, i1, cur, dg, lk, s);                   \
        }                                                                                                 \
        else if (p.ncls <= LDS_CLS_MAX && p.nh == 1) {                                                    \
            if (gh) launch_p<MO, OP, DI, FU, true, false, true, 1>(m, p, Y, dy, i0, i1, cur, dg, lk, s, nq); \
            else launch_p<MO, OP, DI, FU, true, false, false, 1>(m, p, Y, dy, i0, i1, cur, dg, lk, s, nq);   \
        }                                                                                                 \
        else if (p.ncls <= LDS_CLS_MAX && p.nh) {                                                         \
            if (gh) launch_p<MO, OP, DI, FU, true, false, true, 2>(m, p, Y, dy, i0, i1, cur, dg, lk, s, nq); \
            else launch_p<MO, OP, DI, FU, true, false, false, 2>(m, p, Y, dy, i0, i1, cur, dg, lk, s, nq);   \
        }                                                                                                 \
        else if (p.ncls <= LDS_CLS_MAX) {                                                                 \
            if (gh) launch_plain<MO, OP, DI, FU, true>(m, p, Y, dy, i0, i1, cur, dg, lk, s, nq);          \
            else launch_plain<MO, OP, DI, FU, false>(m, p, Y, dy, i0, i1, cur, dg, lk, s, nq);            \
        } else launch_p<MO, OP, DI, FU, false, false, true>(m, p, Y, dy, i0, i1, cur, dg, lk, s); } while (0)
#define LFU(MO, OP, DI) do { if (fu_unit) LP(MO, OP, DI, true); else LP(MO, OP, DI, false); } while (0)
#define LDI(MO, OP) do { if (diag) LFU(MO, OP, true); else LFU(MO, OP, false); } while (0)
#define LOP(MO) do { if (open) LDI(MO, true); else LDI(MO, false); } while (0)
    if (mode == 0) LOP(0); else LOP(1);
#undef LOP
#undef LDI
#undef LFU
#undef LP
    return nq > 0;
}

// false: this configuration has no folded instantiation (the caller launches interior and boundary separately).
// with_qd: the QrivDown blocks follow the boundary ones (and wait for the halo like them); they always ride here.
bool launch_element_kernel_packed_fold(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int n_int,
                                       int n_all, int cur, int mode, bool open, bool fu_unit, const DevDiag &dg,
                                       const HaloWait &hw, hipStream_t s, bool with_qd) {
    if (n_int <= 0 || n_all <= n_int || p.ncls > LDS_CLS_MAX || p.nh) return false;
    const int nb_int = ((n_int + 255) / 256 + 7) / 8 * 8, nb_b = (n_all - n_int + 255) / 256;
    const int nbq = (with_qd && p.qdown && p.nqd > 0) ? ((p.nqd + 255) / 256 + 7) / 8 * 8 : 0;
    // QrivDown blocks among the interior tiles (they wait for the halo like the boundary ones: it has normally
    // arrived long before), pm of the interior blocks before them
    const int q0 = qd_start(nb_int, p.qd_pm_fold);
    // the DY-tail LDS slots as in the single launch (LSP), while 7 workgroups still fit
    const bool lsp = lds_bytes(p, true, true) <= kLspLdsMax;
    const size_t lds = lds_bytes(p, true, lsp);
#define LF(MO, OP, FU) do {                                                                                        \
        if (lsp) hipLaunchKernelGGL((shud_ele_kernel_packed_fold<MO, OP, FU, 1>),                \
                                    dim3(nb_int + nb_b + nbq), dim3(256), lds, s, m, p, Y, dy, n_int, n_all, cur, dg, \
                                    nb_int / 8, nb_int, hw, nbq, q0);                                              \
        else hipLaunchKernelGGL((shud_ele_kernel_packed_fold<MO, OP, FU>), dim3(nb_int + nb_b + nbq), dim3(256),    \
                                lds, s, m, p, Y, dy, n_int, n_all, cur, dg, nb_int / 8, nb_int, hw, nbq, q0);       \
    } while (0)
    if (mode == 0) {
        if (open) { if (fu_unit) LF(0, true, true); else LF(0, true, false); }
        else { if (fu_unit) LF(0, false, true); else LF(0, false, false); }
    } else {
        if (open) { if (fu_unit) LF(1, true, true); else LF(1, true, false); }
        else { if (fu_unit) LF(1, false, true); else LF(1, false, false); }
    }
#undef LF
    return true;
}
void launch_halo_flag(unsigned long long *flag, unsigned long long epoch, hipStream_t s) {
    hipLaunchKernelGGL(shud_halo_flag_kernel, dim3(1), dim3(64), 0, s, flag, epoch);
}
void launch_spin(unsigned long long ticks, hipStream_t s) {
    hipLaunchKernelGGL(shud_spin_kernel, dim3(1), dim3(64), 0, s, ticks);
}
void launch_copy_f64(double *dst, const double *src, size_t n, hipStream_t s) {
    if (!n) return;
    const size_t nb = std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(shud_copy_f64_kernel, dim3((unsigned)nb), dim3(256), 0, s, dst, src, n);
}

void launch_pack_step_kernel(const DevMesh &m, const DevPacked &p, int n, int cur, unsigned what, hipStream_t s) {
    if (n <= 0 || !what) return;
    hipLaunchKernelGGL(shud_pack_step_kernel, dim3((n + 255) / 256), dim3(256), 0, s, m, p, n, cur, what);
}

}  // namespace shud
