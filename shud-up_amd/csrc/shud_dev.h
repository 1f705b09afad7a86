// shud_dev.h — device-side views shared by the kernels (shud_kernels.hip) and the host runtime
// (shud_rhs.cpp).  All arrays are SoA in HBM; per-edge arrays are edge-major [3][num_ele].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace shud {

// counted warnings spread over kWarnSlots counters, one 128-B L2 line each (slot = workgroup index mod
// kWarnSlots): inputs that warn on every element then cost parallel atomics on 64 lines, not a serial
// chain on one address; the host sums the slots when it reads the error word
constexpr int kWarnSlots = 64, kWarnStride = 16;
struct DevErr {                      // per-handle device error word (ShudErr on the host)
    uint32_t flags;
    int32_t first_index[8];          // slot = log2(bit); INT32_MAX = none
    unsigned long long n_warn;       // host side: sum of the slots
    unsigned long long *warn;        // [kWarnSlots * kWarnStride] device counters
};

struct DevMesh {
    int num_ele;                     // local elements incl. ghosts (per-edge stride)
    // elements: topology + geometry
    const int *nabr, *eflags;        // eflags: bits 0-15 iBC (int16), 16-17 iSS class (1: >0, 2: <0)
    const double *area, *z_surf, *z_bottom, *depression, *edge, *dist2nabor, *dist2edge, *avg_rough, *rough;
    // elements: hydraulic parameters
    const double *aq, *macD, *macKsatH, *vAreaF, *KsatH, *KsatV, *infKsatV, *hAreaF, *macKsatV;
    const double *ThetaS, *ThetaR, *Beta, *infD, *Sy, *RzD, *VegFrac, *ImpAF;
    // per-ET-step inputs
    const double *net_prep, *pot_evap, *pot_tran, *etp, *lai, *fu_surf, *fu_sub, *prcp;
    double *e_ic[2], *u_satn[2];     // carried state, ping-pong (read [cur], write [cur^1])
    const double *ugw_stale;
    const double *eybc, *eqbc, *rybc, *rqbc;
    // segments in element-sorted order (stable in reference index)
    const int *seg_off, *seg_riv;
    const double *seg_len, *seg_cwr;
    double *qseg_surf, *qseg_sub;
    // reaches
    const int *riv_down, *riv_bc;
    const double *riv_len, *riv_slope, *riv_d2down, *riv_avg_rough, *riv_depth, *riv_bw, *riv_bankslope;
    const double *riv_ksath, *riv_bedthick;
    const int *up_off, *up_idx;      // upstream reaches of each owned reach, ascending
    const int *rseg_off, *rseg_pos;  // segments of each owned reach, ascending reference order
    DevErr *err;
};

// ---- packed "class" layout (built by shud_rhs_create when the mesh allows it) -----------------------
// Per-element hydraulic parameters of a SHUD model are copies of a few soil/geol/landcover rows
// (_Element::copySoil/copyGeol/copyLandc, Element.cpp:386-418); the handle finds the distinct
// parameter tuples once and stores a class id per element, and interleaves the element's own streams
// into 16-byte records so one lane issues a few wide loads instead of ~45 narrow ones.  Pure layout:
// every value the kernel computes with is bit-identical to the SoA input.
// class table, field-major: ctab[field * ncls + class] (one field of every class is contiguous, so a
// wave-instruction gathering one field for 64 lanes touches a few cache lines, not one per class)
enum ClassField {
    CF_macD, CF_macKsatH, CF_vAreaF, CF_KsatH, CF_KsatV, CF_infKsatV, CF_hAreaF, CF_macKsatV, CF_ThetaS,
    CF_ThetaR, CF_Beta, CF_infD, CF_Sy, CF_RzD, CF_VegFrac, CF_ImpAF, CF_depression, CF_rough,
    CF_NPRIMARY,
    // derived per class on the host, in the kernel's own operation order (bit-identical by construction)
    CF_fcmr = CF_NPRIMARY,  // ThetaS * 0.75 - ThetaR
    CF_dTh,                 // ThetaS - ThetaR
    CF_ex1, CF_ex2,         // Beta / (Beta - 1),  (Beta - 1) / Beta
    CF_pj,                  // 1 - ImpAF  (1 - VegFrac is one subtraction in the kernel: cheaper than its LDS copy)
    CF_omh,                 // 1 - hAreaF
    CF_kmax,                // infKsatV * (1 - hAreaF) + macKsatV * hAreaF
    CF_ekA, CF_ekB,         // infKsatV * (1 - hAreaF),  hAreaF * macKsatV
    // correctly rounded reciprocals of the class-constant divisors (cdiv, shud_physics.h)
    CF_r_fcmr, CF_r_dTh, CF_r_infD, CF_r_Sy,
    CF_COUNT
};
// fields the packed kernel reads; hAreaF, macKsatV, Beta and ImpAF enter only through derived fields and are kept
// out of the class record (every word of the record is copied into each workgroup's LDS: 3 % of the element
// kernel per 10 KiB, profiles/r05/pow_ab)
constexpr bool cf_stored(int f) { return f != CF_hAreaF && f != CF_macKsatV && f != CF_Beta && f != CF_ImpAF; }
constexpr int cf_pos(int f) {
    int q = 0;
    for (int g = 0; g < f; g++) q += cf_stored(g) ? 1 : 0;
    return cf_stored(f) ? q : -1;
}
template <int F> struct CfPos {
    static_assert(F >= 0 && F < CF_COUNT && cf_stored(F), "field not in the class record");
    static constexpr int v = cf_pos(F);
};
constexpr int CF_NSTORED = cf_pos(CF_COUNT - 1) + 1;
// record stride of the class table (8-B words), odd: lanes reading one field of different classes from the
// LDS copy land on different banks (an even stride of 32 put every class on one bank)
constexpr int CF_STRIDE = CF_NSTORED | 1;
// divisors that cdiv (shud_physics.h) may take with a host reciprocal: 0, +-inf, NaN, or |b| in [kCdivBmin,
// kCdivBmax] (the handle checks every such divisor at create and otherwise keeps the plain-division layout)
constexpr double kCdivBmin = 0x1p-20, kCdivBmax = 0x1p20;
inline bool cdiv_divisor_ok(double b) {
    const double a = b < 0 ? -b : b;
    return b == 0. || !(a < 1e308) || (a >= kCdivBmin && a <= kCdivBmax);    // !(a < 1e308): inf or NaN
}
// most classes one workgroup stages in LDS (128 x 27 x 8 B = 27 KiB)
constexpr int kLdsClassMax = 128;
// elements per workgroup of the packed element kernel (shud_ele_packed.hip kEleBS): the tiles the host's edge-sharing
// assignment (shud_rhs.cpp, seg_first bits 26-29) pairs elements within
constexpr int kShareTile = 256;
// the parked DY tail of the packed element kernel (shud_ele_packed.hip LSP): kLspN doubles + one int per thread
// beside the ntab-double class + pow tables, taken while a workgroup's LDS stays <= kLspLdsMax (7 per CU)
constexpr int kLspN = 5;
constexpr size_t kLspLdsMax = 23296;
constexpr size_t lsp_lds_bytes(int ntab) { return (size_t)(ntab + kLspN * kShareTile) * 8 + kShareTile * 4; }
// pow_tab's log + exp tables (shud_pow_tab.h: 256 x 4 + 128 x 2 doubles; SHUD_PT_COMPACT: 128 x 2.5 + 128 x 2), staged in
// LDS after the class table (shud_rhs.cpp checks the sizes against the generated tables)
#ifndef SHUD_PT_COMPACT
#define SHUD_PT_COMPACT 1
#endif
constexpr int kPowTabLogDoubles = SHUD_PT_COMPACT ? 2 * 128 + 64 : 4 * 256;
constexpr int kPowTabDoubles = kPowTabLogDoubles + 2 * 128;
// most classes a 1024-thread workgroup stages in LDS ((560 x 33 + 1280) x 8 B = 154 KiB of the CU's 160 KiB: one
// workgroup per CU, 4 waves/SIMD) — models with 129..560 distinct parameter tuples
constexpr int kLdsClassMaxBig = 560;
// hybrid layout: at most this many class fields streamed per element (DevPacked::hv)
constexpr int kHybMax = 4;

struct DevPacked {
    const double *ctab;     // [ncls][CF_STRIDE] record-major: one class's fields share 2-3 cache lines; then, from
                            //   double pt_off (even: 16-B aligned), pow_tab's log and exp tables (kPowTabDoubles)
    int ncls;
    int pt_off, ntab;       // ntab = pt_off + kPowTabDoubles: the doubles a workgroup copies into LDS
    // hybrid layout (per-element-calibrated models): nh class fields streamed per element instead of read from the
    // class table — hv[hs * i + hslot1[f] - 1] for field f with hslot1[f] > 0 (hs = 1, 2 or 4 doubles per element)
    const double *hv;
    int nh, hs;
    int hnb;                // a streamed field is read for the neighbours too (macD, macKsatH, vAreaF, KsatH, Rough)
    signed char hslot1[CF_NPRIMARY];
    const double2 *zz;      // {z_surf, z_bottom}  (aquifer_depth == z_surf - z_bottom, checked at create)
    const int4 *meta;       // {nabr0, nabr1, nabr2, cf}: cf bits 0-7 iBC (int8), 8-9 iSS class,
                            //   10-15 #river segments, 16-30 class id, 31 lake element
                            //   (zz and meta.w are neighbour-gathered)
    const double2 *ged;     // [3][NE] edge-major {edge_j, dist2nabor_j}
    const double *area;
    int *seg_first;         // bits 0-30: first element-sorted segment of the element; bit 31: t_lai > ZERO
                            //   (f_etFlux's only use of LAI, MD_ET.cpp:381; rewritten with the step inputs)
    const double2 *sg_lc;   // [NS] element-sorted segments: {length, Cwr}
    const int *sg_r;        // [NS] the segment's (local) reach; with rrec [2 * local reaches]
    const double2 *rrec;    //   {depth, KsatH}, {BedThick, (BC column, 0) bits} per reach
    double2 *qseg2;         // [NS] {QsegSurf, QsegSub}, written by the element kernel (element-sorted)
    double2 *s_np;          // {net_prep, pot_evap}        step inputs (packed by shud_pack_step_kernel)
    double2 *s_tl;          // {pot_tran, ETP} (ETP: the eta > 2*ETP warning, MD_ET.cpp:391)
    double2 *s_fu;          // {fu_surf, fu_sub}            read only when not all ones
    double2 *cs[2];         // carried {u_satn, qEleE_IC}, ping-pong
    // reaches (owned first): 16-byte records
    // one 64-B record per reach {BottomWidth, bankslope | Length, BedSlope | Dist2DownStream, avgRough |
    // depth, (down, BC)}: everything a reach's own, its downstream's and its upstream reaches' QrivDown read,
    // so a neighbour reach costs one cache line instead of one line per field pair
    const double2 *rv;      // [4 * NR]
    // one 16-B index word per reach {first reach-sorted segment, #segments | code << 16, w2, w3}: code 0..2 =
    // that many upstream reaches, in w2, w3; code 3 = more, up_idx[w2 .. w2 + w3) (ascending global order)
    const int4 *rv_u;
    int riv_sb;             // segments per batch in the river kernel (6 or 8; choose_riv_sb)
    // QrivDown of every local reach (owned and ghost), computed once per eval by workgroups appended to the last
    // element launch (it depends on y only, MD_f.cpp:41-43); the river kernel then reads a reach's own QrivDown and
    // each upstream reach's from here (MD_f.cpp:236-240) instead of recomputing them from the reach records.
    // nullptr: off (SHUD_RHS_QD=0), the river kernel recomputes them
    double *qdown;          // [nqd]
    int nqd;
    int qd_pm, qd_pm_fold;  // where the QrivDown blocks sit in the element launch: after this many permille of its
                            //   element blocks (single launch / folded partition launch; SHUD_QD_POS[_FOLD])
    int lds_big;            // 1: 129..kLdsClassMaxBig classes take the 1024-thread LDS-table kernel (host dispatch)
};

struct DevDiag {                     // optional diagnostic outputs (ShudFluxOut), local numbering
    double *qele_surf, *qele_sub, *qele_surf_tot, *qele_sub_tot, *q_infil, *q_exfil, *q_recharge;
    double *q_es, *q_eu, *q_eg, *q_tu, *q_tg, *q_eta, *e_ic, *u_satn, *i_beta, *eff_kh;
    double *qe2r_surf, *qe2r_sub, *qriv_down, *qriv_up, *qriv_surf, *qriv_sub;
    double *q_lake_surf, *q_lake_sub, *q_lake_rivin, *q_lake_evap, *q_lake_prcp, *lake_toparea;
};

// ---- lakes (serial semantics, packed layout; partitioned: owned lakes) -------------------
// Lake elements carry bit 31 of DevPacked::meta.w; a non-lake element's edge whose neighbour has it is a
// bank edge (lakenabr, MD_Lake.cpp:131-143).  The element kernel writes each bank edge's fluxes; the lake
// kernel reduces them, the lake elements' PET/precipitation and the inflowing reaches in reference order.
struct DevLake {
    int nl;
    int y_off;                       // first lake stage in y / ydot (3 NE + NR)
    const int *lake_of;              // [NE] 0-based lake of a lake element
    double *bank_qs, *bank_qg;       // [3][NE] bank-edge surface weir Q and subsurface Q (before fu_Sub)
    const int *bathy_off;            // [nl+1] LakeBathymetry rows
    const double *bathy_y, *bathy_a;
    const int *ele_off, *ele_idx;    // lake elements of each lake, ascending
    const int *bank_off, *bank_pos;  // bank edges of each lake, element then edge order; pos = j*NE + i
    const int *rin_off, *rin_idx;    // reaches flowing into each lake (toLake), ascending
};

// state accessors: owned entities read the caller's y, ghosts read the halo buffers
struct YView {
    const double *y;                 // owned block layout [sf|us|gw|riv] over owned counts
    const double *gele;              // ghost elements, AoS records [3*k + {0,1,2}]
    const double *griv;              // ghost reaches
    int n_own, n_own_riv;
#ifdef __HIPCC__
    __device__ __forceinline__ double sf(int i) const { return i < n_own ? y[i] : gele[3 * (i - n_own)]; }
    __device__ __forceinline__ double us(int i) const { return i < n_own ? y[n_own + i] : gele[3 * (i - n_own) + 1]; }
    __device__ __forceinline__ double gw(int i) const { return i < n_own ? y[2 * n_own + i] : gele[3 * (i - n_own) + 2]; }
    __device__ __forceinline__ double riv(int r) const { return r < n_own_riv ? y[3 * n_own + r] : griv[r - n_own_riv]; }
    // GH = false: an unpartitioned handle has no ghosts, every index is owned (no select per access)
    template <bool GH> __device__ __forceinline__ double sf_(int i) const { return GH ? sf(i) : y[i]; }
    template <bool GH> __device__ __forceinline__ double us_(int i) const { return GH ? us(i) : y[n_own + i]; }
    template <bool GH> __device__ __forceinline__ double gw_(int i) const { return GH ? gw(i) : y[2 * n_own + i]; }
    template <bool GH> __device__ __forceinline__ double riv_(int r) const { return GH ? riv(r) : y[3 * n_own + r]; }
#endif
};

void launch_element_kernel(const DevMesh &m, const YView &Y, double *dy, int n_compute, int cur, int cur_e,
                           int mode, bool open, bool diag, const DevDiag &dg, hipStream_t s);
// with_qd: append the QrivDown workgroups (DevPacked::qdown) to this launch — only the last element launch of an
// eval, which runs after the halo; returns whether they were appended (the river kernel then reads the slots)
bool launch_element_kernel_packed(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int i0, int i1,
                                  int cur, int mode, bool open, bool diag, bool fu_unit, const DevDiag &dg,
                                  hipStream_t s, const DevLake *lake = nullptr, bool interior = false,
                                  bool with_qd = false);
// partitioned handles: the boundary + ghost elements [n_int, n_all) ride at the end of the interior element launch;
// their workgroups wait until the comm stream has published the halo (flag >= epoch; epoch 0 = stream-ordered)
struct HaloWait {
    const unsigned long long *flag;
    unsigned long long epoch;
    unsigned long long timeout;          // wall_clock64() ticks a boundary wave polls before SHUD_EF_HALO_WAIT
};
bool launch_element_kernel_packed_fold(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int n_int,
                                       int n_all, int cur, int mode, bool open, bool fu_unit, const DevDiag &dg,
                                       const HaloWait &hw, hipStream_t s, bool with_qd = false);
void launch_halo_flag(unsigned long long *flag, unsigned long long epoch, hipStream_t s);
// test hooks (shud_rhs_debug_halo): a one-lane spin of `ticks` wall-clock ticks, and a plain vector copy (the
// stand-in for RCCL's receive kernels writing the ghost buffers), both on the comm stream
void launch_spin(unsigned long long ticks, hipStream_t s);
void launch_copy_f64(double *dst, const double *src, size_t n, hipStream_t s);
// qd: the eval's element launch wrote DevPacked::qdown
void launch_river_kernel_packed(const DevMesh &m, const DevPacked &p, const YView &Y, double *dy, int mode,
                                bool diag, const DevDiag &dg, hipStream_t s, bool qd = false);
void launch_lake_kernel(const DevMesh &m, const DevPacked &p, const DevLake &L, const YView &Y, double *dy,
                        bool diag, const DevDiag &dg, hipStream_t s);
void launch_pack_step_kernel(const DevMesh &m, const DevPacked &p, int n, int cur, unsigned what, hipStream_t s);
void launch_river_kernel(const DevMesh &m, const YView &Y, double *dy, int mode, bool diag,
                         const DevDiag &dg, hipStream_t s);
void launch_pack_kernel(const double *y, int n_own, int n_own_riv, const int *eidx, int ne, const int *ridx,
                        int nr, double *ebuf, double *rbuf, hipStream_t s);

}  // namespace shud
