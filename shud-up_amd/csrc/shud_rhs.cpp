// shud_rhs.cpp — host runtime behind include/shud_rhs.h (C-ABI).
//
// Replaces the reference RHS callback f() (src/Model/f.cpp:2-32) and the Model_Data arrays it works
// on (src/ModelData/Model_Data.hpp:111-208).  The handle owns device SoA copies of the static mesh and
// parameters (uploaded once, shud_rhs_create), of the per-ET-step inputs (shud_rhs_set_step_inputs),
// and of the carried RHS state (qEleE_IC, u_satn — ping-pong buffers so a diagnostic replay sees the
// exact inputs of the last call).  y / ydot are borrowed per call.
//
// Multi-GPU: one process per GPU, each handle holds its partition (owned + ghost
// entities); ghost states arrive by one grouped RCCL send/recv exchange (= ncclAllToAllv restricted
// to the peers that share a boundary) per eval, before the element kernel.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "shud_handle.h"
#define SHUD_PT_HOST_TABLES           // the pow_tab tables as host arrays, uploaded with the class table
#include "shud_pow_tab.h"

using namespace shud;

namespace {
thread_local std::string g_last_error;
}  // namespace

// Event scopes.  Every event here orders work between queues of one device (the comm stream's pack / exchange and
// the main stream's kernels) or times kernels: a device-scope release is enough for both, and the default
// system-scope release writes the L2's dirty lines back to HBM at every record (profiles/r03/ev_scope/).  RCCL's
// own kernels on s_comm complete before ev_comm, which then publishes their writes to this device's other queues.
static constexpr unsigned kEvSync = hipEventDisableSystemFence;
static constexpr unsigned kEvTime = hipEventReleaseToDevice;

int shud_fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

// Run-time switches read from the environment (A/B measurements and tests).  Each is parsed strictly: a value that is
// not an integer in [lo, hi] is ignored with a warning, and a value that takes effect is announced once per process on
// stderr — a stray variable in a user's environment cannot silently change kernel selection.
static int env_knob(const char *name, int def, int lo, int hi) {
    const char *v = getenv(name);
    if (!v || !*v) return def;
    char *end = nullptr;
    const long x = strtol(v, &end, 10);
    static std::vector<std::string> said;
    const bool first = std::find(said.begin(), said.end(), std::string(name)) == said.end();
    if (first) said.push_back(name);
    if (*end || x < lo || x > hi) {
        if (first) fprintf(stderr, "shud_rhs: ignoring %s=%s (expected an integer in [%d, %d])\n", name, v, lo, hi);
        return def;
    }
    if (first && x != def) fprintf(stderr, "shud_rhs: %s=%ld in effect (default %d)\n", name, x, def);
    return (int)x;
}

int shud_reset_err(shud_rhs *h) {
    DevErr z{};
    z.flags = 0;
    for (int k = 0; k < 8; k++) z.first_index[k] = INT_MAX;
    z.n_warn = 0;
    z.warn = h->d_warn;
    HIP_TRY(hipMemsetAsync(h->d_warn, 0, kWarnSlots * kWarnStride * sizeof(unsigned long long), h->stream));
    HIP_TRY(hipMemcpyAsync(h->d_err, &z, sizeof(DevErr), hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return 0;
}

extern "C" int shud_rhs_abi_version(void) { return SHUD_RHS_ABI_VERSION; }
extern "C" const char *shud_rhs_last_error_string(void) { return g_last_error.c_str(); }

// ---------------------------------------------------------------------------------------------
// create
// ---------------------------------------------------------------------------------------------
// Segments per batch in the river kernel: a wave issues SB flux gathers + its position loads per batch and runs
// as many batches as its lane with the most segments needs; pick the batch size that issues fewer loads over the
// owned reaches' 64-reach waves (6 or 8: 16-B + 8-B or two 16-B position loads)
static int choose_riv_sb(const int *nseg, int nr) {
    long long cost6 = 0, cost8 = 0;
    for (int w = 0; w < nr; w += 64) {
        int mx = 0;
        for (int r = w; r < nr && r < w + 64; r++) mx = std::max(mx, nseg[r]);
        cost6 += (long long)((mx + 5) / 6) * (6 + 2);
        cost8 += (long long)((mx + 7) / 8) * (8 + 2);
    }
    return cost6 < cost8 ? 6 : 8;
}

static int build_packed(shud_rhs *h, const ShudMeshSoA *m, const ShudParamsSoA *p, const std::vector<int> &eflags,
                        const std::vector<int> &seg_off, const std::vector<int> &up_off,
                        const std::vector<int> &up_idx);

static int build_lakes(shud_rhs *h, const ShudMeshSoA *m, const ShudPartition *part);
static int build(shud_rhs *h, const ShudMeshSoA *m, const ShudParamsSoA *p, const ShudRhsOptions *opt,
                 const ShudPartition *part) {
    const int NE = m->num_ele, NR = m->num_riv, NS = m->num_seg;
    if (NE < 0 || NR < 0 || NS < 0) return shud_fail(SHUD_ERR_ARG, "negative sizes");
    h->NE = NE; h->NR = NR; h->NS = NS;
    h->mode = opt ? opt->mode : SHUD_MODE_SERIAL;
    if (h->mode != SHUD_MODE_SERIAL && h->mode != SHUD_MODE_OMP) return shud_fail(SHUD_ERR_ARG, "bad mode %d", h->mode);
    h->check_errors = opt ? opt->check_errors != 0 : true;
    h->open = (m->close_boundary == 0);
    h->device = opt ? opt->device : 0;
    h->n_own = part ? part->n_own_ele : NE;
    h->n_segghost = part ? part->n_segghost_ele : 0;
    h->n_own_riv = part ? part->n_own_riv : NR;
    if (h->n_own < 0 || h->n_own + h->n_segghost > NE || h->n_own_riv < 0 || h->n_own_riv > NR)
        return shud_fail(SHUD_ERR_ARG, "partition counts inconsistent with mesh sizes");

    // ---- validation (the reference exits on these at run time; we reject them up front) ----
    if (!m->nabr || !m->area || !m->z_surf || !m->z_bottom || !m->edge || !m->dist2nabor || !m->avg_rough)
        return shud_fail(SHUD_ERR_ARG, "missing element geometry array");
    if (h->open && (!m->dist2edge || !m->rough)) return shud_fail(SHUD_ERR_ARG, "open boundary needs dist2edge and rough");
    if (NR && (!m->riv_down || !m->riv_length || !m->riv_bed_slope || !m->riv_dist2down || !m->riv_avg_rough ||
               !m->riv_depth || !m->riv_bottom_width || !m->riv_bankslope || !m->riv_ksath || !m->riv_bedthick))
        return shud_fail(SHUD_ERR_ARG, "missing river array");
    if (NS && (!m->seg_ele || !m->seg_riv || !m->seg_length || !m->seg_cwr)) return shud_fail(SHUD_ERR_ARG, "missing segment array");
    const double *pp[17] = {p->aquifer_depth, p->macD, p->macKsatH, p->geo_vAreaF, p->KsatH, p->KsatV,
                            p->infKsatV, p->hAreaF, p->macKsatV, p->ThetaS, p->ThetaR, p->Beta,
                            p->infD, p->Sy, p->RzD, p->VegFrac, p->ImpAF};
    for (int k = 0; k < 17; k++)
        if (!pp[k]) return shud_fail(SHUD_ERR_ARG, "missing parameter array #%d", k);
    for (long long q = 0; q < 3LL * NE; q++)
        if (m->nabr[q] < -1 || m->nabr[q] >= NE) return shud_fail(SHUD_ERR_ARG, "nabr[%lld]=%d out of range", q, m->nabr[q]);
    // lakes: on when any iLake > 0 (MD_readin.cpp:262-263); serial semantics, packed layout.  Partitioned:
    // the plan (shud_partition.h) puts a lake's elements and bank elements on one rank and numbers its lakes
    // locally, so every lake sum is formed from owned elements and owned or ghost reaches
    if (m->ilake)
        for (int i = 0; i < NE; i++)
            if (m->ilake[i] > 0) h->lakeon = true;
    if (h->lakeon) {
        if (h->mode != SHUD_MODE_SERIAL)
            return shud_fail(SHUD_ERR_UNSUPPORTED, "lakes: the OMP path has no lake physics (MD_f_omp.cpp)");
        h->NL = m->num_lake;
        if (h->NL <= 0 || !m->lake_bathy_off || !m->lake_bathy_y || !m->lake_bathy_a)
            return shud_fail(SHUD_ERR_ARG, "lake elements present but no lake bathymetry (num_lake %d)", m->num_lake);
        for (int l = 0; l < h->NL; l++)
            if (m->lake_bathy_off[l + 1] <= m->lake_bathy_off[l])
                return shud_fail(SHUD_ERR_ARG, "lake %d has an empty bathymetry table", l + 1);
        for (int i = 0; i < NE; i++)
            if (m->ilake[i] > h->NL) return shud_fail(SHUD_ERR_ARG, "element %d: iLake %d > num_lake", i, m->ilake[i]);
    }
    for (int r = 0; r < NR; r++) {
        int d = m->riv_down[r];
        if (h->lakeon && d <= -4) {               // toLake = (-3 - down) - 1 (MD_Lake.cpp:46-50)
            if ((-3 - d) - 1 >= h->NL)
                return shud_fail(SHUD_ERR_ARG, "reach %d flows into lake %d > num_lake", r, -3 - d);
            continue;
        }
        if (d >= NR || (d < 0 && d < -4))
            return shud_fail(SHUD_ERR_ARG, "Fatal Error: River Routing Boundary Condition Type Is Wrong! (reach %d down %d)", r, d);
    }
    // reach codes as the kernels see them: a reach into a lake uses the zero-depth-gradient formula (-3)
    std::vector<int> rdown(m->riv_down, m->riv_down + NR);
    if (h->lakeon)
        for (int r = 0; r < NR; r++)
            if (rdown[r] <= -4) rdown[r] = -3;
    for (int s = 0; s < NS; s++)
        if (m->seg_ele[s] < 0 || m->seg_ele[s] >= NE || m->seg_riv[s] < 0 || m->seg_riv[s] >= NR)
            return shud_fail(SHUD_ERR_ARG, "segment %d references element/reach out of range", s);

    // ---- packed element flags, BC column maxima ----
    std::vector<int> eflags(NE);
    for (int i = 0; i < NE; i++) {
        int ibc = m->ibc ? m->ibc[i] : 0, iss = m->iss ? m->iss[i] : 0;
        if (ibc < -32768 || ibc > 32767) return shud_fail(SHUD_ERR_ARG, "iBC out of range at %d", i);
        eflags[i] = (ibc & 0xffff) | ((iss > 0 ? 1 : iss < 0 ? 2 : 0) << 16);
        if (ibc > 0) h->max_col[0] = std::max(h->max_col[0], ibc);
        if (ibc < 0) h->max_col[1] = std::max(h->max_col[1], -ibc);
    }
    std::vector<int> rbc(NR, 0);
    for (int r = 0; r < NR; r++) {
        rbc[r] = m->riv_bc ? m->riv_bc[r] : 0;
        if (rbc[r] > 0) h->max_col[2] = std::max(h->max_col[2], rbc[r]);
        if (rbc[r] < 0) h->max_col[3] = std::max(h->max_col[3], -rbc[r]);
    }

    // ---- segment CSR by element (stable: ascending reference index inside an element) ----
    const int ncomp = h->n_own + h->n_segghost;
    std::vector<int> order(NS);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return m->seg_ele[a] < m->seg_ele[b]; });
    std::vector<int> seg_off(NE + 1, 0), seg_riv(NS), pos_of(NS);
    std::vector<double> seg_len(NS), seg_cwr(NS);
    for (int s = 0; s < NS; s++) seg_off[m->seg_ele[s] + 1]++;
    for (int i = 0; i < NE; i++) seg_off[i + 1] += seg_off[i];
    for (int k = 0; k < NS; k++) {
        int s = order[k];
        seg_riv[k] = m->seg_riv[s];
        seg_len[k] = m->seg_length[s];
        seg_cwr[k] = m->seg_cwr[s];
        pos_of[s] = k;
    }
    // only elements < ncomp compute their segments; segments of pure ghosts must not be needed
    for (int s = 0; s < NS; s++)
        if (m->seg_ele[s] >= ncomp && m->seg_riv[s] < h->n_own_riv)
            return shud_fail(SHUD_ERR_ARG, "segment %d of an owned reach belongs to a non-computed ghost element", s);
    h->seg_perm = order;
    // ---- partitioned: owned elements [0, n_int) read no ghost data (all lateral neighbours owned, all their
    // segments' reaches owned); they run while the halo exchange is in flight (eval_device) ----
    h->n_int = 0;
    if (part) {
        int i = 0;
        for (; i < h->n_own; i++) {
            bool dep = false;
            for (int j = 0; j < 3 && !dep; j++) dep = m->nabr[(size_t)j * NE + i] >= h->n_own;
            for (int k = seg_off[i]; k < seg_off[i + 1] && !dep; k++) dep = seg_riv[k] >= h->n_own_riv;
            if (dep) break;
        }
        h->n_int = i;
    }
    // ---- per owned reach: its segments (ascending reference order) and upstream reaches ----
    std::vector<int> rseg_off(h->n_own_riv + 1, 0), rseg_pos;
    for (int s = 0; s < NS; s++)
        if (m->seg_riv[s] < h->n_own_riv) rseg_off[m->seg_riv[s] + 1]++;
    for (int r = 0; r < h->n_own_riv; r++) rseg_off[r + 1] += rseg_off[r];
    rseg_pos.resize(rseg_off[h->n_own_riv]);
    {
        std::vector<int> fillp(rseg_off.begin(), rseg_off.end() - 1);
        for (int s = 0; s < NS; s++) {
            int r = m->seg_riv[s];
            if (r < h->n_own_riv) rseg_pos[fillp[r]++] = pos_of[s];
        }
        rseg_pos.resize(rseg_pos.size() + 8, 0);   // the river kernel may read a whole 8-position batch past the end
    }
    std::vector<int> up_off(h->n_own_riv + 1, 0), up_idx;
    for (int r = 0; r < NR; r++) {
        int d = m->riv_down[r];
        if (d >= 0 && d < h->n_own_riv) up_off[d + 1]++;
    }
    for (int r = 0; r < h->n_own_riv; r++) up_off[r + 1] += up_off[r];
    up_idx.resize(up_off[h->n_own_riv]);
    {
        // ascending reach order (MD_f.cpp:236-240); in a partition, ascending GLOBAL reach id
        std::vector<int> fillp(up_off.begin(), up_off.end() - 1);
        for (int r = 0; r < NR; r++) {
            int d = m->riv_down[r];
            if (d >= 0 && d < h->n_own_riv) up_idx[fillp[d]++] = r;
        }
        if (part && part->riv_gid)
            for (int r = 0; r < h->n_own_riv; r++)
                std::sort(up_idx.begin() + up_off[r], up_idx.begin() + up_off[r + 1],
                          [&](int a, int b) { return part->riv_gid[a] < part->riv_gid[b]; });
    }

    // ---- device ----
    HIP_TRY(hipSetDevice(h->device));
    if (opt && opt->stream) {
        h->stream = (hipStream_t)opt->stream;
    } else {
        HIP_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        h->own_stream = true;
    }
    DevMesh &d = h->dm;
    d.num_ele = NE;
    int rc = 0;
#define UP(field, src, n) if ((rc = h->upload(&field##_w, src, n))) return rc; d.field = field##_w
    {
        int *nabr_w, *eflags_w;
        double *area_w, *z_surf_w, *z_bottom_w, *depression_w, *edge_w, *dist2nabor_w, *dist2edge_w, *avg_rough_w, *rough_w;
        UP(nabr, m->nabr, 3 * (size_t)NE);
        UP(eflags, eflags.data(), NE);
        UP(area, m->area, NE);
        UP(z_surf, m->z_surf, NE);
        UP(z_bottom, m->z_bottom, NE);
        if ((rc = h->upload_fill(&depression_w, m->depression, NE, 0.0002))) return rc;
        d.depression = depression_w;
        UP(edge, m->edge, 3 * (size_t)NE);
        UP(dist2nabor, m->dist2nabor, 3 * (size_t)NE);
        UP(avg_rough, m->avg_rough, 3 * (size_t)NE);
        UP(dist2edge, h->open ? m->dist2edge : (const double *)nullptr, h->open ? 3 * (size_t)NE : 1);
        UP(rough, h->open ? m->rough : (const double *)nullptr, h->open ? (size_t)NE : 1);
    }
    {
        double *aq_w, *macD_w, *macKsatH_w, *vAreaF_w, *KsatH_w, *KsatV_w, *infKsatV_w, *hAreaF_w, *macKsatV_w;
        double *ThetaS_w, *ThetaR_w, *Beta_w, *infD_w, *Sy_w, *RzD_w, *VegFrac_w, *ImpAF_w;
        UP(aq, p->aquifer_depth, NE); UP(macD, p->macD, NE); UP(macKsatH, p->macKsatH, NE);
        UP(vAreaF, p->geo_vAreaF, NE); UP(KsatH, p->KsatH, NE); UP(KsatV, p->KsatV, NE);
        UP(infKsatV, p->infKsatV, NE); UP(hAreaF, p->hAreaF, NE); UP(macKsatV, p->macKsatV, NE);
        UP(ThetaS, p->ThetaS, NE); UP(ThetaR, p->ThetaR, NE); UP(Beta, p->Beta, NE); UP(infD, p->infD, NE);
        UP(Sy, p->Sy, NE); UP(RzD, p->RzD, NE); UP(VegFrac, p->VegFrac, NE); UP(ImpAF, p->ImpAF, NE);
    }
    {
        double *net_prep_w, *pot_evap_w, *pot_tran_w, *etp_w, *lai_w, *fu_surf_w, *fu_sub_w, *ugw_stale_w, *prcp_w;
        UP(prcp, (const double *)nullptr, NE);
        UP(net_prep, (const double *)nullptr, NE); UP(pot_evap, (const double *)nullptr, NE); UP(pot_tran, (const double *)nullptr, NE); UP(etp, (const double *)nullptr, NE);
        UP(lai, (const double *)nullptr, NE);
        if ((rc = h->upload_fill(&fu_surf_w, (const double *)nullptr, NE, 1.0))) return rc;
        d.fu_surf = fu_surf_w;
        if ((rc = h->upload_fill(&fu_sub_w, (const double *)nullptr, NE, 1.0))) return rc;
        d.fu_sub = fu_sub_w;
        UP(ugw_stale, (const double *)nullptr, NE);
        for (int k = 0; k < 2; k++) {
            if ((rc = h->upload(&d.e_ic[k], (const double *)nullptr, NE))) return rc;
            if ((rc = h->upload(&d.u_satn[k], (const double *)nullptr, NE))) return rc;
        }
    }
    for (int k = 0; k < 4; k++) {
        h->tab_len[k] = h->max_col[k] + 1;
        if ((rc = h->upload(&h->d_tab[k], (const double *)nullptr, h->tab_len[k]))) return rc;
    }
    d.eybc = h->d_tab[0]; d.eqbc = h->d_tab[1]; d.rybc = h->d_tab[2]; d.rqbc = h->d_tab[3];
    {
        int *seg_off_w, *seg_riv_w;
        double *seg_len_w, *seg_cwr_w;
        UP(seg_off, seg_off.data(), NE + 1);
        UP(seg_riv, seg_riv.data(), NS);
        UP(seg_len, seg_len.data(), NS);
        UP(seg_cwr, seg_cwr.data(), NS);
        if ((rc = h->upload(&d.qseg_surf, (const double *)nullptr, NS))) return rc;
        if ((rc = h->upload(&d.qseg_sub, (const double *)nullptr, NS))) return rc;
    }
    {
        int *riv_down_w, *riv_bc_w, *up_off_w, *up_idx_w, *rseg_off_w, *rseg_pos_w;
        double *riv_len_w, *riv_slope_w, *riv_d2down_w, *riv_avg_rough_w, *riv_depth_w, *riv_bw_w,
            *riv_bankslope_w, *riv_ksath_w, *riv_bedthick_w;
        UP(riv_down, rdown.data(), NR); UP(riv_bc, rbc.data(), NR);
        UP(riv_len, m->riv_length, NR); UP(riv_slope, m->riv_bed_slope, NR); UP(riv_d2down, m->riv_dist2down, NR);
        UP(riv_avg_rough, m->riv_avg_rough, NR); UP(riv_depth, m->riv_depth, NR); UP(riv_bw, m->riv_bottom_width, NR);
        UP(riv_bankslope, m->riv_bankslope, NR); UP(riv_ksath, m->riv_ksath, NR); UP(riv_bedthick, m->riv_bedthick, NR);
        UP(up_off, up_off.data(), up_off.size()); UP(up_idx, up_idx.data(), up_idx.size());
        UP(rseg_off, rseg_off.data(), rseg_off.size()); UP(rseg_pos, rseg_pos.data(), rseg_pos.size());
    }
#undef UP
    if ((rc = build_packed(h, m, p, eflags, seg_off, up_off, up_idx))) return rc;
    if (h->lakeon && (rc = build_lakes(h, m, part))) return rc;
    if ((rc = h->dalloc(&h->d_err, 1))) return rc;
    if ((rc = h->dalloc(&h->d_warn, (size_t)kWarnSlots * kWarnStride))) return rc;
    d.err = h->d_err;
    HIP_TRY(hipHostMalloc((void **)&h->h_err, sizeof(DevErr), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void **)&h->h_warn, kWarnSlots * kWarnStride * sizeof(unsigned long long),
                          hipHostMallocDefault));
    if ((rc = shud_reset_err(h))) return rc;
    const size_t ny = 3 * (size_t)h->n_own + h->n_own_riv + h->NL;
    if ((rc = h->dalloc(&h->d_y, ny))) return rc;
    if ((rc = h->dalloc(&h->d_ydot, ny))) return rc;
    if ((rc = h->dalloc(&h->d_scratch_dy, ny))) return rc;
    return 0;
}

// Distinct fixed-length tuples of 64-bit words (bit patterns: two doubles are the same key when their bits are), each
// numbered in first-seen order: open addressing over a power-of-two slot table, the tuples stored flat.  The class
// search below runs it over every element several times per handle (one pass per candidate hybrid field set), so it
// avoids per-element heap keys (std::string keys of 144 B cost seconds at 10M elements).
class TupleSet {
  public:
    explicit TupleSet(int k) : k_(k), slots_(1024, -1) {}     // k <= 32
    int size() const { return (int)(words_.size() / k_); }
    const uint64_t *tuple(int id) const { return &words_[(size_t)id * k_]; }
    // id of the tuple at p (k 8-byte words, any type: copied as bits), inserted if new
    int insert(const void *p) {
        uint64_t t[32];
        memcpy(t, p, (size_t)k_ * 8);
        if ((size_t)(size() + 1) * 2 > slots_.size()) grow();
        size_t j = hash(t) & (slots_.size() - 1);
        for (;; j = (j + 1) & (slots_.size() - 1)) {
            const int id = slots_[j];
            if (id < 0) break;
            if (!memcmp(tuple(id), t, (size_t)k_ * 8)) return id;
        }
        const int id = size();
        slots_[j] = id;
        words_.insert(words_.end(), t, t + k_);
        return id;
    }

  private:
    uint64_t hash(const uint64_t *t) const {
        uint64_t h = 0x9e3779b97f4a7c15ull;
        for (int q = 0; q < k_; q++) {                  // splitmix64 finaliser per word, chained
            uint64_t x = t[q] + h;
            x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
            x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
            h = x ^ (x >> 31);
        }
        return h;
    }
    void grow() {
        std::vector<int> old;
        old.swap(slots_);
        slots_.assign(old.size() * 2, -1);
        for (int id : old) {
            if (id < 0) continue;
            size_t j = hash(tuple(id)) & (slots_.size() - 1);
            while (slots_[j] >= 0) j = (j + 1) & (slots_.size() - 1);
            slots_[j] = id;
        }
    }
    int k_;
    std::vector<int> slots_;
    std::vector<uint64_t> words_;
};

// Packed class layout (shud_dev.h DevPacked).  Returns 0 with h->packed set, 0 with h->packed clear when
// the mesh does not qualify (the SoA kernel is used), or an error code.
static int build_packed(shud_rhs *h, const ShudMeshSoA *m, const ShudParamsSoA *p, const std::vector<int> &eflags,
                        const std::vector<int> &seg_off, const std::vector<int> &up_off,
                        const std::vector<int> &up_idx) {
    if (!env_knob("SHUD_RHS_PACKED", 1, 0, 1)) return 0;         // 0: the SoA kernel (tests, A/B)
    const int NE = m->num_ele;
    if (!m->rough || NE == 0) return 0;
    // avgRough must be the reference's 0.5*(Rough_i + Rough_nabr) / Rough_i (Element.cpp:249-265).  Owned
    // elements only: a ghost never computes lateral fluxes, and its neighbours outside the rank's local mesh
    // appear as boundary edges (-1) while its avgRough is the global one
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < h->n_own; i++) {
            const int nb = m->nabr[(size_t)j * NE + i];
            const double want = nb >= 0 ? 0.5 * (m->rough[i] + m->rough[nb]) : m->rough[i];
            if (!(m->avg_rough[(size_t)j * NE + i] == want)) return 0;
        }
    // identities the packed record relies on (else the SoA kernel runs): AquiferDepth == z_surf - z_bottom
    // (InitElement after rmSinks, Model_Data.cpp:262-264), |iBC| fits int8, <= 63 segments per element
    // the packed kernel addresses its element / segment streams with 32-bit byte offsets (at(), shud_ele_packed.hip)
    if ((uint64_t)48 * NE >= (1ull << 32) || (uint64_t)48 * m->num_seg >= (1ull << 32) ||
        (uint64_t)24 * NE + 8ull * m->num_riv >= (1ull << 32))
        return 0;
    {                                                               // 16-bit segment count in the reach index word
        std::vector<int> cnt(m->num_riv, 0);
        for (int s = 0; s < m->num_seg; s++)
            if (++cnt[m->seg_riv[s]] > 0xffff) return 0;
    }
    for (int i = 0; i < NE; i++) {
        if (!(p->aquifer_depth[i] == m->z_surf[i] - m->z_bottom[i])) return 0;
        const int ibc = m->ibc ? m->ibc[i] : 0;
        if (ibc > 127 || ibc < -127) return 0;
        if (seg_off[i + 1] - seg_off[i] > 63) return 0;
    }
    // distinct parameter tuples -> class ids
    std::vector<std::vector<double>> table;           // [class][field]
    std::vector<int> cls(NE);
    const double dep_default = 0.0002;
    auto prim = [&](int i, std::vector<double> &r) {
        r[CF_macD] = p->macD[i]; r[CF_macKsatH] = p->macKsatH[i]; r[CF_vAreaF] = p->geo_vAreaF[i];
        r[CF_KsatH] = p->KsatH[i]; r[CF_KsatV] = p->KsatV[i]; r[CF_infKsatV] = p->infKsatV[i];
        r[CF_hAreaF] = p->hAreaF[i]; r[CF_macKsatV] = p->macKsatV[i]; r[CF_ThetaS] = p->ThetaS[i];
        r[CF_ThetaR] = p->ThetaR[i]; r[CF_Beta] = p->Beta[i]; r[CF_infD] = p->infD[i]; r[CF_Sy] = p->Sy[i];
        r[CF_RzD] = p->RzD[i]; r[CF_VegFrac] = p->VegFrac[i]; r[CF_ImpAF] = p->ImpAF[i];
        r[CF_depression] = m->depression ? m->depression[i] : dep_default;
        r[CF_rough] = m->rough[i];
    };
    // the distinct tuples of the fields outside `mask` (mask fields zeroed), counting stops past `cap`
    auto count_tuples = [&](uint32_t mask, int cap) {
        TupleSet seen(CF_NPRIMARY);
        std::vector<double> r(CF_NPRIMARY);
        for (int i = 0; i < NE && seen.size() <= cap; i++) {
            prim(i, r);
            for (int f = 0; f < CF_NPRIMARY; f++)
                if (mask >> f & 1) r[f] = 0.;
            seen.insert(r.data());
        }
        return seen.size();
    };
    // classes of the fields outside `mask` (mask fields zeroed); false past 32768 classes
    auto build_classes = [&](uint32_t mask) {
        table.clear();
        TupleSet ids(CF_NPRIMARY);
        std::vector<double> r(CF_NPRIMARY);
        for (int i = 0; i < NE; i++) {
            prim(i, r);
            for (int f = 0; f < CF_NPRIMARY; f++)
                if (mask >> f & 1) r[f] = 0.;
            const int id = ids.insert(r.data());
            if (id == (int)table.size()) {
                if (id >= 32768) return false;
                table.push_back(r);
            }
            cls[i] = id;
        }
        return true;
    };
    const bool fits = build_classes(0);
    // Hybrid layout (per-element-calibrated models): when the full tuples exceed one workgroup's LDS table, stream up
    // to kHybMax fields per element (8 B each) and keep the rest in the LDS class table — the fields that split the
    // classes of the non-streamable fields the most first, among those the kernel reads directly (no host-derived
    // class constant depends on them; Sy's reciprocal is replaced by the IEEE division, the same bits).
    // SHUD_RHS_HYB=0: off (A/B); =2: KsatH streamed even when the classes fit (timing the hybrid path on any model).
    uint32_t hmask = 0;
    const int hyb = env_knob("SHUD_RHS_HYB", 1, 0, 2);
    if (hyb == 2 && !h->lakeon) {
        hmask = 1u << CF_KsatH;
    } else {
        const uint32_t streamable = 1u << CF_macD | 1u << CF_macKsatH | 1u << CF_vAreaF | 1u << CF_KsatH |
                                    1u << CF_KsatV | 1u << CF_Sy | 1u << CF_RzD | 1u << CF_depression | 1u << CF_rough;
        if (!h->lakeon && hyb != 0 && (!fits || (int)table.size() > kLdsClassMax) &&
            count_tuples(streamable, kLdsClassMax) <= kLdsClassMax) {
            // base classes: the tuples of the fields that cannot be streamed; then, per streamable field, how many
            // (base class, value) pairs it makes — the fields that split the base classes most are streamed first
            TupleSet bid(CF_NPRIMARY);
            std::vector<int> base(NE);
            std::vector<double> r(CF_NPRIMARY);
            for (int i = 0; i < NE; i++) {
                prim(i, r);
                for (int f = 0; f < CF_NPRIMARY; f++)
                    if (streamable >> f & 1) r[f] = 0.;
                base[i] = bid.insert(r.data());
            }
            std::vector<std::pair<size_t, int>> split;       // (distinct (base, value) pairs, field)
            for (int f = 0; f < CF_NPRIMARY; f++) {
                if (!(streamable >> f & 1)) continue;
                TupleSet pairs(2);                           // (base class, field value bits)
                for (int i = 0; i < NE && pairs.size() <= 1 << 20; i++) {
                    prim(i, r);
                    uint64_t key[2];
                    key[0] = (uint64_t)base[i];
                    memcpy(&key[1], &r[f], 8);
                    pairs.insert(key);
                }
                if (pairs.size() > bid.size()) split.push_back({(size_t)pairs.size(), f});
            }
            std::stable_sort(split.begin(), split.end(),
                             [](const std::pair<size_t, int> &a, const std::pair<size_t, int> &b) {
                                 return a.first > b.first;
                             });
            for (int k = 0; k < (int)split.size() && k < kHybMax; k++) {
                hmask |= 1u << split[k].second;
                if (count_tuples(hmask, kLdsClassMax) <= kLdsClassMax) break;
                if (k + 1 == kHybMax || k + 1 == (int)split.size()) hmask = 0;   // not enough: no hybrid layout
            }
        }
    }
    if (hmask) {
        if (!build_classes(hmask)) return 0;
    } else if (!fits) {
        return 0;
    }
    const int ncls = (int)table.size();
    // beyond what a 256-thread workgroup's LDS copy holds (128 classes) the class table goes to 1024-thread
    // workgroups (up to kLdsClassMaxBig = 600 classes, one per CU); beyond that the lookups would be dependent
    // L2 trips.  Measured on syn-10M (tools/class_sweep.py, profiles/r02/class_sweep.log): element kernel 0.65 ms
    // with 33 classes in LDS; from L2 0.83 ms at 132 classes, 1.21 at 495, 1.49 at 1,980, 1.66 at 13,200; the
    // SoA kernel 1.09 ms at any count -> SoA above 600 (SHUD_RHS_L2_CLASS=1 forces the L2 table at any count and
    // disables the 1024-thread LDS kernel, =0 forces SoA above 128: A/B and bench.py many_class)
    const int l2 = env_knob("SHUD_RHS_L2_CLASS", -1, 0, 1);
    const int l2_max = l2 == 1 ? 32768 : l2 == 0 ? kLdsClassMax : kLdsClassMaxBig;
    if (ncls > l2_max) return 0;
    h->dp.lds_big = l2 == 1 ? 0 : 1;
    std::vector<double> ctab((size_t)CF_STRIDE * ncls, 0.0);
    for (int c = 0; c < ncls; c++) {
        std::vector<double> &t = table[c];
        t.resize(CF_COUNT);
        // same expressions, same order as the element kernel (-ffp-contract=off on both sides)
        t[CF_fcmr] = t[CF_ThetaS] * 0.75 - t[CF_ThetaR];
        t[CF_dTh] = t[CF_ThetaS] - t[CF_ThetaR];
        t[CF_ex1] = t[CF_Beta] / (t[CF_Beta] - 1.);
        t[CF_ex2] = (t[CF_Beta] - 1.) / t[CF_Beta];
        // the packed kernel's satKfun uses pow_tab (positive bases, finite exponents: shud_physics.h);
        // any other Beta keeps the SoA layout, whose kernel calls the full pow for it
        if (!(t[CF_Beta] > 1.) || !std::isfinite(t[CF_ex1]) || !std::isfinite(t[CF_ex2])) return 0;
        t[CF_pj] = 1. - t[CF_ImpAF];
        t[CF_omh] = 1. - t[CF_hAreaF];
        t[CF_kmax] = t[CF_infKsatV] * (1. - t[CF_hAreaF]) + t[CF_macKsatV] * t[CF_hAreaF];
        t[CF_ekA] = t[CF_infKsatV] * (1. - t[CF_hAreaF]);
        t[CF_ekB] = t[CF_hAreaF] * t[CF_macKsatV];
        // cdiv's range (shud_dev.h cdiv_divisor_ok); otherwise plain divisions in the SoA kernel
        if (!cdiv_divisor_ok(t[CF_fcmr]) || !cdiv_divisor_ok(t[CF_dTh]) || !cdiv_divisor_ok(t[CF_infD]) ||
            !cdiv_divisor_ok(t[CF_Sy]))
            return 0;
        t[CF_r_fcmr] = 1. / t[CF_fcmr];
        t[CF_r_dTh] = 1. / t[CF_dTh];
        t[CF_r_infD] = 1. / t[CF_infD];
        t[CF_r_Sy] = 1. / t[CF_Sy];
        for (int f = 0; f < CF_COUNT; f++)
            if (cf_stored(f)) ctab[(size_t)c * CF_STRIDE + cf_pos(f)] = t[f];
    }
    // pow_tab's tables (shud_pow_tab.h) after the class table, 16-B aligned: one buffer, one LDS copy per workgroup
    const int pt_off = ((int)ctab.size() + 1) & ~1;
    ctab.resize((size_t)pt_off + kPowTabDoubles, 0.0);
#if SHUD_PT_COMPACT
    static_assert(sizeof shud_pt_clogtab == 8 * kPowTabLogDoubles, "pow_tab");
    memcpy(&ctab[pt_off], shud_pt_clogtab, sizeof shud_pt_clogtab);
#else
    static_assert(kPowTabLogDoubles == 4 * SHUD_PT_LOG_N && sizeof shud_pt_logtab == 8 * kPowTabLogDoubles, "pow_tab");
    memcpy(&ctab[pt_off], shud_pt_logtab, sizeof shud_pt_logtab);
#endif
    static_assert(kPowTabDoubles == kPowTabLogDoubles + 2 * SHUD_PT_EXP_N, "pow_tab table size");
    memcpy(&ctab[pt_off + kPowTabLogDoubles], shud_pt_exptab, sizeof shud_pt_exptab);
    std::vector<double2> zz(NE), ged(3 * (size_t)NE);
    std::vector<int4> meta(NE);
    std::vector<int> sfirst(NE);
    for (int i = 0; i < NE; i++) {
        zz[i] = make_double2(m->z_surf[i], m->z_bottom[i]);
        const int nseg = seg_off[i + 1] - seg_off[i];
        const int ibc = (int8_t)(eflags[i] & 0xff);
        const bool lake_ele = m->ilake && m->ilake[i] > 0 && h->lakeon;
        const unsigned cf = (unsigned)(ibc & 0xff) | ((unsigned)((eflags[i] >> 16) & 3) << 8) |
                            ((unsigned)nseg << 10) | ((unsigned)cls[i] << 16) | (lake_ele ? 0x80000000u : 0u);
        meta[i] = make_int4(m->nabr[i], m->nabr[(size_t)NE + i], m->nabr[2 * (size_t)NE + i], (int)cf);
        for (int j = 0; j < 3; j++)
            ged[(size_t)j * NE + i] = make_double2(m->edge[(size_t)j * NE + i], m->dist2nabor[(size_t)j * NE + i]);
        sfirst[i] = seg_off[i];
    }
    // In-tile edge sharing (shud_ele_packed.hip, SH): an interior edge between two elements of one 256-element tile
    // whose fluxes are exactly antisymmetric (same edge length and Dist2Nabor bits from both sides, same depression,
    // positive finite avgRough, neither a lake element) is evaluated by one of them and read by the other from LDS.
    // Greedy in element order: every element publishes at most one edge and receives at most one, never both
    // directions of one edge.  seg_first bits 26-27: the published slot + 1, bits 28-29: the received slot + 1.
    // Elements [0, lim): a single-GPU handle's all, a partitioned handle's interior prefix (its ghost-free launch
    // tiles from element 0; the boundary launch ignores the bits), no hybrid layout; the instantiations without
    // sharing (diagnostics, lakes, hybrid, the 1024-thread table) ignore them.
    const int lim = h->n_int > 0 ? h->n_int : (h->n_own == NE ? NE : 0);
    // Only for handles that take the LSP instantiations (class + pow tables small enough, no lakes, no hybrid
    // layout): the other instantiations read seg_first with a 31-bit mask (shud_ele_packed.hip ele_body).
    if (lim > 1 && !hmask && !h->lakeon && lsp_lds_bytes((int)ctab.size()) <= kLspLdsMax && m->num_seg < (1 << 26) &&
        env_knob("SHUD_RHS_SHARE", 1, 0, 1)) {
        std::vector<signed char> pub(NE, -1), rcv(NE, -1);
        auto lake_of = [&](int e) { return m->ilake && m->ilake[e] > 0 && h->lakeon; };
        for (int i = 0; i < lim; i++) {
            for (int k = 0; k < 3 && rcv[i] < 0; k++) {
                const int v = m->nabr[(size_t)k * NE + i];
                if (v < 0 || v >= lim || v == i || (v / kShareTile) != (i / kShareTile) || pub[v] >= 0) continue;
                int kk = -1, hits = 0;
                for (int q = 0; q < 3; q++)
                    if (m->nabr[(size_t)q * NE + v] == i) { kk = q; hits++; }
                if (hits != 1 || pub[i] == k) continue;
                const size_t a = (size_t)k * NE + i, b = (size_t)kk * NE + v;
                const double ar = m->avg_rough[a];
                if (memcmp(&m->edge[a], &m->edge[b], 8) || memcmp(&m->dist2nabor[a], &m->dist2nabor[b], 8) ||
                    memcmp(&m->depression[i], &m->depression[v], 8) || memcmp(&ar, &m->avg_rough[b], 8) ||
                    !(ar > 0. && std::isfinite(ar)) || lake_of(i) || lake_of(v))
                    continue;
                pub[v] = (signed char)kk;
                rcv[i] = (signed char)k;
            }
        }
        for (int i = 0; i < NE; i++) sfirst[i] |= ((pub[i] + 1) << 26) | ((rcv[i] + 1) << 28);
        h->n_shared = (int)std::count_if(rcv.begin(), rcv.end(), [](signed char r) { return r >= 0; });
    }
    int rc;
    DevPacked &P = h->dp;
    double *ctab_d, *area_d; double2 *zz_d, *ged_d; int4 *meta_d; int *sf_d;
    if ((rc = h->upload(&ctab_d, ctab.data(), ctab.size()))) return rc;
    if ((rc = h->upload(&zz_d, zz.data(), NE))) return rc;
    if ((rc = h->upload(&meta_d, meta.data(), NE))) return rc;
    if ((rc = h->upload(&ged_d, ged.data(), ged.size()))) return rc;
    if ((rc = h->upload(&area_d, m->area, NE))) return rc;
    if ((rc = h->upload(&sf_d, sfirst.data(), NE))) return rc;
    P.ctab = ctab_d; P.ncls = ncls; P.pt_off = pt_off; P.ntab = (int)ctab.size(); P.zz = zz_d;
    if (hmask) {                                                     // the streamed fields, per element
        int nh = 0;
        for (int f = 0; f < CF_NPRIMARY; f++)
            if (hmask >> f & 1) P.hslot1[f] = (signed char)++nh;
        const int hs = nh == 1 ? 1 : nh == 2 ? 2 : 4;
        std::vector<double> hv((size_t)hs * NE, 0.0), rr(CF_NPRIMARY);
        for (int i = 0; i < NE; i++) {
            prim(i, rr);
            for (int f = 0; f < CF_NPRIMARY; f++)
                if (P.hslot1[f]) hv[(size_t)hs * i + P.hslot1[f] - 1] = rr[f];
        }
        double *hv_d;
        if ((rc = h->upload(&hv_d, hv.data(), hv.size()))) return rc;
        P.hv = hv_d; P.nh = nh; P.hs = hs;
        P.hnb = (hmask & (1u << CF_macD | 1u << CF_macKsatH | 1u << CF_vAreaF | 1u << CF_KsatH | 1u << CF_rough)) != 0;
    } P.meta = meta_d; P.ged = ged_d; P.area = area_d;
    P.seg_first = sf_d;
    {   // element-sorted segments {length, Cwr} + their reach; one 32-B record per reach with the statics the segment
        // fluxes read (seg_perm: element-sorted -> reference)
        const int NSg = m->num_seg, NRl = m->num_riv;
        std::vector<double2> lc(NSg), rr(2 * (size_t)NRl);
        std::vector<int> sr(NSg);
        for (int k = 0; k < NSg; k++) {
            const int s = h->seg_perm[k];
            lc[k] = make_double2(m->seg_length[s], m->seg_cwr[s]);
            sr[k] = m->seg_riv[s];
        }
        for (int r = 0; r < NRl; r++) {
            const int32_t two[2] = {m->riv_bc ? m->riv_bc[r] : 0, 0};
            double bits;
            memcpy(&bits, two, sizeof bits);
            rr[2 * (size_t)r] = make_double2(m->riv_depth[r], m->riv_ksath[r]);
            rr[2 * (size_t)r + 1] = make_double2(m->riv_bedthick[r], bits);
        }
        double2 *lc_d, *rr_d; int *sr_d;
        if ((rc = h->upload(&lc_d, lc.data(), NSg))) return rc;
        if ((rc = h->upload(&sr_d, sr.data(), NSg))) return rc;
        if ((rc = h->upload(&rr_d, rr.data(), rr.size()))) return rc;
        P.sg_lc = lc_d; P.sg_r = sr_d; P.rrec = rr_d;
        if ((rc = h->upload(&P.qseg2, (const double2 *)nullptr, NSg))) return rc;
    }
    if ((rc = h->upload(&P.s_np, (const double2 *)nullptr, NE))) return rc;
    if ((rc = h->upload(&P.s_tl, (const double2 *)nullptr, NE))) return rc;
    if ((rc = h->upload(&P.cs[0], (const double2 *)nullptr, NE))) return rc;
    if ((rc = h->upload(&P.cs[1], (const double2 *)nullptr, NE))) return rc;
    std::vector<double2> ones(NE, make_double2(1.0, 1.0));
    if ((rc = h->upload(&P.s_fu, ones.data(), NE))) return rc;

    // ---- segments in reach order (stable: reference order inside a reach) and reach records ----
    const int NS = m->num_seg, NR = m->num_riv;
    std::vector<int> rorder(NS);
    std::iota(rorder.begin(), rorder.end(), 0);
    std::stable_sort(rorder.begin(), rorder.end(), [&](int a, int b) { return m->seg_riv[a] < m->seg_riv[b]; });
    std::vector<int> rstart(NR, 0), rcnt(NR, 0);
    for (int q = NS - 1; q >= 0; q--) rstart[m->seg_riv[rorder[q]]] = q;
    for (int s = 0; s < NS; s++) rcnt[m->seg_riv[s]]++;
    std::vector<double2> rv(4 * (size_t)NR);
    std::vector<int4> ru(NR);
    const int nor = h->n_own_riv;
    for (int r = 0; r < NR; r++) {
        const int dn = (h->lakeon && m->riv_down[r] <= -4) ? -3 : m->riv_down[r];   // into a lake: outlet formula
        const int bc = m->riv_bc ? m->riv_bc[r] : 0;
        double ib;                                                   // (down, BC) packed into the 4th slot
        const int32_t two[2] = {dn, bc};
        memcpy(&ib, two, sizeof ib);
        rv[4 * (size_t)r + 0] = make_double2(m->riv_bottom_width[r], m->riv_bankslope[r]);
        rv[4 * (size_t)r + 1] = make_double2(m->riv_length[r], m->riv_bed_slope[r]);
        rv[4 * (size_t)r + 2] = make_double2(m->riv_dist2down[r], m->riv_avg_rough[r]);
        rv[4 * (size_t)r + 3] = make_double2(m->riv_depth[r], ib);
        int4 u = make_int4(rstart[r], rcnt[r], 0, 0);                // rv_u (shud_dev.h); ghosts: segments only
        if (r < nor) {
            const int n = up_off[r + 1] - up_off[r];
            u = n <= 2 ? make_int4(rstart[r], rcnt[r] | (n << 16), n > 0 ? up_idx[up_off[r]] : 0,
                                   n > 1 ? up_idx[up_off[r] + 1] : 0)
                       : make_int4(rstart[r], rcnt[r] | (3 << 16), up_off[r], n);
        }
        ru[r] = u;
    }
    double2 *rv_d; int4 *ru_d;
    if ((rc = h->upload(&rv_d, rv.data(), rv.size()))) return rc;
    if ((rc = h->upload(&ru_d, ru.data(), NR))) return rc;
    P.rv = rv_d; P.rv_u = ru_d;
    P.riv_sb = choose_riv_sb(rcnt.data(), nor);
    if (const int sb = env_knob("SHUD_RIV_SB", 0, 6, 8); sb == 6 || sb == 8) P.riv_sb = sb;   // tests: both batch sizes
    // QrivDown pre-pass slots (shud_dev.h DevPacked::qdown); SHUD_RHS_QD=0: the river kernel recomputes (tests, A/B)
    if (NR > 0 && env_knob("SHUD_RHS_QD", 1, 0, 1)) {
        if ((rc = h->upload(&P.qdown, (const double *)nullptr, NR))) return rc;
        P.nqd = NR;
    }
    P.qd_pm = env_knob("SHUD_QD_POS", 1000, 0, 1000);
    P.qd_pm_fold = env_knob("SHUD_QD_POS_FOLD", 1000, 0, 1000);
    h->n_classes = ncls;
    h->packed = true;
    return 0;
}

// Lakes: lake / bank-edge / inflow lists in the reference's summation orders, bathymetry.
static int build_lakes(shud_rhs *h, const ShudMeshSoA *m, const ShudPartition *part) {
    const int NE = m->num_ele, NR = m->num_riv, NL = h->NL;
    const int NO = h->n_own;                   // lake and bank elements are owned (partition plan)
    if (!h->packed)
        return shud_fail(SHUD_ERR_UNSUPPORTED, "lakes need the packed layout (mesh did not qualify or SHUD_RHS_PACKED=0)");
    if (h->n_classes > 128) return shud_fail(SHUD_ERR_UNSUPPORTED, "lakes: more than 128 parameter classes");
    std::vector<int> lake_of(NE, -1), ele_off(NL + 1, 0), bank_off(NL + 1, 0), rin_off(NL + 1, 0);
    std::vector<int> ele_idx, bank_pos, rin_idx;
    for (int i = 0; i < NE; i++) {
        if (m->ilake[i] <= 0) continue;
        if (i >= NO) return shud_fail(SHUD_ERR_ARG, "lake element %d is a ghost (partition splits a lake group)", i);
        lake_of[i] = m->ilake[i] - 1;
        ele_off[m->ilake[i]]++;
    }
    // bank edges: a non-lake element's edge whose neighbour is a lake element (lakenabr, MD_Lake.cpp:131-143)
    auto bank_lake = [&](int i, int j) -> int {
        if (i >= NO || m->ilake[i] > 0) return -1;
        const int nb = m->nabr[(size_t)j * NE + i];
        return (nb >= 0 && m->ilake[nb] > 0) ? m->ilake[nb] - 1 : -1;
    };
    for (int i = 0; i < NE; i++)
        for (int j = 0; j < 3; j++) { const int l = bank_lake(i, j); if (l >= 0) bank_off[l + 1]++; }
    for (int r = 0; r < NR; r++)
        if (m->riv_down[r] <= -4) rin_off[(-3 - m->riv_down[r])]++;
    for (int l = 0; l < NL; l++) {
        ele_off[l + 1] += ele_off[l]; bank_off[l + 1] += bank_off[l]; rin_off[l + 1] += rin_off[l];
    }
    ele_idx.resize(ele_off[NL]); bank_pos.resize(bank_off[NL]); rin_idx.resize(rin_off[NL]);
    {
        std::vector<int> fe(ele_off.begin(), ele_off.end() - 1), fb(bank_off.begin(), bank_off.end() - 1),
            fr(rin_off.begin(), rin_off.end() - 1);
        for (int i = 0; i < NE; i++) {                  // ascending element, then edge: the reference's order
            if (m->ilake[i] > 0) ele_idx[fe[m->ilake[i] - 1]++] = i;
            for (int j = 0; j < 3; j++) { const int l = bank_lake(i, j); if (l >= 0) bank_pos[fb[l]++] = j * NE + i; }
        }
        for (int r = 0; r < NR; r++)
            if (m->riv_down[r] <= -4) { const int l = (-3 - m->riv_down[r]) - 1; rin_idx[fr[l]++] = r; }
    }
    // partitioned: local order is [interior | boundary | ghosts] / [owned | ghosts], so put every lake list in
    // global order (the single-GPU summation order, hence bit-identical sums)
    if (part && part->ele_gid && part->riv_gid) {
        const int32_t *eg = part->ele_gid, *rg = part->riv_gid;
        for (int l = 0; l < NL; l++) {
            std::sort(ele_idx.begin() + ele_off[l], ele_idx.begin() + ele_off[l + 1],
                      [&](int a, int b) { return eg[a] < eg[b]; });
            std::sort(bank_pos.begin() + bank_off[l], bank_pos.begin() + bank_off[l + 1], [&](int a, int b) {
                const int ia = a % NE, ib = b % NE;                 // pos = j*NE + i: element, then edge
                return eg[ia] != eg[ib] ? eg[ia] < eg[ib] : a / NE < b / NE;
            });
            std::sort(rin_idx.begin() + rin_off[l], rin_idx.begin() + rin_off[l + 1],
                      [&](int a, int b) { return rg[a] < rg[b]; });
        }
    }
    for (int l = 0; l < NL; l++)
        if (ele_off[l + 1] == ele_off[l]) return shud_fail(SHUD_ERR_ARG, "lake %d has no lake element", l + 1);
    DevLake &L = h->lk;
    L.nl = NL;
    L.y_off = 3 * h->n_own + h->n_own_riv;    // [sf|us|gw|riv|lake] over owned entities
    int rc;
    int *lo, *eo, *ei, *bo, *bp, *ro, *ri, *bto;
    double *by, *ba;
    const int nb = m->lake_bathy_off[NL];
    if ((rc = h->upload(&lo, lake_of.data(), NE)) || (rc = h->upload(&eo, ele_off.data(), NL + 1)) ||
        (rc = h->upload(&ei, ele_idx.data(), ele_idx.size())) || (rc = h->upload(&bo, bank_off.data(), NL + 1)) ||
        (rc = h->upload(&bp, bank_pos.data(), bank_pos.size())) || (rc = h->upload(&ro, rin_off.data(), NL + 1)) ||
        (rc = h->upload(&ri, rin_idx.data(), rin_idx.size())) || (rc = h->upload(&bto, m->lake_bathy_off, NL + 1)) ||
        (rc = h->upload(&by, m->lake_bathy_y, nb)) || (rc = h->upload(&ba, m->lake_bathy_a, nb)) ||
        (rc = h->upload(&L.bank_qs, (const double *)nullptr, 3 * (size_t)NE)) ||
        (rc = h->upload(&L.bank_qg, (const double *)nullptr, 3 * (size_t)NE)))
        return rc;
    L.lake_of = lo; L.ele_off = eo; L.ele_idx = ei; L.bank_off = bo; L.bank_pos = bp; L.rin_off = ro; L.rin_idx = ri;
    L.bathy_off = bto; L.bathy_y = by; L.bathy_a = ba;
    return 0;
}

static int setup_partition(shud_rhs *h, const ShudPartition *part) {
    h->partitioned = true;
    h->rank = part->rank;
    h->nranks = part->nranks;
    const int P = part->nranks;
    if (P < 1 || part->rank < 0 || part->rank >= P) return shud_fail(SHUD_ERR_ARG, "bad rank/nranks");
    h->esend_off.assign(part->ele_send_off, part->ele_send_off + P + 1);
    h->erecv_off.assign(part->ele_recv_off, part->ele_recv_off + P + 1);
    h->rsend_off.assign(part->riv_send_off, part->riv_send_off + P + 1);
    h->rrecv_off.assign(part->riv_recv_off, part->riv_recv_off + P + 1);
    h->n_esend = h->esend_off[P];
    h->n_rsend = h->rsend_off[P];
    h->n_eghost = h->erecv_off[P];
    h->n_rghost = h->rrecv_off[P];
    if (h->n_own + h->n_eghost != h->NE) return shud_fail(SHUD_ERR_ARG, "ghost element count mismatch");
    if (h->n_own_riv + h->n_rghost != h->NR) return shud_fail(SHUD_ERR_ARG, "ghost reach count mismatch");
    for (int k = 0; k < h->n_esend; k++)
        if (part->ele_send_idx[k] < 0 || part->ele_send_idx[k] >= h->n_own) return shud_fail(SHUD_ERR_ARG, "bad ele_send_idx");
    for (int k = 0; k < h->n_rsend; k++)
        if (part->riv_send_idx[k] < 0 || part->riv_send_idx[k] >= h->n_own_riv) return shud_fail(SHUD_ERR_ARG, "bad riv_send_idx");
    int rc;
    if ((rc = h->upload(&h->d_esend_idx, part->ele_send_idx, h->n_esend))) return rc;
    if ((rc = h->upload(&h->d_rsend_idx, part->riv_send_idx, h->n_rsend))) return rc;
    if ((rc = h->dalloc(&h->d_esend, 3 * (size_t)h->n_esend))) return rc;
    if ((rc = h->dalloc(&h->d_rsend, (size_t)h->n_rsend))) return rc;
    if ((rc = h->dalloc(&h->d_gele, 3 * (size_t)h->n_eghost))) return rc;
    if ((rc = h->dalloc(&h->d_griv, (size_t)h->n_rghost))) return rc;
    if (part->nccl_unique_id) {
        ncclUniqueId id;
        memcpy(&id, part->nccl_unique_id, sizeof(id));
        h->use_nccl = true;
        NCCL_TRY(ncclCommInitRank(&h->comm, P, id, part->rank));
    }
    // the pack kernel and the exchange run on a side stream beside the interior element kernel (RCCL and
    // external transport alike, so the one-GPU rank timings measure the same pipeline)
    HIP_TRY(hipStreamCreateWithFlags(&h->s_comm, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&h->ev_pack, hipEventDisableTiming | kEvSync));
    HIP_TRY(hipEventCreateWithFlags(&h->ev_comm, hipEventDisableTiming | kEvSync));
    if ((rc = h->upload(&h->d_halo_flag, (const unsigned long long *)nullptr, 1))) return rc;
    h->fold = env_knob("SHUD_RHS_FOLD", 1, 0, 1) != 0;
    // the trailing join of the comm stream after a folded eval costs ~4 us per eval at 8 ranks (one more packet for
    // the command processor between evals; profiles/r04/rankjoin): off by default.  Without it, after a poll timeout
    // (SHUD_EF_HALO_WAIT, fatal) the late pack / exchange may still run beside later main-stream work — results that
    // the fatal flag already invalidates; the error read (shud_read_err) drains the comm stream before reporting
    h->fold_join = env_knob("SHUD_RHS_FOLD_JOIN", 0, 0, 1) != 0;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device) == hipSuccess && khz > 0)
        h->wall_khz = khz;
    const double ms = env_knob("SHUD_HALO_TIMEOUT_MS", 5000, 1, 3600000);
    h->halo_timeout = (unsigned long long)(ms * h->wall_khz);
    return 0;
}

static void destroy_handle(shud_rhs *h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->s_comm) (void)hipStreamSynchronize(h->s_comm);
    if (h->comm) ncclCommDestroy(h->comm);
    shud_et_free(h);
    if (h->ev_pack) (void)hipEventDestroy(h->ev_pack);
    if (h->ev_comm) (void)hipEventDestroy(h->ev_comm);
    for (auto e : h->tm_ev) (void)hipEventDestroy(e);
    if (h->s_comm) (void)hipStreamDestroy(h->s_comm);
    for (void *p : h->allocs) (void)hipFree(p);
    if (h->h_err) (void)hipHostFree(h->h_err);
    if (h->h_warn) (void)hipHostFree(h->h_warn);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

extern "C" int shud_rhs_create(const ShudMeshSoA *mesh, const ShudParamsSoA *par, const ShudRhsOptions *opt,
                               shud_rhs_t *out) {
    if (!mesh || !par || !out) return shud_fail(SHUD_ERR_ARG, "null argument");
    shud_rhs *h = new shud_rhs();
    int rc = build(h, mesh, par, opt, nullptr);
    if (rc) { destroy_handle(h); return rc; }
    *out = h;
    return SHUD_OK;
}

extern "C" int shud_rhs_nccl_unique_id(char out[128]) {
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    memcpy(out, &id, sizeof(id));
    return SHUD_OK;
}

extern "C" int shud_rhs_create_partitioned(const ShudMeshSoA *mesh, const ShudParamsSoA *par,
                                           const ShudRhsOptions *opt, const ShudPartition *part,
                                           shud_rhs_t *out) {
    if (!mesh || !par || !part || !out) return shud_fail(SHUD_ERR_ARG, "null argument");
    shud_rhs *h = new shud_rhs();
    int rc = build(h, mesh, par, opt, part);
    if (!rc) rc = setup_partition(h, part);
    if (rc) { destroy_handle(h); return rc; }
    *out = h;
    return SHUD_OK;
}

extern "C" int shud_rhs_destroy(shud_rhs_t h) {
    destroy_handle(h);
    return SHUD_OK;
}

// ---------------------------------------------------------------------------------------------
// step inputs
// ---------------------------------------------------------------------------------------------
extern "C" int shud_rhs_set_step_inputs(shud_rhs_t h, const ShudStepInputs *in) {
    if (!h || !in) return shud_fail(SHUD_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(h->device));
    const size_t nb = (size_t)h->NE * sizeof(double);
    // packed layout: carried-state overrides go through SoA staging slot 0, then into the packed record
    const double *eic_dst = h->packed ? h->dm.e_ic[0] : h->dm.e_ic[h->cur_e];
    const double *satn_dst = h->packed ? h->dm.u_satn[0] : h->dm.u_satn[h->cur];
    struct { const double *src; const double *dst; } arr[] = {
        {in->net_prep, h->dm.net_prep}, {in->pot_evap, h->dm.pot_evap}, {in->pot_tran, h->dm.pot_tran},
        {in->etp, h->dm.etp}, {in->lai, h->dm.lai}, {in->fu_surf, h->dm.fu_surf}, {in->fu_sub, h->dm.fu_sub},
        {in->ugw_stale, h->dm.ugw_stale}, {in->e_ic, eic_dst}, {in->u_satn, satn_dst}, {in->prcp, h->dm.prcp}};
    for (auto &a : arr)
        if (a.src) HIP_TRY(hipMemcpyAsync((void *)a.dst, a.src, nb, hipMemcpyHostToDevice, h->stream));
    if (h->packed) {
        auto all_ones = [&](const double *v) {
            for (int i = 0; i < h->NE; i++)
                if (!(v[i] == 1.0)) return false;
            return true;
        };
        if (in->fu_surf) h->fu_unit[0] = all_ones(in->fu_surf);
        if (in->fu_sub) h->fu_unit[1] = all_ones(in->fu_sub);
        unsigned what = 0;
        if (in->net_prep || in->pot_evap) what |= 1;
        if (in->pot_tran || in->lai || in->etp) what |= 2;
        if (in->fu_surf || in->fu_sub) what |= 4;
        if (in->u_satn) what |= 8;
        if (in->e_ic) what |= 16;
        launch_pack_step_kernel(h->dm, h->dp, h->NE, h->cur, what, h->stream);
        HIP_TRY(hipGetLastError());
    }
    const double *tabs[4] = {in->ele_ybc, in->ele_qbc, in->riv_ybc, in->riv_qbc};
    const int ns[4] = {in->n_ele_ybc, in->n_ele_qbc, in->n_riv_ybc, in->n_riv_qbc};
    for (int k = 0; k < 4; k++) {
        if (!tabs[k]) continue;
        if (ns[k] < h->max_col[k])
            return shud_fail(SHUD_ERR_ARG, "BC table %d has %d columns, mesh references column %d", k, ns[k], h->max_col[k]);
        HIP_TRY(hipMemcpyAsync(h->d_tab[k], tabs[k], (size_t)h->tab_len[k] * sizeof(double), hipMemcpyHostToDevice,
                               h->stream));
    }
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->have_last = false;
    return SHUD_OK;
}

// ---------------------------------------------------------------------------------------------
// eval
// ---------------------------------------------------------------------------------------------
// on the comm stream, once y is ready on the main stream (ev_pack): pack the owned states peers need, then the
// grouped RCCL send/recv; ev_comm marks the ghost buffers filled.  The main stream meanwhile runs the interior
// elements, so the pack (~4 us at 8 ranks) and the exchange leave the critical path.  s_comm is in order and
// waits for everything enqueued on the main stream before this eval, so neither the send buffers nor the
// ghost buffers are rewritten while the previous eval still reads them.
static int exchange(shud_rhs *h, const double *y) {
    if (!h->partitioned) return 0;
    HIP_TRY(hipEventRecord(h->ev_pack, h->stream));
    HIP_TRY(hipStreamWaitEvent(h->s_comm, h->ev_pack, 0));
    launch_pack_kernel(y, h->n_own, h->n_own_riv, h->d_esend_idx, h->n_esend, h->d_rsend_idx, h->n_rsend,
                       h->d_esend, h->d_rsend, h->s_comm);
    if (h->use_nccl) {
    NCCL_TRY(ncclGroupStart());
    for (int p = 0; p < h->nranks; p++) {
        if (p == h->rank) continue;
        size_t se = h->esend_off[p + 1] - h->esend_off[p], re = h->erecv_off[p + 1] - h->erecv_off[p];
        size_t sr = h->rsend_off[p + 1] - h->rsend_off[p], rr = h->rrecv_off[p + 1] - h->rrecv_off[p];
        if (se) NCCL_TRY(ncclSend(h->d_esend + 3 * (size_t)h->esend_off[p], 3 * se, ncclDouble, p, h->comm, h->s_comm));
        if (re) NCCL_TRY(ncclRecv(h->d_gele + 3 * (size_t)h->erecv_off[p], 3 * re, ncclDouble, p, h->comm, h->s_comm));
        if (sr) NCCL_TRY(ncclSend(h->d_rsend + h->rsend_off[p], sr, ncclDouble, p, h->comm, h->s_comm));
        if (rr) NCCL_TRY(ncclRecv(h->d_griv + h->rrecv_off[p], rr, ncclDouble, p, h->comm, h->s_comm));
    }
    NCCL_TRY(ncclGroupEnd());
    }                                // external transport (tests): the caller placed the ghost buffers
    if (h->dbg_armed) {              // test hook: the halo arrives late (spin), written by a kernel, or never
        if (h->dbg_spin) launch_spin(h->dbg_spin, h->s_comm);
        if (h->dbg_gele) launch_copy_f64(h->d_gele, h->dbg_gele, 3 * (size_t)h->n_eghost, h->s_comm);
        if (h->dbg_griv) launch_copy_f64(h->d_griv, h->dbg_griv, (size_t)h->n_rghost, h->s_comm);
    }
    ++h->halo_epoch;
    if (h->fold && !(h->dbg_armed && !h->dbg_publish)) launch_halo_flag(h->d_halo_flag, h->halo_epoch, h->s_comm);
    HIP_TRY(hipEventRecord(h->ev_comm, h->s_comm));
    h->n_exch++;
    return 0;
}

static void launch_ele(shud_rhs *h, const double *y, double *dy, int cur, int cur_e, bool diag, int i0 = 0,
                       int i1 = -1) {
    YView Y{y, h->d_gele, h->d_griv, h->n_own, h->n_own_riv};
    if (i1 < 0) i1 = h->n_own + h->n_segghost;
    // the last element launch of an eval (after the halo in every partitioned path) carries the QrivDown pre-pass
    const bool last = i1 == h->n_own + h->n_segghost;
    if (h->packed) {
        const bool qd = launch_element_kernel_packed(h->dm, h->dp, Y, dy, i0, i1, cur, h->mode, h->open, diag,
                                                     h->fu_unit[0] && h->fu_unit[1], h->dd, h->stream,
                                                     h->lakeon ? &h->lk : nullptr, h->partitioned && i1 <= h->n_int,
                                                     last);
        if (last) h->qd_now = qd;
    } else {
        launch_element_kernel(h->dm, Y, dy, h->n_own + h->n_segghost, cur, cur_e, h->mode, h->open, diag, h->dd,
                              h->stream);
        h->qd_now = false;
    }
}
static void launch_riv(shud_rhs *h, const double *y, double *dy, bool diag) {
    YView Y{y, h->d_gele, h->d_griv, h->n_own, h->n_own_riv};
    if (h->packed)
        launch_river_kernel_packed(h->dm, h->dp, Y, dy, h->mode, diag, h->dd, h->stream, h->qd_now);
    else
        launch_river_kernel(h->dm, Y, dy, h->mode, diag, h->dd, h->stream);
    if (h->lakeon) launch_lake_kernel(h->dm, h->dp, h->lk, Y, dy, diag, h->dd, h->stream);
}
static void launch_all(shud_rhs *h, const double *y, double *dy, int cur, int cur_e, bool diag) {
    launch_ele(h, y, dy, cur, cur_e, diag);
    launch_riv(h, y, dy, diag);
}
// carried-state ping-pong after an eval: the packed record carries {u_satn, e_ic} together
static void flip(shud_rhs *h) {
    h->cur ^= 1;
    if (h->packed) h->cur_e = h->cur;
    else if (h->mode == SHUD_MODE_SERIAL) h->cur_e ^= 1;
}

int shud_read_err(shud_rhs *h) {
    HIP_TRY(hipMemcpyAsync(h->h_err, h->d_err, sizeof(DevErr), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->h_err->n_warn = 0;
    if (h->h_err->flags & SHUD_EF_AET_WARN) {          // the only counted report
        HIP_TRY(hipMemcpyAsync(h->h_warn, h->d_warn, kWarnSlots * kWarnStride * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        for (int k = 0; k < kWarnSlots; k++) h->h_err->n_warn += h->h_warn[k * kWarnStride];
    }
    // a halo poll timed out: the pack / exchange it gave up on may still be running — drain the comm stream before
    // the failure reaches the caller, so nothing of that eval is still in flight when the caller reacts
    if ((h->h_err->flags & SHUD_EF_HALO_WAIT) && h->s_comm) HIP_TRY(hipStreamSynchronize(h->s_comm));
    return 0;
}
static int read_err(shud_rhs *h) { return shud_read_err(h); }

static const uint32_t kFatal = SHUD_EF_NAN_QELE | SHUD_EF_EFFKH | SHUD_EF_ET_NEG | SHUD_EF_ET_NAN | SHUD_EF_HALO_WAIT;

// partitioned handles: the interior elements [0, n_int) run while the halo exchange is in flight (RCCL on
// s_comm); boundary + ghost elements and the reaches wait for it.  Unpartitioned: one launch each.
// stream_halo: the halo is already ordered on the main stream (eval_compute, external transport) — the folded
// launch's boundary workgroups then skip the flag
static int launch_split(shud_rhs *h, const double *y, double *dy, hipEvent_t e_mid = nullptr,
                        bool stream_halo = false) {
    // an RCCL communicator connects its peers lazily on the first send/recv (can take far longer than any eval):
    // that first exchange is waited for on the stream (split path), never polled by workgroups
    const bool first_rccl = h->use_nccl && h->n_exch <= 1 && !stream_halo;
    if (h->fold && h->packed && !h->lakeon && !first_rccl) {
        YView Y{y, h->d_gele, h->d_griv, h->n_own, h->n_own_riv};
        const HaloWait hw{h->d_halo_flag, stream_halo ? 0ull : h->halo_epoch, h->halo_timeout};
        if (launch_element_kernel_packed_fold(h->dm, h->dp, Y, dy, h->n_int, h->n_own + h->n_segghost, h->cur,
                                              h->mode, h->open, h->fu_unit[0] && h->fu_unit[1], h->dd, hw,
                                              h->stream, true)) {
            h->qd_now = h->dp.qdown != nullptr && h->dp.nqd > 0;
            if (e_mid) HIP_TRY(hipEventRecord(e_mid, h->stream));
            launch_riv(h, y, dy, false);             // after the boundary workgroups, which saw the halo
            // optional join of the comm stream (normally complete long before: the boundary workgroups saw its flag),
            // so that after a poll timeout no later main-stream work runs beside the late pack / exchange
            if (h->fold_join && !stream_halo) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_comm, 0));
            HIP_TRY(hipGetLastError());
            return 0;
        }
    }
    if (h->partitioned && h->packed && h->n_int > 0) {
        launch_ele(h, y, dy, h->cur, h->cur_e, false, 0, h->n_int);
        HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_comm, 0));
        launch_ele(h, y, dy, h->cur, h->cur_e, false, h->n_int, h->n_own + h->n_segghost);
        if (e_mid) HIP_TRY(hipEventRecord(e_mid, h->stream));
        launch_riv(h, y, dy, false);
    } else {
        if (h->partitioned) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_comm, 0));
        launch_ele(h, y, dy, h->cur, h->cur_e, false);
        if (e_mid) HIP_TRY(hipEventRecord(e_mid, h->stream));
        launch_riv(h, y, dy, false);
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

static int eval_device(shud_rhs *h, double t, const double *y, double *dy) {
    (void)t;
    hipEvent_t *E = nullptr;
    if (h->tm_n < h->tm_cap && (h->tm_seen++ % h->tm_stride) == 0) E = &h->tm_ev[3 * (size_t)h->tm_n++];
    if (E) HIP_TRY(hipEventRecord(E[0], h->stream));
    int rc = exchange(h, y);
    if (rc) return rc;
    h->last_cur = h->cur;
    h->last_cur_e = h->cur_e;
    if ((rc = launch_split(h, y, dy, E ? E[1] : nullptr))) return rc;
    if (E) HIP_TRY(hipEventRecord(E[2], h->stream));
    flip(h);
    h->last_y = y;
    h->have_last = true;
    h->ncalls++;
    return 0;
}

extern "C" int shud_rhs_eval(shud_rhs_t h, double t, const double *y, double *ydot, int where) {
    if (!h || !y || !ydot) return shud_fail(SHUD_ERR_ARG, "null argument");
    const size_t ny = 3 * (size_t)h->n_own + h->n_own_riv + h->NL;
    if (where == SHUD_WHERE_DEVICE) return eval_device(h, t, y, ydot);
    if (where != SHUD_WHERE_HOST) return shud_fail(SHUD_ERR_ARG, "bad where");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipMemcpyAsync(h->d_y, y, ny * sizeof(double), hipMemcpyHostToDevice, h->stream));
    int rc = eval_device(h, t, h->d_y, h->d_ydot);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(ydot, h->d_ydot, ny * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    if (h->check_errors) {
        if ((rc = read_err(h))) return rc;
        if (h->h_err->flags & kFatal) return shud_fail(SHUD_ERR_PHYSICS, "physics error flags 0x%x", h->h_err->flags);
    } else {
        HIP_TRY(hipStreamSynchronize(h->stream));
    }
    return SHUD_OK;
}

extern "C" long long shud_rhs_num_calls(shud_rhs_t h) { return h ? h->ncalls : -1; }

extern "C" int shud_rhs_layout_streamed(shud_rhs_t h, int *n_streamed) {
    if (!h || !n_streamed) return shud_fail(SHUD_ERR_ARG, "null argument");
    *n_streamed = h->packed ? h->dp.nh : 0;
    return SHUD_OK;
}

extern "C" int shud_rhs_layout_shared(shud_rhs_t h, int *n_shared) {
    if (!h || !n_shared) return shud_fail(SHUD_ERR_ARG, "null argument");
    *n_shared = h->packed ? h->n_shared : 0;
    return SHUD_OK;
}

extern "C" int shud_rhs_layout(shud_rhs_t h, int *packed, int *n_classes) {
    if (!h) return shud_fail(SHUD_ERR_ARG, "null argument");
    if (packed) *packed = h->packed ? 1 : 0;
    if (n_classes) *n_classes = h->n_classes;
    return SHUD_OK;
}

// ---------------------------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------------------------
extern "C" int shud_rhs_get_error(shud_rhs_t h, ShudErr *e) {
    if (!h || !e) return shud_fail(SHUD_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(h->device));
    int rc = read_err(h);
    if (rc) return rc;
    const DevErr &d = *h->h_err;
    memset(e, 0, sizeof(*e));
    e->flags = d.flags;
    for (int k = 0; k < 8; k++) e->first_index[k] = (d.first_index[k] == INT_MAX) ? -1 : d.first_index[k];
    e->n_aet_warn = (int64_t)d.n_warn;
    // ET-step prelude (shud_et_step): tReadForcing's CheckNonZero(ra) then CheckNANi(qPotTran), per element
    if (d.flags & (SHUD_EF_ET_RA | SHUD_EF_ET_PT_NAN)) {
        const int ra = (d.flags & SHUD_EF_ET_RA) ? d.first_index[5] : INT_MAX;
        const int pt = (d.flags & SHUD_EF_ET_PT_NAN) ? d.first_index[6] : INT_MAX;
        e->exit_code = 10;
        if (ra <= pt)
            snprintf(e->message, sizeof(e->message),
                     "ERROR: Value for Aerodynamic Resistance of Element %d is not allowed. Please check again.", ra + 1);
        else
            snprintf(e->message, sizeof(e->message), "ERROR: NAN error for qPotTran[i] %d", pt + 1);
        return SHUD_OK;
    }
    // the reference stops at the first myexit() in loop order: loop A (f_etFlux then effKH, per element,
    // MD_f.cpp:11-26), then the applyDY NaN check (MD_f.cpp:73-74)
    int et = INT_MAX;
    if (d.flags & SHUD_EF_ET_NEG) et = std::min(et, d.first_index[2]);
    if (d.flags & SHUD_EF_ET_NAN) et = std::min(et, d.first_index[3]);
    int kh = (d.flags & SHUD_EF_EFFKH) ? d.first_index[1] : INT_MAX;
    if (et != INT_MAX || kh != INT_MAX) {
        if (et <= kh) {
            e->exit_code = 10;
            bool neg = (d.flags & SHUD_EF_ET_NEG) && d.first_index[2] == et;
            snprintf(e->message, sizeof(e->message), neg ? "ERROR: Negative ET flux of Element %d is not allowed."
                                                         : "ERROR: NAN error for ET flux %d", et + 1);
        } else {
            e->exit_code = 13;
            snprintf(e->message, sizeof(e->message), "Wrong effKH for ground water (element %d)", kh + 1);
        }
    } else if (d.flags & SHUD_EF_NAN_QELE) {
        e->exit_code = 10;
        snprintf(e->message, sizeof(e->message), "ERROR: NAN error for QeleSurf/QeleSub %d", d.first_index[0] + 1);
    }
    return SHUD_OK;
}

extern "C" int shud_rhs_clear_error(shud_rhs_t h) {
    if (!h) return shud_fail(SHUD_ERR_ARG, "null argument");
    return shud_reset_err(h);
}

extern "C" int shud_rhs_cvrhs(double t, const double *y, double *ydot, void *user_data) {
    shud_rhs *h = (shud_rhs *)user_data;
    int rc = shud_rhs_eval(h, t, y, ydot, SHUD_WHERE_HOST);
    if (rc == SHUD_OK) return 0;
    if (rc == SHUD_ERR_PHYSICS && env_knob("SHUD_RHS_STRICT_EXIT", 0, 0, 1)) {
        ShudErr e;
        shud_rhs_get_error(h, &e);
        printf("\n%s\n", e.message);
        fprintf(stderr, "\nEXIT with error code %d\n", e.exit_code);
        exit(e.exit_code);
    }
    return -1;
}

// ---------------------------------------------------------------------------------------------
// diagnostics (replay of the last call with DIAG kernels)
// ---------------------------------------------------------------------------------------------
int shud_ensure_diag(shud_rhs *h) {
    if (h->have_diag) return 0;
    const size_t NE = h->NE, NR = h->NR;
    double **e1[] = {&h->dd.qele_surf_tot, &h->dd.qele_sub_tot, &h->dd.q_infil, &h->dd.q_exfil, &h->dd.q_recharge,
                     &h->dd.q_es, &h->dd.q_eu, &h->dd.q_eg, &h->dd.q_tu, &h->dd.q_tg, &h->dd.q_eta,
                     &h->dd.e_ic, &h->dd.u_satn, &h->dd.i_beta, &h->dd.eff_kh, &h->dd.qe2r_surf, &h->dd.qe2r_sub};
    int rc;
    for (auto pp : e1)
        if ((rc = h->upload(pp, (const double *)nullptr, NE))) return rc;
    if ((rc = h->upload(&h->dd.qele_surf, (const double *)nullptr, 3 * NE))) return rc;
    if ((rc = h->upload(&h->dd.qele_sub, (const double *)nullptr, 3 * NE))) return rc;
    double **r1[] = {&h->dd.qriv_down, &h->dd.qriv_up, &h->dd.qriv_surf, &h->dd.qriv_sub};
    for (auto pp : r1)
        if ((rc = h->upload(pp, (const double *)nullptr, NR))) return rc;
    double **l1[] = {&h->dd.q_lake_surf, &h->dd.q_lake_sub, &h->dd.q_lake_rivin, &h->dd.q_lake_evap,
                     &h->dd.q_lake_prcp, &h->dd.lake_toparea};
    for (auto pp : l1)
        if ((rc = h->upload(pp, (const double *)nullptr, std::max(h->NL, 1)))) return rc;
    h->have_diag = true;
    return 0;
}

// replay of the last evaluation with diagnostic stores: same y, same carried-state inputs (it rewrites the
// same carried outputs), ydot into scratch; stream-ordered, the diagnostics stay in HBM (DevDiag)
int shud_diag_replay(shud_rhs *h) {
    if (!h->have_last) return shud_fail(SHUD_ERR_ARG, "no evaluation to report diagnostics for");
    HIP_TRY(hipSetDevice(h->device));
    int rc = shud_ensure_diag(h);
    if (rc) return rc;
    launch_all(h, h->last_y, h->d_scratch_dy, h->last_cur, h->last_cur_e, true);
    HIP_TRY(hipGetLastError());
    return 0;
}

extern "C" int shud_rhs_sync_diagnostics(shud_rhs_t h, ShudFluxOut *o) {
    if (!h || !o) return shud_fail(SHUD_ERR_ARG, "null argument");
    int rc = shud_diag_replay(h);
    if (rc) return rc;
    const size_t NE = h->NE, NR = h->NR, NS = h->NS;
    auto get = [&](double *dst, const double *src, size_t n) -> int {
        if (dst && n) HIP_TRY(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        return 0;
    };
    const DevDiag &g = h->dd;
    if ((rc = get(o->qele_surf, g.qele_surf, 3 * NE)) || (rc = get(o->qele_sub, g.qele_sub, 3 * NE)) ||
        (rc = get(o->qele_surf_tot, g.qele_surf_tot, NE)) || (rc = get(o->qele_sub_tot, g.qele_sub_tot, NE)) ||
        (rc = get(o->q_infil, g.q_infil, NE)) || (rc = get(o->q_exfil, g.q_exfil, NE)) ||
        (rc = get(o->q_recharge, g.q_recharge, NE)) || (rc = get(o->q_es, g.q_es, NE)) ||
        (rc = get(o->q_eu, g.q_eu, NE)) || (rc = get(o->q_eg, g.q_eg, NE)) || (rc = get(o->q_tu, g.q_tu, NE)) ||
        (rc = get(o->q_tg, g.q_tg, NE)) || (rc = get(o->q_eta, g.q_eta, NE)) || (rc = get(o->e_ic, g.e_ic, NE)) ||
        (rc = get(o->u_satn, g.u_satn, NE)) || (rc = get(o->i_beta, g.i_beta, NE)) ||
        (rc = get(o->eff_kh, g.eff_kh, NE)) || (rc = get(o->qe2r_surf, g.qe2r_surf, NE)) ||
        (rc = get(o->qe2r_sub, g.qe2r_sub, NE)) || (rc = get(o->qriv_down, g.qriv_down, NR)) ||
        (rc = get(o->qriv_up, g.qriv_up, NR)) || (rc = get(o->qriv_surf, g.qriv_surf, NR)) ||
        (rc = get(o->qriv_sub, g.qriv_sub, NR)) || (rc = get(o->q_lake_surf, g.q_lake_surf, h->NL)) ||
        (rc = get(o->q_lake_sub, g.q_lake_sub, h->NL)) || (rc = get(o->q_lake_rivin, g.q_lake_rivin, h->NL)) ||
        (rc = get(o->q_lake_evap, g.q_lake_evap, h->NL)) || (rc = get(o->q_lake_prcp, g.q_lake_prcp, h->NL)) ||
        (rc = get(o->lake_toparea, g.lake_toparea, h->NL)))
        return rc;
    std::vector<double> tmp;
    if (o->qseg_surf || o->qseg_sub) tmp.resize(std::max<size_t>(NS, 1));
    HIP_TRY(hipStreamSynchronize(h->stream));
    const std::vector<int> &perm = h->seg_perm;
    if (h->packed && NS && (o->qseg_surf || o->qseg_sub)) {
        std::vector<double2> q2(NS);
        HIP_TRY(hipMemcpy(q2.data(), h->dp.qseg2, NS * sizeof(double2), hipMemcpyDeviceToHost));
        for (size_t k = 0; k < NS; k++) {
            if (o->qseg_surf) o->qseg_surf[perm[k]] = q2[k].x;
            if (o->qseg_sub) o->qseg_sub[perm[k]] = q2[k].y;
        }
        return SHUD_OK;
    }
    if (o->qseg_surf) {
        HIP_TRY(hipMemcpy(tmp.data(), h->dm.qseg_surf, NS * sizeof(double), hipMemcpyDeviceToHost));
        for (size_t k = 0; k < NS; k++) o->qseg_surf[perm[k]] = tmp[k];
    }
    if (o->qseg_sub) {
        HIP_TRY(hipMemcpy(tmp.data(), h->dm.qseg_sub, NS * sizeof(double), hipMemcpyDeviceToHost));
        for (size_t k = 0; k < NS; k++) o->qseg_sub[perm[k]] = tmp[k];
    }
    return SHUD_OK;
}

// ---------------------------------------------------------------------------------------------
// measurement helpers
// ---------------------------------------------------------------------------------------------
extern "C" int shud_rhs_device_alloc(shud_rhs_t h, size_t bytes, void **dptr) {
    if (!h || !dptr) return shud_fail(SHUD_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipMalloc(dptr, bytes ? bytes : 8));
    return SHUD_OK;
}
extern "C" int shud_rhs_device_free(shud_rhs_t h, void *dptr) {
    (void)h;
    HIP_TRY(hipFree(dptr));
    return SHUD_OK;
}
extern "C" int shud_rhs_memcpy(shud_rhs_t h, void *dst, const void *src, size_t bytes, int kind) {
    if (!h) return shud_fail(SHUD_ERR_ARG, "null argument");
    hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : kind == 2 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, k, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return SHUD_OK;
}
extern "C" int shud_rhs_synchronize(shud_rhs_t h) {
    if (!h) return shud_fail(SHUD_ERR_ARG, "null argument");
    HIP_TRY(hipStreamSynchronize(h->stream));
    return SHUD_OK;
}
extern "C" void *shud_rhs_stream(shud_rhs_t h) { return h ? (void *)h->stream : nullptr; }

// halo buffers of a partitioned handle (external-transport tests move them between handles)
extern "C" int shud_rhs_halo_buffers(shud_rhs_t h, double **esend, double **rsend, double **gele, double **griv) {
    if (!h || !h->partitioned) return shud_fail(SHUD_ERR_ARG, "not a partitioned handle");
    *esend = h->d_esend; *rsend = h->d_rsend; *gele = h->d_gele; *griv = h->d_griv;
    return SHUD_OK;
}
// test hook: a late, kernel-written or missing halo on the comm stream of every following device eval
extern "C" int shud_rhs_debug_halo(shud_rhs_t h, double spin_us, const double *d_ele_src, const double *d_riv_src,
                                   int publish, double timeout_ms) {
    if (!h || !h->partitioned) return shud_fail(SHUD_ERR_ARG, "not a partitioned handle");
    if (spin_us < 0 || spin_us > 1e7) return shud_fail(SHUD_ERR_ARG, "spin_us out of range");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipStreamSynchronize(h->s_comm));
    h->dbg_spin = (unsigned long long)(spin_us * 1e-3 * h->wall_khz);
    h->dbg_gele = d_ele_src;
    h->dbg_griv = d_riv_src;
    h->dbg_publish = publish != 0;
    h->dbg_armed = h->dbg_spin || d_ele_src || d_riv_src || !h->dbg_publish;
    const double ms = timeout_ms > 0 ? timeout_ms : env_knob("SHUD_HALO_TIMEOUT_MS", 5000, 1, 3600000);
    h->halo_timeout = (unsigned long long)(ms * h->wall_khz);
    return SHUD_OK;
}
// split eval for external transport: pack, (caller exchanges), compute
extern "C" int shud_rhs_eval_pack(shud_rhs_t h, const double *d_y) {
    if (!h || !h->partitioned) return shud_fail(SHUD_ERR_ARG, "not a partitioned handle");
    launch_pack_kernel(d_y, h->n_own, h->n_own_riv, h->d_esend_idx, h->n_esend, h->d_rsend_idx, h->n_rsend,
                       h->d_esend, h->d_rsend, h->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->ev_comm, h->stream));      // what eval_compute's boundary launch waits for
    return SHUD_OK;
}
extern "C" int shud_rhs_eval_compute(shud_rhs_t h, double t, const double *d_y, double *d_ydot) {
    (void)t;
    if (!h) return shud_fail(SHUD_ERR_ARG, "null argument");
    h->last_cur = h->cur;
    h->last_cur_e = h->cur_e;
    int rc = launch_split(h, d_y, d_ydot, nullptr, true);
    if (rc) return rc;
    flip(h);
    h->last_y = d_y;
    h->have_last = true;
    h->ncalls++;
    return SHUD_OK;
}

extern "C" int shud_rhs_timing(shud_rhs_t h, int max_evals, int stride) {
    if (!h || max_evals < 0 || stride < 1) return shud_fail(SHUD_ERR_ARG, "bad argument");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    const size_t need = 3 * (size_t)max_evals;
    while (h->tm_ev.size() < need) {
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, kEvTime));
        h->tm_ev.push_back(e);
    }
    h->tm_cap = max_evals;
    h->tm_n = 0;
    h->tm_seen = 0;
    h->tm_stride = stride;
    return SHUD_OK;
}

extern "C" int shud_rhs_timing_read(shud_rhs_t h, double *ms_ele, double *ms_riv, double *ms_eval, int *n_evals) {
    if (!h) return shud_fail(SHUD_ERR_ARG, "null handle");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    double a = 0., b = 0., c = 0.;
    for (int r = 0; r < h->tm_n; r++) {
        hipEvent_t *E = &h->tm_ev[3 * (size_t)r];
        float x = 0.f, y = 0.f, z = 0.f;
        HIP_TRY(hipEventElapsedTime(&x, E[0], E[1]));
        HIP_TRY(hipEventElapsedTime(&y, E[1], E[2]));
        HIP_TRY(hipEventElapsedTime(&z, E[0], E[2]));
        a += x; b += y; c += z;
    }
    const int n = h->tm_n;
    if (ms_ele) *ms_ele = n ? a / n : 0.;
    if (ms_riv) *ms_riv = n ? b / n : 0.;
    if (ms_eval) *ms_eval = n ? c / n : 0.;
    if (n_evals) *n_evals = n;
    h->tm_n = 0;
    h->tm_cap = 0;
    return SHUD_OK;
}

extern "C" int shud_rhs_time_kernels(shud_rhs_t h, double t, const double *d_y, double *d_ydot, int reps,
                                     double *ms_eval, double *ms_out, int *nk, char *names_out, int names_len) {
    (void)t;
    if (!h || reps <= 0) return shud_fail(SHUD_ERR_ARG, "bad argument");
    HIP_TRY(hipSetDevice(h->device));
    const int K = h->partitioned ? 3 : 2;
    std::vector<hipEvent_t> ev((size_t)reps * (K + 1));
    for (auto &e : ev) HIP_TRY(hipEventCreateWithFlags(&e, kEvTime));
    for (int r = 0; r < reps; r++) {
        hipEvent_t *E = &ev[(size_t)r * (K + 1)];
        int k = 0;
        HIP_TRY(hipEventRecord(E[k++], h->stream));
        if (h->partitioned) {
            int rc = exchange(h, d_y);        // serialized here (no overlap) so each phase is timed alone
            if (rc) return rc;
            HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_comm, 0));
            HIP_TRY(hipEventRecord(E[k++], h->stream));
        }
        launch_ele(h, d_y, d_ydot, h->cur, h->cur_e, false);
        HIP_TRY(hipEventRecord(E[k++], h->stream));
        launch_riv(h, d_y, d_ydot, false);
        HIP_TRY(hipEventRecord(E[k++], h->stream));
        h->last_cur = h->cur; h->last_cur_e = h->cur_e;
        flip(h);
        h->last_y = d_y; h->have_last = true; h->ncalls++;
    }
    HIP_TRY(hipStreamSynchronize(h->stream));
    std::vector<double> acc(K, 0.0);
    double tot = 0.0;
    for (int r = 0; r < reps; r++) {
        hipEvent_t *E = &ev[(size_t)r * (K + 1)];
        for (int k = 0; k < K; k++) {
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, E[k], E[k + 1]));
            acc[k] += ms;
        }
        float all = 0.f;
        HIP_TRY(hipEventElapsedTime(&all, E[0], E[K]));
        tot += all;
    }
    for (auto &e : ev) (void)hipEventDestroy(e);
    const char *nm = h->partitioned ? "halo_exchange,shud_ele_kernel,shud_riv_kernel" : "shud_ele_kernel,shud_riv_kernel";
    int n = std::min(*nk, K);
    for (int k = 0; k < n; k++) ms_out[k] = acc[k] / reps;
    *nk = K;
    if (ms_eval) *ms_eval = tot / reps;
    if (names_out && names_len > 0) snprintf(names_out, names_len, "%s", nm);
    return SHUD_OK;
}
