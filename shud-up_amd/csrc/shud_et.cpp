// shud_et.cpp — host runtime of the ET-step prelude (include/shud_et.h).
//
// Keeps, per RHS handle, the prelude's device statics and carried state (yEleIS, yEleSnow, TSR factor
// cache, cryosphere day-mean queues) and, per ET step, uploads the few KB of shared rows (forcing stations,
// LAI and melt-factor rows, TSR solar samples) in one copy, then runs one fused kernel that writes the RHS
// step inputs in place.  The queue bookkeeping every element shares (AccTemperature.hpp: N_of_day,
// Time_start, queue length/front) lives here; the per-element sums live on the device.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstring>
#include <vector>

#include "shud_et.h"
#include "shud_out.h"
#include "shud_et_dev.h"
#include "shud_handle.h"

struct EtState {
    DevEt e{};
    ShudEtParams par{};
    bool tsr_ready = false;             // factors computed at least once
    int max_forc = -1, max_lc = -1, max_mf = -1;   // highest station / LAI / MF column referenced
    // cryosphere shared bookkeeping (_AccTemp: Time_start, N_of_day, queue of day means)
    double time_start = -9999.;
    int n_of_day = 0;
    int cap_surf = 1, cap_sub = 1, head_surf = 0, size_surf = 0, head_sub = 0, size_sub = 0;
    // per-step upload: [station 6*ns | station_z ns | lai ncol | mf ncol | tsr 4*n]
    double *d_stage = nullptr;
    size_t stage_cap = 0;
    std::vector<double> h_stage;
};

void shud_et_free(shud_rhs *h) {
    if (h && h->et) {
        delete h->et;
        h->et = nullptr;
    }
}

extern "C" int shud_et_attach(shud_rhs_t h, const ShudEtMeshSoA *m, const ShudEtParams *p) {
    if (!h || !m || !p) return shud_fail(SHUD_ERR_ARG, "null argument");
    if (h->et) return shud_fail(SHUD_ERR_ARG, "ET prelude already attached");
    const int NE = h->NE;
    if (m->num_ele != NE) return shud_fail(SHUD_ERR_ARG, "ET mesh has %d elements, handle %d", m->num_ele, NE);
    if (!m->iforc || !m->ilc || !m->imf || !m->z_surf || !m->albedo || !m->fix_pressure || !m->wind_h ||
        !m->veg_frac)
        return shud_fail(SHUD_ERR_ARG, "missing ET mesh array");
    if (p->terrain_radiation && (!m->nx || !m->ny || !m->nz))
        return shud_fail(SHUD_ERR_ARG, "terrain_radiation needs element normals");
    if (p->cryosphere && (p->ft_surf_day < 0 || p->ft_sub_day < 0))
        return shud_fail(SHUD_ERR_ARG, "bad cryosphere accumulator length");
    int mx[3] = {-1, -1, -1};
    for (int i = 0; i < NE; i++) {
        if (m->iforc[i] < 0 || m->ilc[i] < 1 || m->imf[i] < 1)
            return shud_fail(SHUD_ERR_ARG, "element %d: iforc < 0 or iLC/iMF < 1", i);
        mx[0] = std::max(mx[0], m->iforc[i]);
        mx[1] = std::max(mx[1], m->ilc[i]);
        mx[2] = std::max(mx[2], m->imf[i]);
    }
    HIP_TRY(hipSetDevice(h->device));
    EtState *s = new EtState();
    s->max_forc = mx[0]; s->max_lc = mx[1]; s->max_mf = mx[2];
    h->et = s;
    s->par = *p;
    DevEt &e = s->e;
    e.ne = NE;
    int rc;
    int *iforc, *ilc, *imf, *ilake;
    double *dz, *dalb, *dfp, *dwh, *dvf, *dnx = nullptr, *dny = nullptr, *dnz = nullptr;
    if ((rc = h->upload(&iforc, m->iforc, NE)) || (rc = h->upload(&ilc, m->ilc, NE)) ||
        (rc = h->upload(&imf, m->imf, NE)) || (rc = h->upload_fill(&ilake, m->ilake, NE, 0)) ||
        (rc = h->upload(&dz, m->z_surf, NE)) || (rc = h->upload(&dalb, m->albedo, NE)) ||
        (rc = h->upload(&dfp, m->fix_pressure, NE)) || (rc = h->upload(&dwh, m->wind_h, NE)) ||
        (rc = h->upload(&dvf, m->veg_frac, NE)))
        return rc;
    if (p->terrain_radiation &&
        ((rc = h->upload(&dnx, m->nx, NE)) || (rc = h->upload(&dny, m->ny, NE)) || (rc = h->upload(&dnz, m->nz, NE))))
        return rc;
    e.iforc = iforc; e.ilc = ilc; e.imf = imf; e.ilake = ilake;
    e.z_surf = dz; e.albedo = dalb; e.fixp = dfp; e.windh = dwh; e.vegf = dvf; e.nx = dnx; e.ny = dny; e.nz = dnz;
    double **state[] = {&e.y_is, &e.y_snow, &e.tsr_factor, &e.tacc_surf, &e.tacc_sub, &e.acc_surf, &e.acc_sub,
                        &e.t_prcp, &e.t_temp, &e.t_mf, &e.t_rn, &e.t_wind, &e.t_rh, &e.rn_factor, &e.rn_h, &e.rn_t};
    for (double **q : state)
        if ((rc = h->upload(q, (const double *)nullptr, NE))) return rc;   // zero: ACC starts at 0 (see DESIGN)
    if (p->cryosphere) {
        s->cap_surf = p->ft_surf_day + 1;
        s->cap_sub = p->ft_sub_day + 1;
        if ((rc = h->upload(&e.ring_surf, (const double *)nullptr, (size_t)s->cap_surf * NE)) ||
            (rc = h->upload(&e.ring_sub, (const double *)nullptr, (size_t)s->cap_sub * NE)))
            return rc;
    }
    // the RHS step inputs are the prelude's outputs (SoA staging of the handle; the handle owns them —
    // DevMesh declares them const only for the RHS kernels)
    e.t_lai = const_cast<double *>(h->dm.lai);
    e.q_pet = const_cast<double *>(h->dm.pot_evap);
    e.q_ptr = const_cast<double *>(h->dm.pot_tran);
    e.q_etp = const_cast<double *>(h->dm.etp);
    e.q_netp = const_cast<double *>(h->dm.net_prep);
    e.fu_surf = const_cast<double *>(h->dm.fu_surf);
    e.fu_sub = const_cast<double *>(h->dm.fu_sub);
    e.q_prep = const_cast<double *>(h->dm.prcp);           // qElePrep: lake elements' precipitation
    return SHUD_OK;
}

extern "C" int shud_et_set_state(shud_rhs_t h, const double *y_is, const double *y_snow) {
    if (!h || !h->et) return shud_fail(SHUD_ERR_ARG, "no ET prelude attached");
    HIP_TRY(hipSetDevice(h->device));
    const size_t nb = (size_t)h->NE * sizeof(double);
    if (y_is) HIP_TRY(hipMemcpy(h->et->e.y_is, y_is, nb, hipMemcpyHostToDevice));
    if (y_snow) HIP_TRY(hipMemcpy(h->et->e.y_snow, y_snow, nb, hipMemcpyHostToDevice));
    return SHUD_OK;
}

extern "C" int shud_et_step(shud_rhs_t h, const ShudEtForcing *f) {
    if (!h || !h->et || !f) return shud_fail(SHUD_ERR_ARG, "no ET prelude attached / null forcing");
    EtState *s = h->et;
    const ShudEtParams &p = s->par;
    if (f->n_station <= 0 || !f->station || !f->station_z || !f->lai_row || !f->mf_row || f->n_lai_col <= 0 ||
        f->n_mf_col <= 0)
        return shud_fail(SHUD_ERR_ARG, "missing forcing rows");
    const int tsr_mode = p.terrain_radiation ? f->tsr_mode : SHUD_TSR_OFF;
    if (p.terrain_radiation && (tsr_mode < 1 || tsr_mode > 3))
        return shud_fail(SHUD_ERR_ARG, "terrain_radiation: tsr_mode must be 1..3");
    if (tsr_mode == SHUD_TSR_CACHED && !s->tsr_ready)
        return shud_fail(SHUD_ERR_ARG, "tsr_mode CACHED before any RECOMPUTE");
    const int ntsr = (tsr_mode == SHUD_TSR_RECOMPUTE) ? f->tsr_n : 0;
    if (ntsr < 0 || (ntsr > 0 && (!f->tsr_sx || !f->tsr_sy || !f->tsr_sz || !f->tsr_wdt)))
        return shud_fail(SHUD_ERR_ARG, "missing TSR samples");
    HIP_TRY(hipSetDevice(h->device));
    // every index the kernel will use must be inside the rows given (checked against attach-time maxima)
    if (f->n_station <= s->max_forc || f->n_lai_col <= s->max_lc || f->n_mf_col <= s->max_mf)
        return shud_fail(SHUD_ERR_ARG, "forcing rows too short: %d stations / %d LAI / %d MF columns, mesh uses "
                         "%d / %d / %d", f->n_station, f->n_lai_col, f->n_mf_col, s->max_forc + 1, s->max_lc + 1,
                         s->max_mf + 1);
    const int ns = f->n_station;
    const size_t n_stage = 6 * (size_t)ns + ns + f->n_lai_col + f->n_mf_col + 4 * (size_t)ntsr;
    s->h_stage.resize(n_stage);
    double *w = s->h_stage.data();
    memcpy(w, f->station, sizeof(double) * 6 * ns); w += 6 * ns;
    memcpy(w, f->station_z, sizeof(double) * ns); w += ns;
    memcpy(w, f->lai_row, sizeof(double) * f->n_lai_col); w += f->n_lai_col;
    memcpy(w, f->mf_row, sizeof(double) * f->n_mf_col); w += f->n_mf_col;
    if (ntsr) {
        memcpy(w, f->tsr_sx, sizeof(double) * ntsr); w += ntsr;
        memcpy(w, f->tsr_sy, sizeof(double) * ntsr); w += ntsr;
        memcpy(w, f->tsr_sz, sizeof(double) * ntsr); w += ntsr;
        memcpy(w, f->tsr_wdt, sizeof(double) * ntsr); w += ntsr;
    }
    if (n_stage > s->stage_cap) {
        int rc = h->dalloc(&s->d_stage, n_stage);
        if (rc) return rc;
        s->stage_cap = n_stage;
    }
    HIP_TRY(hipMemcpyAsync(s->d_stage, s->h_stage.data(), n_stage * sizeof(double), hipMemcpyHostToDevice, h->stream));

    EtStepDev d{};
    d.t = f->t; d.t_next = f->t_next;
    const double *b = s->d_stage;
    d.station = b; b += 6 * ns;
    d.station_z = b; b += ns;
    d.lai_row = b; b += f->n_lai_col;
    d.mf_row = b; b += f->n_mf_col;
    d.tsr_sx = b; d.tsr_sy = b + ntsr; d.tsr_sz = b + 2 * ntsr; d.tsr_wdt = b + 3 * ntsr;
    d.cPrep = p.cPrep; d.cTemp = p.cTemp; d.cLAItsd = p.cLAItsd; d.cMF = p.cMF; d.cETP = p.cETP; d.cISmax = p.cISmax;
    d.terrain = p.terrain_radiation ? 1 : 0;
    d.tsr_mode = tsr_mode; d.tsr_n = ntsr; d.tsr_den = f->tsr_den;
    d.radiation_input_mode = p.radiation_input_mode;
    d.rad_factor_cap = p.rad_factor_cap; d.rad_cosz_min = p.rad_cosz_min;
    // cryosphere: _AccTemp::push(x, tnow) bookkeeping shared by every element (AccTemperature.hpp:48-58)
    d.cryosphere = p.cryosphere ? 1 : 0;
    int pop_surf = 0, pop_sub = 0;
    if (p.cryosphere) {
        s->n_of_day++;
        d.n_of_day = s->n_of_day;
        d.push_day = (f->t - s->time_start) >= 1440. ? 1 : 0;
        if (d.push_day) {
            d.surf_tail = (s->head_surf + s->size_surf) % s->cap_surf;
            d.sub_tail = (s->head_sub + s->size_sub) % s->cap_sub;
            pop_surf = (s->size_surf + 1) > p.ft_surf_day;
            pop_sub = (s->size_sub + 1) > p.ft_sub_day;
        }
        d.surf_head = s->head_surf; d.sub_head = s->head_sub;
        d.surf_pop = pop_surf; d.sub_pop = pop_sub;
        d.surf_size = s->size_surf + d.push_day - pop_surf;
        d.sub_size = s->size_sub + d.push_day - pop_sub;
        d.ft_surf_max = p.ft_surf_max; d.ft_surf_min = p.ft_surf_min;
        d.ft_sub_max = p.ft_sub_max; d.ft_sub_min = p.ft_sub_min;
    }
    // outputs into the handle: carried qEleE_IC goes to the slot the next RHS reads
    DevEt e = s->e;
    e.q_eic = const_cast<double *>(h->packed ? h->dm.e_ic[0] : h->dm.e_ic[h->cur_e]);
    d.packed = h->packed ? 1 : 0;
    if (h->packed) {
        d.s_np = h->dp.s_np; d.s_tl = h->dp.s_tl; d.s_fu = h->dp.s_fu; d.cs_cur = h->dp.cs[h->cur];
        d.sfl = h->dp.seg_first;
    }
    launch_et_kernel(e, d, h->d_err, h->stream);
    HIP_TRY(hipGetLastError());
    // commit the shared bookkeeping the kernel used
    if (p.cryosphere && d.push_day) {
        s->size_surf += 1;
        s->size_sub += 1;
        if (pop_surf) { s->head_surf = (s->head_surf + 1) % s->cap_surf; s->size_surf -= 1; }
        if (pop_sub) { s->head_sub = (s->head_sub + 1) % s->cap_sub; s->size_sub -= 1; }
        s->n_of_day = 0;
        s->time_start = f->t;
    }
    if (tsr_mode == SHUD_TSR_RECOMPUTE) s->tsr_ready = true;
    h->fu_unit[0] = h->fu_unit[1] = !p.cryosphere;
    h->have_last = false;                 // step inputs changed: no diagnostic replay of the last RHS
    // the reference exits from tReadForcing (myexit(10)); report it like the RHS errors
    if (int rc = shud_read_err(h)) return rc;
    if (h->h_err->flags & (SHUD_EF_ET_RA | SHUD_EF_ET_PT_NAN))
        return shud_fail(SHUD_ERR_PHYSICS, "ET prelude error flags 0x%x", h->h_err->flags);
    return SHUD_OK;
}

extern "C" int shud_et_get(shud_rhs_t h, ShudEtOut *o) {
    if (!h || !h->et || !o) return shud_fail(SHUD_ERR_ARG, "no ET prelude attached / null output");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    const DevEt &e = h->et->e;
    const size_t nb = (size_t)h->NE * sizeof(double);
    const double *eic = h->packed ? h->dm.e_ic[0] : h->dm.e_ic[h->cur_e];
    struct { double *dst; const double *src; } m[] = {
        {o->t_prcp, e.t_prcp}, {o->t_temp, e.t_temp}, {o->t_lai, e.t_lai}, {o->t_mf, e.t_mf}, {o->t_rn, e.t_rn},
        {o->t_wind, e.t_wind}, {o->t_rh, e.t_rh}, {o->qEleprep, e.q_prep}, {o->qPotEvap, e.q_pet},
        {o->qPotTran, e.q_ptr}, {o->qEleETP, e.q_etp}, {o->qEleNetPrep, e.q_netp}, {o->qEleE_IC, eic},
        {o->yEleIS, e.y_is}, {o->yEleSnow, e.y_snow}, {o->fu_surf, e.fu_surf}, {o->fu_sub, e.fu_sub},
        {o->rn_factor, e.rn_factor}};
    for (auto &x : m)
        if (x.dst) HIP_TRY(hipMemcpy(x.dst, x.src, nb, hipMemcpyDeviceToHost));
    return SHUD_OK;
}

const double *shud_et_array(shud_rhs *h, int which) {
    if (!h || !h->et) return nullptr;
    const DevEt &e = h->et->e;
    switch (which) {
        case SHUD_ARR_Y_ELE_IS: return e.y_is;
        case SHUD_ARR_Y_ELE_SNOW: return e.y_snow;
        case SHUD_ARR_RN_H: return e.rn_h;
        case SHUD_ARR_RN_T: return e.rn_t;
        case SHUD_ARR_RN_FACTOR: return e.rn_factor;
        default: return nullptr;
    }
}
