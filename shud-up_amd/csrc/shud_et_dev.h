// shud_et_dev.h — device-side structures of the ET-step prelude (shud_et.hip / shud_et.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include "shud_dev.h"

namespace shud {

struct DevEt {                       // per element: statics, carried state, outputs (SoA)
    int ne;
    const int *iforc, *ilc, *imf, *ilake;
    const double *z_surf, *albedo, *fixp, *windh, *vegf, *nx, *ny, *nz;
    double *y_is, *y_snow, *tsr_factor;                       // carried
    double *ring_surf, *ring_sub;                             // cryosphere day-mean queues [cap][ne]
    double *tacc_surf, *tacc_sub, *acc_surf, *acc_sub;        // T_AccDay, ACC per element
    double *t_prcp, *t_temp, *t_lai, *t_mf, *t_rn, *t_wind, *t_rh, *rn_factor;
    double *rn_h, *rn_t;                                      // ele_rn_h_wm2 / ele_rn_t_wm2 (MD_ET.cpp:201-202)
    double *q_prep, *q_pet, *q_ptr, *q_etp, *q_netp, *q_eic, *fu_surf, *fu_sub;
};

struct EtStepDev {                   // per ET step (uniform across threads)
    double t, t_next;
    const double *station, *station_z, *lai_row, *mf_row;     // device copies of the current rows
    double cPrep, cTemp, cLAItsd, cMF, cETP, cISmax;
    int terrain, tsr_mode, tsr_n, radiation_input_mode;
    const double *tsr_sx, *tsr_sy, *tsr_sz, *tsr_wdt;
    double tsr_den, rad_factor_cap, rad_cosz_min;
    int cryosphere, push_day, n_of_day;
    int surf_tail, surf_head, surf_pop, surf_size, sub_tail, sub_head, sub_pop, sub_size;
    double ft_surf_max, ft_surf_min, ft_sub_max, ft_sub_min;
    int packed;
    double2 *s_np, *s_tl, *s_fu, *cs_cur;                     // packed RHS records (when packed)
    int *sfl;                                                 // packed seg_first words: bit 31 = LAI > ZERO
};

void launch_et_kernel(const DevEt &e, const EtStepDev &s, DevErr *err, hipStream_t st);

}  // namespace shud
