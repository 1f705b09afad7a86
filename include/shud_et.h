/* shud_et.h — C-ABI of the ET-step prelude on the device.
 *
 * Replaces, per ET step, the reference's
 *   Model_Data::updateforcing(t)  src/ModelData/MD_ET.cpp:14-20   (its tReadForcing half; the
 *                                                                  updateElement half is the RHS handle's
 *                                                                  carried u_satn, see below)
 *   Model_Data::tReadForcing(t,i) src/ModelData/MD_ET.cpp:21-281  (forcing, TSR terrain radiation factor,
 *                                                                  Penman-Monteith PET / open-water PET)
 *   Model_Data::ET(t, tnext)      src/ModelData/MD_ET.cpp:282-341 (snow, interception, cryosphere fu)
 * as called from the time loop (src/Model/shud.cpp:106-109).  Its outputs are written straight into the
 * RHS handle's device step inputs (qEleNetPrep, qPotEvap, qPotTran, qEleETP, t_lai, fu_Surf, fu_Sub and the
 * carried qEleE_IC): after shud_et_step, no per-step host->device copy of step inputs is needed.
 *
 * u_satn: updateforcing's Ele[i].updateElement(uYsf, uYus, uYgw) (MD_ET.cpp:17) recomputes u_satn from the
 * globals the last RHS call left; the handle's carried u_satn is exactly that value (same formula, same
 * state), so the prelude does not touch it.  Before the first RHS call pass it once through
 * shud_rhs_set_step_inputs (ShudStepInputs.u_satn), as the reference's initialisation does.
 *
 * Shared per-interval work stays on the host, as in the reference: the current forcing rows (zero-order
 * hold, _TimeSeriesData::getX ignores t: TimeSeriesData.cpp:270-273) and the TSR solar samples of the
 * forcing interval (MD_ET.cpp:66-136; the bucket bookkeeping decides tsr_mode below).
 */
#ifndef SHUD_ET_H
#define SHUD_ET_H

#include <stdint.h>

#include "shud_rhs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* per-element statics of the prelude (local elements of a partitioned handle: owned + ghosts) */
typedef struct {
    int32_t num_ele;              /* must equal the RHS handle's element count                      */
    const int32_t *iforc;         /* forcing station, 0-based (Ele[i].iForc - 1)                    */
    const int32_t *ilc;           /* LAI column of tsd_LAI, Ele[i].iLC (1-based: column 0 is time)  */
    const int32_t *imf;           /* melt-factor column of tsd_MF, Ele[i].iMF (1-based)             */
    const double *z_surf;
    const double *albedo;         /* Ele[i].Albedo                                                  */
    const double *fix_pressure;   /* Ele[i].FixPressure = PressureElevation(z_surf) (Element.cpp:222)*/
    const double *wind_h;         /* Ele[i].windH (HeightWindMeasure, MD_initialize.cpp:182)        */
    const double *veg_frac;       /* Ele[i].VegFrac                                                 */
    const int32_t *ilake;         /* Ele[i].iLake (> 0: open-water PET)                             */
    const double *nx, *ny, *nz;   /* element unit normal (Element.cpp:160-190); NULL if TSR off     */
} ShudEtMeshSoA;

typedef struct {
    double cPrep, cTemp, cLAItsd, cMF, cETP, cISmax;   /* gc.* calibration (Model_Control)          */
    int32_t radiation_input_mode;                      /* 0 SWDOWN (x (1 - Albedo)), 1 SWNET        */
    int32_t terrain_radiation;                         /* CS.terrain_radiation                      */
    double rad_factor_cap, rad_cosz_min;               /* CS.rad_factor_cap, CS.rad_cosz_min        */
    int32_t cryosphere;                                /* CS.cryosphere: frozen-ground fu           */
    int32_t ft_surf_day, ft_sub_day;                   /* gc.cfrozen.FT_*_Day (accumulator lengths) */
    double ft_surf_max, ft_surf_min, ft_sub_max, ft_sub_min;
} ShudEtParams;

/* TSR factor source for this step (MD_ET.cpp:62-200), decided by the host's bucket bookkeeping */
enum {
    SHUD_TSR_OFF = 0,        /* terrain_radiation == 0: factor 1                                     */
    SHUD_TSR_NO_TIME = 1,    /* forcing t0 not finite: factor 0 this step, cache untouched (:68-69)   */
    SHUD_TSR_CACHED = 2,     /* same forcing interval as the cached factors (tsr_factor_bucket == b)  */
    SHUD_TSR_RECOMPUTE = 3   /* new interval: recompute every element's factor from the samples       */
};

typedef struct {
    double t, t_next;                  /* ET step [t, t_next) in minutes (ET(t, tout), shud.cpp:109)    */
    int32_t n_station;
    const double *station;             /* [n_station][6]: current tsd_weather row (time, APCP, TMP,     */
                                       /*   RH, wind, radiation) — columns as i_prcp..i_rn (Macros.hpp) */
    const double *station_z;           /* [n_station] tsd_weather[k].xyz[2] (NA_VALUE = -9999 allowed)  */
    int32_t n_lai_col;                 /* columns of the tsd_LAI row (incl. time)                       */
    const double *lai_row;
    int32_t n_mf_col;
    const double *mf_row;
    int32_t tsr_mode;                  /* SHUD_TSR_*                                                    */
    int32_t tsr_n;                     /* samples of the interval (tsr_forcing_n)                       */
    const double *tsr_sx, *tsr_sy, *tsr_sz, *tsr_wdt;
    double tsr_den;                    /* tsr_forcing_den                                               */
} ShudEtForcing;

/* host copies of the prelude's per-element outputs/state (any pointer may be NULL) */
typedef struct {
    double *t_prcp, *t_temp, *t_lai, *t_mf, *t_rn, *t_wind, *t_rh;
    double *qEleprep, *qPotEvap, *qPotTran, *qEleETP, *qEleNetPrep, *qEleE_IC;
    double *yEleIS, *yEleSnow, *fu_surf, *fu_sub, *rn_factor;
} ShudEtOut;

/* attach the prelude to an RHS handle (once, after shud_rhs_create[_partitioned]) */
int shud_et_attach(shud_rhs_t h, const ShudEtMeshSoA *mesh, const ShudEtParams *par);
/* initial storages yEleIS / yEleSnow (LoadIC), host arrays of num_ele; NULL keeps the current value (0) */
int shud_et_set_state(shud_rhs_t h, const double *y_is, const double *y_snow);
/* one ET step: tReadForcing for every element, then ET(); writes the RHS step inputs on the device.
 * Errors as the reference's myexit(10): CheckNonZero(ra) and CheckNANi(qPotTran) -> SHUD_ERR_PHYSICS,
 * details in shud_rhs_get_error (flags SHUD_EF_ET_RA / SHUD_EF_ET_PT_NAN, first element index). */
int shud_et_step(shud_rhs_t h, const ShudEtForcing *f);
int shud_et_get(shud_rhs_t h, ShudEtOut *out);

#ifdef __cplusplus
}
#endif
#endif /* SHUD_ET_H */
