/* shud_out.h — C-ABI of the output path on the device (`.dat` binary outputs).
 *
 * Replaces, for a model whose state and fluxes live in HBM (shud_rhs.h / shud_ode.h), the reference's
 *   Model_Data::summary(udata)          src/ModelData/MD_update.cpp:190-216   -> shud_rhs_summary
 *   Control_Data::ExportResults(t)      src/classes/Model_Control.cpp:123-127 -> shud_out_export
 *   Print_Ctrl::Init / InitIJ           src/classes/Model_Control.cpp:759-858 -> shud_out_add
 *   Print_Ctrl::open_file               src/classes/Model_Control.cpp:683-758 (1024-B header, StartTime,
 *                                        NumVar, icol[NumVar]; optional ASCII twin)
 *   Print_Ctrl::PrintData               src/classes/Model_Control.cpp:926-960 (running sum, mean over the
 *                                        interval times tau, quantised left-endpoint time stamp, reset)
 *   Print_Ctrl::fun_printBINARY/ASCII   src/classes/Model_Control.cpp:893-909
 * Each exported step adds every registered variable into its device-resident buffer with one batched
 * kernel (no PCIe traffic); only at the end of an output interval is the buffer scaled on the device,
 * copied to the host and written, in the reference's byte layout.  NetCDF sinks are out of scope.
 */
#ifndef SHUD_OUT_H
#define SHUD_OUT_H

#include <stdint.h>

#include "shud_rhs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* device arrays a print control can point at (shud_rhs_device_array) */
enum {
    /* Model_Data::summary (filled by shud_rhs_summary from a state vector) */
    SHUD_ARR_Y_ELE_SURF = 0,     /* yEleSurf                                     NE  */
    SHUD_ARR_Y_ELE_UNSAT,        /* yEleUnsat                                    NE  */
    SHUD_ARR_Y_ELE_GW,           /* yEleGW (yBC where iBC > 0)                   NE  */
    SHUD_ARR_Y_RIV_STG,          /* yRivStg (Riv.yBC where BC > 0)              NR  */
    SHUD_ARR_Y_LAKE_STG,         /* yLakeStg                                     NL  */
    /* fluxes of the last RHS evaluation (filled by shud_rhs_refresh_diagnostics) */
    SHUD_ARR_QELE_SURF_TOT,      /* QeleSurfTot                                  NE  */
    SHUD_ARR_QELE_SUB_TOT,       /* QeleSubTot                                   NE  */
    SHUD_ARR_QELE_SURF,          /* QeleSurf, edge-major [3][NE]: column j at +j*NE   */
    SHUD_ARR_QELE_SUB,           /* QeleSub,  edge-major [3][NE]                      */
    SHUD_ARR_QE2R_SURF,          /* Qe2r_Surf                                    NE  */
    SHUD_ARR_QE2R_SUB,           /* Qe2r_Sub                                     NE  */
    SHUD_ARR_Q_INFIL,            /* qEleInfil                                    NE  */
    SHUD_ARR_Q_EXFIL,            /* qEleExfil                                    NE  */
    SHUD_ARR_Q_RECHARGE,         /* qEleRecharge                                 NE  */
    SHUD_ARR_Q_ETA,              /* qEleETA                                      NE  */
    SHUD_ARR_Q_E_IC,             /* qEleE_IC (as mutated by the last RHS)        NE  */
    SHUD_ARR_Q_TRANS,            /* qEleTrans = qTu + qTg (MD_ET.cpp:384)       NE  */
    SHUD_ARR_Q_EVAPO,            /* qEleEvapo = qEu + qEg + qEs (MD_ET.cpp:385) NE  */
    SHUD_ARR_QRIV_DOWN,          /* QrivDown                                     NR  */
    SHUD_ARR_QRIV_UP,            /* QrivUp                                       NR  */
    SHUD_ARR_QRIV_SURF,          /* QrivSurf                                     NR  */
    SHUD_ARR_QRIV_SUB,           /* QrivSub                                      NR  */
    /* per-ET-step inputs on the device (after shud_rhs_set_step_inputs or shud_et_step) */
    SHUD_ARR_Q_PRCP,             /* qElePrep                                     NE  */
    SHUD_ARR_Q_NET_PRCP,         /* qEleNetPrep                                  NE  */
    SHUD_ARR_Q_ETP,              /* qEleETP                                      NE  */
    /* ET-step prelude state (shud_et_attach'ed handles; NULL otherwise) */
    SHUD_ARR_Y_ELE_IS,           /* yEleIS (interception storage)                NE  */
    SHUD_ARR_Y_ELE_SNOW,         /* yEleSnow                                     NE  */
    SHUD_ARR_RN_H,               /* ele_rn_h_wm2: forcing shortwave (MD_ET.cpp:201) NE */
    SHUD_ARR_RN_T,               /* ele_rn_t_wm2: terrain-corrected shortwave    NE  */
    SHUD_ARR_RN_FACTOR,          /* ele_rn_factor: TSR factor                    NE  */
    /* lake fluxes of the last RHS evaluation (lake models; MD_initialize.cpp:331-342 order) */
    SHUD_ARR_LAKE_TOPAREA,       /* y2LakeArea                                   NL  */
    SHUD_ARR_Q_LAKE_EVAP,        /* qLakeEvap                                    NL  */
    SHUD_ARR_Q_LAKE_PRCP,        /* qLakePrcp                                    NL  */
    SHUD_ARR_Q_LAKE_RIVIN,       /* QLakeRivIn                                   NL  */
    SHUD_ARR_Q_LAKE_RIVOUT,      /* QLakeRivOut: zeroed by f_update, never assigned (MD_update.cpp:184) NL */
    SHUD_ARR_Q_LAKE_SURF,        /* QLakeSurf                                    NL  */
    SHUD_ARR_Q_LAKE_SUB,         /* QLakeSub                                     NL  */
    SHUD_ARR_COUNT
};

/* fills the SHUD_ARR_Y_* arrays from y (device pointer, NY values; the Model_Data::summary step) */
int shud_rhs_summary(shud_rhs_t h, const double *d_y);
/* replays the last RHS evaluation with diagnostic stores into the device arrays (no host copy; carried
 * state unchanged): what the reference's flux arrays hold after CVODE's last f() call */
int shud_rhs_refresh_diagnostics(shud_rhs_t h);
/* allocates every array above (zero-filled) without evaluating anything, so print controls can be registered
 * before the first RHS call (the serial RHS is stateful: an extra evaluation would change the trajectory) */
int shud_rhs_prepare_outputs(shud_rhs_t h);
/* device pointer of one of the arrays above (NULL if unknown / not yet materialised) and its length */
const double *shud_rhs_device_array(shud_rhs_t h, int which, int64_t *n);

typedef struct shud_out *shud_out_t;

typedef struct {
    const char *basename;        /* Print_Ctrl::filename: writes <basename>.dat and/or <basename>.csv     */
    const double *d_src;         /* device array with n_all values (PrintVar targets), stride 1             */
    int32_t n_all;               /* NumAll                                                                  */
    const int32_t *flag_io;      /* host, n_all flags (Init with flag_IO); NULL = every column              */
    int32_t interval;            /* Interval [min] (> 0; the reference exits with ERRCONSIS on 0)           */
    int32_t iflux;               /* tau = 1440 if iflux else 1                                              */
    int64_t start_time;          /* StartTime (ForcStartTime, written into the header as a double)          */
    int32_t binary, ascii;       /* files to write (reference defaults: binary 1, ascii 0)                  */
    int32_t radiation_input_mode;/* header: 0 SWDOWN, 1 SWNET                                               */
    int32_t terrain_radiation;   /* header: TSR ON/OFF                                                      */
    const char *solar_lonlat_mode; /* header: SolarLonLatModeName(...)                                      */
    double solar_lon_deg, solar_lat_deg;
} ShudPrintSpec;

/* an output set on `stream` (hipStream_t; NULL = the default stream) of `device` */
int shud_out_create(int device, void *stream, shud_out_t *out);
/* Print_Ctrl::Init[IJ] + open_file: creates/truncates the files and writes their headers */
int shud_out_add(shud_out_t o, const ShudPrintSpec *spec);
/* Control_Data::ExportResults(t): every control adds its source into its buffer; controls whose interval
 * ends at t (floor(t + 0.001) % Interval == 0) write the interval mean and reset.  Sources must hold the
 * values to export (shud_rhs_summary / shud_rhs_refresh_diagnostics first), stream-ordered.  The rows of a
 * finished interval reach the files asynchronously (copy stream + writer thread; same bytes, same order):
 * shud_out_flush / shud_out_rows / shud_out_destroy wait for them. */
int shud_out_export(shud_out_t o, double t);
/* wait until every exported row is written to the files (fflush'ed).  Returns the first failure of the
 * asynchronous writer (a failed snapshot copy: that row is not written; a file write / flush error) */
int shud_out_flush(shud_out_t o);
/* number of rows written so far by control k (tests; waits for the writer); a writer failure returns its
 * negative SHUD_ERR_* code */
int64_t shud_out_rows(shud_out_t o, int k);
/* flushes and closes the files, frees the buffers; returns the writer's first failure, if any */
int shud_out_destroy(shud_out_t o);

#ifdef __cplusplus
}
#endif
#endif /* SHUD_OUT_H */
