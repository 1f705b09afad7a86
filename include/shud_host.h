/* shud_host.h — C-ABI of the C++ host that feeds the device path from a SHUD project directory
 * (SURVEY §8f f4 readers, f1 host side).  libshud_host.so is plain C++ (no HIP); the driver shud_gpu
 * (shud-up_amd/host/shud_gpu.cpp) and the Python tests sit on top of it.
 *
 * It replaces, for the device path, the host half of the reference's setup and time loop:
 *   FileIn paths                       src/classes/IO.cpp:53-91        (input/<prj>/<prj>.<ext>)
 *   Control_Data::read (.cfg.para)     src/classes/Model_Control.cpp:141-502
 *   globalCal::read/push (.cfg.calib)  src/classes/ModelConfigure.cpp:443-459, 109-262
 *   Model_Data::loadinput readers      src/ModelData/MD_readin.cpp:106-363 (mesh, att, soil, geol, lc,
 *                                      riv, rivseg), :555-729 (tsd.forc + forcing csv), :942-951 (lai, mf)
 *   TabularData::read                  src/classes/TabularData.cpp:27-55 (strtold per token)
 *   _TimeSeriesData read_csv/movePointer/getX  src/classes/TimeSeriesData.cpp (zero-order hold)
 *   Model_Data::initialize             src/ModelData/MD_initialize.cpp:168-245 (geometry, calibration,
 *                                      InitElement, rmSinks, applyNabor, rivers, segments)
 *   Model_Data::LoadIC (INIT_MODE 0-3) src/ModelData/MD_initialize.cpp:66-135
 *   Model_Data::initialize_output      src/ModelData/MD_initialize.cpp:246-345 (print controls)
 *   tReadForcing's shared TSR bucket   src/ModelData/MD_ET.cpp:60-136 + solarPosition
 *                                      (src/Equations/SolarRadiation.cpp:92-176, TimeContext.cpp)
 * All returned pointers are owned by the project and stay valid until shud_project_free (forcing rows:
 * until the next shud_project_forcing call).  Errors: non-zero return, message in shud_project_error().
 */
#ifndef SHUD_HOST_H
#define SHUD_HOST_H

#include <stdint.h>

#include "shud_et.h"
#include "shud_rhs.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct shud_project *shud_project_t;

/* Control_Data after read() (Model_Control.hpp:150-232 defaults; Model_Control.cpp:132-137, 502) */
typedef struct {
    double start_time, end_time;         /* CS.StartTime, CS.EndTime [min]                            */
    int64_t num_steps;                   /* CS.NumSteps = (EndTime - StartTime) / SolverStep          */
    double solver_step, et_step;         /* SolverStep (= MAX_SOLVER_STEP), ETStep (LSM_STEP/ET_STEP)  */
    double reltol, abstol, init_step, max_step;
    int32_t init_type, close_boundary, ascii, binary, cryosphere, verbose;
    int32_t terrain_radiation, radiation_input_mode, solar_lonlat_mode;   /* 0 FORCING_FIRST, 1 MEAN, 2 FIXED */
    double solar_lon_deg, solar_lat_deg;  /* selected after the forcing list is read (MD_readin.cpp:645-690) */
    double rad_factor_cap, rad_cosz_min;
    int32_t tsr_integration_step_min;
    int64_t forc_start_time;             /* ForcStartTime (yyyymmdd of the forcing list header)        */
    int32_t num_forc, lakeon, num_lake;
} ShudControl;

/* one print control of initialize_output (MD_initialize.cpp:246-345), in the reference's order */
typedef struct {
    const char *basename;                /* <outdir>/<prj>.<suffix> without extension                 */
    int32_t array;                       /* SHUD_ARR_* of shud_out.h                                   */
    int32_t column;                      /* InitIJ column (QeleSurf/QeleSub j) or -1                   */
    int32_t n_all;                       /* NumEle / NumRiv / NumLake                                  */
    int32_t interval, iflux;             /* Interval [min], 1 = flux (tau 1440)                        */
    const int32_t *flag_io;              /* io_ele / io_riv / io_lake of <prj>.cfg.output (read_cfgout,
                                            MD_readin.cpp:25-104); NULL = every column                   */
} ShudOutputDecl;

/* reads <indir>/<prj>.* and runs the reference's initialisation; `cwd` resolves the forcing csv paths
 * the way the reference (run from its repository root) does; NULL = the process cwd.  end_day >= 0
 * overrides END (days).  The forcing csv files are read in full at load. */
int shud_project_load(const char *indir, const char *prj, const char *cwd, double end_day, shud_project_t *out);
const char *shud_project_error(void);
void shud_project_free(shud_project_t p);

int shud_project_control(shud_project_t p, ShudControl *c);
/* the RHS handle inputs (pointers into the project) */
int shud_project_mesh(shud_project_t p, ShudMeshSoA *mesh, ShudParamsSoA *par);
/* the ET prelude statics and parameters (shud_et_attach) */
int shud_project_et(shud_project_t p, ShudEtMeshSoA *mesh, ShudEtParams *par);
/* named host arrays (tests, driver): "y0" (NY), "y_is", "y_snow" (NE; LoadIC), "x", "y" (centroids),
 * "slope_angle", "aspect" (applyGeometry), "albedo", "fix_pressure", "nx", "ny", "nz".  NULL if unknown. */
const double *shud_project_array(shud_project_t p, const char *name, int64_t *n);
/* print controls for output directory `outdir` (created by the caller); returns the count, fills up to max */
int shud_project_outputs(shud_project_t p, const char *outdir, ShudOutputDecl *decl, int max);

/* Per ET step [t, tout): updateAllTimeSeries(t) (movePointer of every forcing / LAI / MF series) and the
 * inputs of tReadForcing + ET for shud_et_step: the current station rows, LAI and MF rows, and the TSR
 * bucket decision with the solar samples of a new forcing interval (MD_ET.cpp:60-136).  Errors as the
 * reference's movePointer (missing forcing data -> message, code ERRFileIO). */
int shud_project_forcing(shud_project_t p, double t, double tout, ShudEtForcing *f);

/* Boundary-condition rows at the current ET step (after shud_project_forcing): the rows of <prj>.tsd.ebc1 /
 * .ebc2 / .rbc1 / .rbc2 that f_update reads through getX (MD_update.cpp:114-125, 145-160), as the ele_ybc /
 * ele_qbc / riv_ybc / riv_qbc fields (n_* = data columns) of `in`; the other fields are left untouched.
 * Returns 1 when the model has boundary conditions (pass `in` to shud_rhs_set_step_inputs), 0 otherwise. */
int shud_project_bc_rows(shud_project_t p, ShudStepInputs *in);

/* solarPosition(t_min, lat, lon, Time, tz) (SolarRadiation.cpp:92-176) with the project's ForcStartTime as
 * the base date: out[0..4] = cosZ, zenith, azimuth, declination, hourAngle (KAT tests) */
int shud_project_solar(shud_project_t p, double t_min, double lat_deg, double lon_deg, double tz_hours,
                       double *out5);

#ifdef __cplusplus
}
#endif
#endif /* SHUD_HOST_H */
