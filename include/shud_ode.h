/* shud_ode.h — C-ABI of the device-resident time integrator.
 *
 * Replaces the reference's SUNDIALS CVODE 6.0.0 instance (configure:17) as SetCVODE configures it
 * (src/Equations/cvode_config.cpp:149-197) and SHUD() drives it (src/Model/shud.cpp:89-131):
 *   CVodeCreate(CV_BDF) + CVodeInit(f, t0, y0)        -> shud_ode_create / shud_ode_create_fn
 *   CVodeSStolerances(reltol, abstol)                   ShudOdeOptions.reltol / abstol
 *   SUNLinSol_SPGMR(y, 0, 0) + CVodeSetLinearSolver      Newton + GMRES (maxl 5, no preconditioner,
 *                                                        modified Gram-Schmidt, DQ J*v), ShudOdeOptions.maxl
 *   CVodeSetMinStep / SetMaxNumSteps / SetInitStep / SetMaxStep   ShudOdeOptions
 *   CVodeSetStopTime(tout)                            -> shud_ode_set_stop_time
 *   CVode(mem, tout, y, &t, CV_NORMAL | CV_ONE_STEP)  -> shud_ode_solve
 *   CVodeGetDky(mem, t, k, dky)                       -> shud_ode_get_dky
 *   CVodeGet{NumSteps,NumRhsEvals,...} / PrintFinalStats (cvode_config.cpp:33-85) -> shud_ode_get_stats
 * The N_Vector lives in device memory (HBM) for the whole run: every RHS call is a device-pointer
 * shud_rhs_eval on the handle's stream, so no state crosses PCIe per RHS call (the reference's serial
 * N_Vector would cost 2*NY*8 bytes of PCIe per call).  Return codes are CVODE's (CV_SUCCESS = 0, ...).
 */
#ifndef SHUD_ODE_H
#define SHUD_ODE_H

#include <stdint.h>

#include "shud_rhs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* return codes (cvode.h values) */
#define SHUD_ODE_SUCCESS 0
#define SHUD_ODE_TSTOP_RETURN 1
#define SHUD_ODE_TOO_MUCH_WORK (-1)
#define SHUD_ODE_TOO_MUCH_ACC (-2)
#define SHUD_ODE_ERR_FAILURE (-3)
#define SHUD_ODE_CONV_FAILURE (-4)
#define SHUD_ODE_LSOLVE_FAIL (-7)
#define SHUD_ODE_RHSFUNC_FAIL (-8)
#define SHUD_ODE_FIRST_RHSFUNC_ERR (-9)
#define SHUD_ODE_MEM_FAIL (-20)
#define SHUD_ODE_MEM_NULL (-21)
#define SHUD_ODE_ILL_INPUT (-22)
#define SHUD_ODE_BAD_K (-24)
#define SHUD_ODE_BAD_T (-25)
#define SHUD_ODE_DEVICE_ERR (-100)   /* HIP error; message in shud_rhs_last_error_string() */

#define SHUD_ODE_NORMAL 1            /* CV_NORMAL   */
#define SHUD_ODE_ONE_STEP 2          /* CV_ONE_STEP */

typedef struct {
    double  reltol, abstol;          /* CS.reltol, CS.abstol                                       */
    double  init_step;               /* CS.InitStep (> 0; CVODE's own estimate is not provided)    */
    double  max_step;                /* CS.MaxStep; 0 = unbounded                                  */
    double  min_step;                /* 1e-6 in SetCVODE                                           */
    int64_t max_num_steps;           /* 1e6 in SetCVODE; <= 0 = CVODE default 500                  */
    int32_t maxl;                    /* SPGMR Krylov dimension; 0 = SUNDIALS default 5             */
    int32_t max_order;               /* BDF max order; 0 = 5                                       */
} ShudOdeOptions;

typedef struct {
    int64_t nst, nfe, nfe_ls, nni, ncfn, nnf, netf, nsetups, nli, ncfl, njtimes;
    int32_t qlast, qcur;
    double  hlast, hcur, tcur, hnext;
    int64_t n_sync;                  /* host<->device synchronisations (device integrator only)    */
} ShudOdeStats;

typedef struct shud_ode *shud_ode_t;

/* Generic RHS on device pointers, stream-ordered on the integrator's stream.  0 = ok, < 0 =
 * unrecoverable (CVRhsFn convention). */
typedef int (*ShudOdeRhsFn)(double t, const double *d_y, double *d_ydot, void *user);

/* Integrator over a SHUD RHS handle (serial or OMP semantics, unpartitioned, lakes allowed).  y0 is
 * NY = 3*NE + NR + NL values on the host (where = SHUD_WHERE_HOST) or the device.  Physics errors of the
 * RHS (the reference's exits 10/13) end the solve with SHUD_ODE_RHSFUNC_FAIL; shud_rhs_get_error gives
 * the reference message. */
int shud_ode_create(shud_rhs_t rhs, double t0, const double *y0, int where, const ShudOdeOptions *opt,
                    shud_ode_t *out);
/* Integrator over any device RHS (tests: published problems).  stream = hipStream_t the RHS uses. */
int shud_ode_create_fn(int64_t n, ShudOdeRhsFn f, void *user, void *stream, double t0, const double *y0,
                       int where, const ShudOdeOptions *opt, shud_ode_t *out);
int shud_ode_set_stop_time(shud_ode_t o, double tstop);
/* CVode(): advances to tout (NORMAL) or by one internal step (ONE_STEP); y_out (NY values, host or
 * device per `where`, may be NULL) receives y(*tret).  Returns a SHUD_ODE_* code. */
int shud_ode_solve(shud_ode_t o, double tout, double *y_out, int where, double *tret, int itask);
/* CVodeGetDky: k-th derivative of the interpolating polynomial at t (tcur - hlast <= t <= tcur). */
int shud_ode_get_dky(shud_ode_t o, double t, int k, double *dky, int where);
int shud_ode_get_stats(shud_ode_t o, ShudOdeStats *st);
/* device pointer of the current Nordsieck zn[0] (y at tcur), NY doubles; valid until the next solve; read-only
 * (the integrator keeps the next step's error weights, computed from this zn[0] at the end of the last step).
 * Complete on return: a deferred completion of zn[0] is applied and the integrator's stream is synchronized, so
 * any stream may read it (NULL on a device error). */
const double *shud_ode_state_device(shud_ode_t o);
int shud_ode_destroy(shud_ode_t o);

#ifdef __cplusplus
}
#endif
#endif /* SHUD_ODE_H */
