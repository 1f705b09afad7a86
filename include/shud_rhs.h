/*
 * shud_rhs.h — C-ABI of the MI355X-native SHUD right-hand-side (RHS) flux assembly.
 *
 * This is the drop-in boundary for ONE hot path of DankerMu/SHUD-up: the CVODE RHS callback
 *     int f(double t, N_Vector CV_Y, N_Vector CV_Ydot, void *DS)        (src/Model/f.hpp:12, f.cpp:2-32)
 * and the Model_Data state it reads and mutates (src/ModelData/Model_Data.hpp:111-208).
 * Everything here is plain C: pointers + sizes, no torch / HIP types in the signatures.
 *
 * Index conventions (all arrays are 0-based, SoA):
 *   y / ydot block layout is unchanged from the reference:  [sf(NE) | us(NE) | gw(NE) | riv(NR)]
 *   (src/Model/Macros.hpp:21-25 iSF/iUS/iGW/iRIV).  Lakes (iLAKE) are not supported.
 *   Per-edge element arrays are edge-major: a[j*NE + i] is edge j of element i (j = 0,1,2).
 *   nabr:  0-based neighbour element, or -1 on the domain boundary (file value 0, Element.hpp:25).
 *   riv_down: 0-based downstream reach, or an outlet code -1/-2/-3 (zero-depth gradient) or -4
 *            (critical depth) exactly as the reference's negative `down` (MD_RiverFlux.cpp:36-54).
 *   ibc / iss / riv_bc keep the reference's signed 1-based time-series column numbers.
 *
 * Thread-safety: single caller per handle (CVODE calls f from one host thread).
 */
#ifndef SHUD_RHS_H
#define SHUD_RHS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHUD_RHS_ABI_VERSION 2   /* 2: lakes (ShudMeshSoA/ShudStepInputs/ShudFluxOut tails) */

/* ---- return codes (CVODE convention: 0 ok, <0 unrecoverable, >0 recoverable) ---- */
#define SHUD_OK              0
#define SHUD_ERR_PHYSICS    -1   /* reference would have called myexit(); see ShudErr       */
#define SHUD_ERR_ARG        -2   /* invalid argument / inconsistent mesh                     */
#define SHUD_ERR_HIP        -3   /* HIP runtime failure                                       */
#define SHUD_ERR_NCCL       -4   /* RCCL failure (partitioned handles)                        */
#define SHUD_ERR_UNSUPPORTED -5  /* lake elements / lake reaches             */

/* ---- semantics selector ---- */
#define SHUD_MODE_SERIAL     0   /* f_update/f_loop/f_applyDY: MD_update.cpp:102-189, MD_f.cpp:9-257 */
#define SHUD_MODE_OMP        1   /* f_update_omp/f_loop_omp/f_applyDY_omp: MD_f_omp.cpp:9-170       */

/* ---- where y / ydot live for shud_rhs_eval ---- */
#define SHUD_WHERE_HOST      0   /* host pointers; eval is synchronous on return                    */
#define SHUD_WHERE_DEVICE    1   /* device pointers; eval is stream-ordered on the handle's stream  */

/* ---- error bits reported in ShudErr.flags (reference exit code in brackets) ---- */
#define SHUD_EF_NAN_QELE     0x01u  /* CheckNANij(QeleSurf/QeleSub) MD_f.cpp:73-74          [10] */
#define SHUD_EF_EFFKH        0x02u  /* effKH out of [0,1e9]        Equations.cpp:130-131      [13] */
#define SHUD_EF_ET_NEG       0x04u  /* CheckNonNegative(Es..Tg)    MD_ET.cpp:394-398          [10] */
#define SHUD_EF_ET_NAN       0x08u  /* CheckNANi(qEleETA..)        MD_ET.cpp:399-401          [10] */
#define SHUD_EF_AET_WARN     0x10u  /* printf warning AET > 2 PET   MD_ET.cpp:391-393 (not fatal)  */
/* ET-step prelude (include/shud_et.h, shud_et_step) */
#define SHUD_EF_ET_RA        0x20u  /* CheckNonZero(Aerodynamic Resistance) MD_ET.cpp:273     [10] */
#define SHUD_EF_ET_PT_NAN    0x40u  /* CheckNANi(qPotTran)          MD_ET.cpp:278              [10] */
/* partitioned handles */
#define SHUD_EF_HALO_WAIT    0x80u  /* boundary elements timed out waiting for the halo exchange (no reference analogue) */

/* Static mesh description (uploaded once by shud_rhs_create).  Mirrors the derived geometry the
 * reference holds after Model_Data::initialize() (MD_initialize.cpp:168-245). */
typedef struct ShudMeshSoA {
    int32_t num_ele, num_riv, num_seg;
    int32_t close_boundary;        /* CS.CloseBoundary (Model_Control.hpp:164), default 1         */
    /* elements */
    const int32_t *nabr;           /* [3*NE]                                                      */
    const double  *area;           /* [NE]  Triangle::area                                        */
    const double  *z_surf;         /* [NE]                                                        */
    const double  *z_bottom;       /* [NE]                                                        */
    const double  *depression;     /* [NE]  _Element::depression (Element.hpp:93)                 */
    const double  *edge;           /* [3*NE]                                                      */
    const double  *dist2nabor;     /* [3*NE] _Element::Dist2Nabor (Element.cpp:249-265)           */
    const double  *dist2edge;      /* [3*NE] read only when close_boundary == 0                   */
    const double  *avg_rough;      /* [3*NE]                                                      */
    const double  *rough;          /* [NE]  Landcover::Rough, read only when close_boundary == 0  */
    const int32_t *ibc;            /* [NE]  AttriuteIndex::iBC                                    */
    const int32_t *iss;            /* [NE]  AttriuteIndex::iSS                                    */
    const int32_t *ilake;          /* [NE]  AttriuteIndex::iLake (> 0: lake element), may be NULL */
    /* river reaches (_River, River.hpp:47-93) */
    const int32_t *riv_down;       /* [NR]                                                        */
    const int32_t *riv_bc;         /* [NR]  _River::BC                                            */
    const double  *riv_length;     /* [NR]                                                        */
    const double  *riv_bed_slope;  /* [NR]                                                        */
    const double  *riv_dist2down;  /* [NR]  Dist2DownStream (River.cpp:74-84)                    */
    const double  *riv_avg_rough;  /* [NR]  avgRough                                              */
    const double  *riv_depth;      /* [NR]                                                        */
    const double  *riv_bottom_width; /* [NR]                                                      */
    const double  *riv_bankslope;  /* [NR]                                                        */
    const double  *riv_ksath;      /* [NR]                                                        */
    const double  *riv_bedthick;   /* [NR]                                                        */
    /* river segments (RiverSegement, River.hpp:95-104), reference order */
    const int32_t *seg_ele;        /* [NS]  0-based element                                       */
    const int32_t *seg_riv;        /* [NS]  0-based reach                                         */
    const double  *seg_length;     /* [NS]                                                        */
    const double  *seg_cwr;        /* [NS]                                                        */
    /* lakes (MD_Lake.cpp, Lake.hpp/.cpp).  Lakes are on when any ilake > 0 (MD_readin.cpp:
     * 262-263); lake ids are 1..num_lake; a reach with riv_down <= -4 then flows into lake (-3 - down)
     * (MD_Lake.cpp:46-50) instead of the critical-depth outlet.  The y/ydot vectors gain num_lake stages
     * after the reaches ([sf|us|gw|riv|lake], Macros.hpp:21-25).  Serial semantics; partitioned handles take
     * the local mesh of shud_plan_local_mesh (owned lakes only, include/shud_partition.h). */
    int32_t num_lake;
    const int32_t *lake_bathy_off; /* [num_lake+1] row offsets of each lake's bathymetry table       */
    const double  *lake_bathy_y;   /* LakeBathymetry::yi (stage datum; zmin = yi[0]), lake_readBathy */
    const double  *lake_bathy_a;   /* LakeBathymetry::ai (top area)                                 */
} ShudMeshSoA;

/* Per-element hydraulic parameters after calibration and init (Soil_Layer / Geol_Layer /
 * Landcover copies in _Element, ModelConfigure.hpp:53-104, MD_initialize.cpp:176-186). */
typedef struct ShudParamsSoA {
    const double *aquifer_depth, *macD, *macKsatH, *geo_vAreaF, *KsatH, *KsatV;
    const double *infKsatV, *hAreaF, *macKsatV, *ThetaS, *ThetaR, *Beta, *infD;
    const double *Sy, *RzD, *VegFrac, *ImpAF;
} ShudParamsSoA;

/* Per-ET-step inputs (produced by updateforcing()/ET(), MD_ET.cpp:14-342).  Any pointer may be
 * NULL to keep the previous value.  e_ic and u_satn are also CARRIED state: the serial RHS
 * mutates qEleE_IC (MD_ET.cpp:370,381) and reads the previous call's u_satn (MD_f.cpp:19 vs :22). */
typedef struct ShudStepInputs {
    const double *net_prep;   /* qEleNetPrep [NE] */
    const double *pot_evap;   /* qPotEvap    [NE] */
    const double *pot_tran;   /* qPotTran    [NE] */
    const double *etp;        /* qEleETP     [NE] (only the AET>2PET warning reads it) */
    const double *lai;        /* t_lai       [NE] */
    const double *fu_surf;    /* fu_Surf     [NE] */
    const double *fu_sub;     /* fu_Sub      [NE] */
    const double *e_ic;       /* qEleE_IC    [NE] carried in/out */
    const double *u_satn;     /* Ele[i].u_satn [NE] carried in/out */
    const double *ugw_stale;  /* uYgw for iBC<0 elements: f_update never refreshes it
                                 (MD_update.cpp:123-125); [NE], default 0 */
    /* boundary-condition time-series rows at the current ET step (TimeSeriesData::getX ignores t,
       TimeSeriesData.cpp:270-273): value of column c is x[c], c = 1..ncol (x[0] unused). */
    const double *ele_ybc; int32_t n_ele_ybc;   /* tsd_eyBC, indexed by  iBC  (iBC > 0) */
    const double *ele_qbc; int32_t n_ele_qbc;   /* tsd_eqBC, indexed by -iBC  (iBC < 0) */
    const double *riv_ybc; int32_t n_riv_ybc;   /* tsd_ryBC, indexed by  BC   (BC > 0)  */
    const double *riv_qbc; int32_t n_riv_qbc;   /* tsd_rqBC, indexed by -BC   (BC < 0)  */
    const double *prcp;       /* qElePrep [NE]: precipitation of lake elements (MD_f.cpp:17)    */
} ShudStepInputs;

typedef struct ShudRhsOptions {
    int32_t mode;         /* SHUD_MODE_SERIAL | SHUD_MODE_OMP                                  */
    int32_t device;       /* HIP device ordinal                                                 */
    void   *stream;       /* hipStream_t to launch on; NULL = handle-owned non-blocking stream  */
    int32_t check_errors; /* 1 = read the device error word after every host-pointer eval      */
} ShudRhsOptions;

/* Fluxes the reference leaves in Model_Data after f() (read by ExportResults/WaterBalanceDiag).
 * Any pointer may be NULL.  Filled lazily by shud_rhs_sync_diagnostics (re-evaluates the last
 * call from its saved inputs, so the carried state is not advanced twice). */
typedef struct ShudFluxOut {
    double *qele_surf;   /* QeleSurf [3*NE] edge-major */
    double *qele_sub;    /* QeleSub  [3*NE] */
    double *qele_surf_tot, *qele_sub_tot;            /* [NE] */
    double *q_infil, *q_exfil, *q_recharge;          /* qEleInfil/Exfil/Recharge [NE] */
    double *q_es, *q_eu, *q_eg, *q_tu, *q_tg;        /* [NE] ET components (serial mode) */
    double *q_eta;                                   /* qEleETA [NE] */
    double *e_ic, *u_satn, *i_beta, *eff_kh;         /* carried / scratch [NE] */
    double *qe2r_surf, *qe2r_sub;                    /* [NE] */
    double *qseg_surf, *qseg_sub;                    /* [NS] reference segment order */
    double *qriv_down, *qriv_up, *qriv_surf, *qriv_sub; /* [NR] */
    double *q_lake_surf, *q_lake_sub, *q_lake_rivin; /* QLakeSurf/QLakeSub/QLakeRivIn [num_lake]       */
    double *q_lake_evap, *q_lake_prcp, *lake_toparea; /* qLakeEvap/qLakePrcp, y2LakeArea [num_lake]   */
} ShudFluxOut;

typedef struct ShudErr {
    uint32_t flags;       /* OR of SHUD_EF_* seen since the last clear                          */
    int32_t  exit_code;   /* code the reference's myexit() would have used, 0 if none          */
    int32_t  first_index[8]; /* per bit (log2 of flag): lowest element index (0-based), -1 none */
    int64_t  n_aet_warn;  /* number of AET>2PET warnings                                        */
    char     message[256];
} ShudErr;

typedef struct shud_rhs *shud_rhs_t;

/* ---- single-device API ---- */
int  shud_rhs_abi_version(void);
int  shud_rhs_create(const ShudMeshSoA *mesh, const ShudParamsSoA *par,
                     const ShudRhsOptions *opt, shud_rhs_t *out);
int  shud_rhs_set_step_inputs(shud_rhs_t h, const ShudStepInputs *in);
/* One RHS evaluation = reference f(): f_update -> f_loop -> f_applyDY, nFCall++ (f.cpp:2-32). */
int  shud_rhs_eval(shud_rhs_t h, double t, const double *y, double *ydot, int where);
int  shud_rhs_sync_diagnostics(shud_rhs_t h, ShudFluxOut *out);
int  shud_rhs_get_error(shud_rhs_t h, ShudErr *err);
int  shud_rhs_clear_error(shud_rhs_t h);
long long shud_rhs_num_calls(shud_rhs_t h);  /* Model_Data::nFCall */
/* device layout chosen at create: *packed = 1 when per-element parameters were folded into
 * *n_classes distinct parameter tuples (the fast element kernel); 0 = plain SoA kernel */
int  shud_rhs_layout(shud_rhs_t h, int *packed, int *n_classes);
/* hybrid layout of a packed handle: *n_streamed class fields (of KsatH, macD, macKsatH, vAreaF, KsatV, Sy, RzD,
 * depression, Rough) are streamed per element because the full parameter tuples exceed one workgroup's LDS class
 * table (per-element-calibrated models); 0 = every field from the class table */
int  shud_rhs_layout_streamed(shud_rhs_t h, int *n_streamed);
/* in-tile edge sharing of a packed handle: *n_shared interior edges are evaluated once and read by the other element
 * of the edge (exactly antisymmetric pairs within one 256-element tile, single-GPU handles; SHUD_RHS_SHARE=0: off) */
int  shud_rhs_layout_shared(shud_rhs_t h, int *n_shared);
int  shud_rhs_destroy(shud_rhs_t h);
const char *shud_rhs_last_error_string(void);

/* CVRhsFn body with raw arrays: a SUNDIALS build registers
 *   int shud_f(double t, N_Vector y, N_Vector yd, void *ud)
 *   { return shud_rhs_cvrhs(t, N_VGetArrayPointer(y), N_VGetArrayPointer(yd), ud); }
 * with user_data = shud_rhs_t.  Returns 0, or -1 after a physics error
 * (exits with the reference code when SHUD_RHS_STRICT_EXIT=1). */
int  shud_rhs_cvrhs(double t, const double *y, double *ydot, void *user_data);

/* ---- measurement helpers (bench / profiling only) ---- */
/* Device-resident scratch for y/ydot of this handle (for device-pointer evals). */
int  shud_rhs_device_alloc(shud_rhs_t h, size_t bytes, void **dptr);
int  shud_rhs_device_free(shud_rhs_t h, void *dptr);
int  shud_rhs_memcpy(shud_rhs_t h, void *dst, const void *src, size_t bytes, int kind /*1 H2D,2 D2H,3 D2D*/);
int  shud_rhs_synchronize(shud_rhs_t h);
void *shud_rhs_stream(shud_rhs_t h);
/* Time `reps` device evals with HIP events on the handle's stream; per kernel average ms in
 * ms_out[k] for k < *nk (order: element kernel, river kernel, pack, exchange, ...), names in
 * names_out (comma separated).  Returns wall ms per eval in *ms_eval. */
int  shud_rhs_time_kernels(shud_rhs_t h, double t, const double *d_y, double *d_ydot, int reps,
                           double *ms_eval, double *ms_out, int *nk, char *names_out, int names_len);
/* In-loop timing of ordinary evals: while enabled, every `stride`-th eval (up to `max_evals` of them)
 * records HIP events on the handle's stream before its first launch, after its element kernel(s) and
 * after its river (+lake) kernel (an event between two kernels keeps them from overlapping, so sampling
 * keeps the timed loop's throughput intact).  _read returns the per-eval averages (ms) and disables it.
 * For a partitioned handle the element interval includes the pack kernel and any halo-exchange wait. */
int  shud_rhs_timing(shud_rhs_t h, int max_evals, int stride);
int  shud_rhs_timing_read(shud_rhs_t h, double *ms_ele, double *ms_riv, double *ms_eval, int *n_evals);

/* ---- partitioned (one process per GPU, RCCL halo) API, SURVEY §8e ----
 * Local numbering: elements [owned | seg-ghost | ghost], reaches [owned | ghost]; segments are
 * every segment whose element or reach is local-owned, in global segment order.  Owned y/ydot of a
 * rank use the reference block layout over its owned entities: [sf(NEo)|us(NEo)|gw(NEo)|riv(NRo)].
 * Ghost y values arrive by one RCCL all-to-all-v per eval. */
typedef struct ShudPartition {
    int32_t rank, nranks;
    int32_t n_own_ele, n_segghost_ele;   /* the mesh passed to create has num_ele = all local */
    int32_t n_own_riv;                   /* num_riv = owned + ghost reaches                 */
    /* element ghosts: for peer p, ghost elements [ele_recv_off[p], ele_recv_off[p+1]) (offsets
       relative to n_own_ele) are filled from owned element indices ele_send_idx[ele_send_off[p]..) of p */
    const int32_t *ele_send_off;   /* [nranks+1] */
    const int32_t *ele_send_idx;   /* local owned indices to send */
    const int32_t *ele_recv_off;   /* [nranks+1] */
    const int32_t *riv_send_off;   /* [nranks+1] */
    const int32_t *riv_send_idx;
    const int32_t *riv_recv_off;   /* [nranks+1], relative to n_own_riv */
    const int32_t *ele_gid;        /* [num_ele] global element id of each local element          */
    const int32_t *riv_gid;        /* [num_riv] global reach id (orders junction sums globally)  */
    const char    *nccl_unique_id; /* 128 bytes from shud_rhs_nccl_unique_id on rank 0, or NULL
                                      for external transport (shud_rhs_eval_pack/_compute)      */
} ShudPartition;

/* external-transport hooks of a partitioned handle (tests; RCCL handles do this internally) */
int  shud_rhs_halo_buffers(shud_rhs_t h, double **ele_send, double **riv_send, double **ele_ghost,
                           double **riv_ghost);
int  shud_rhs_eval_pack(shud_rhs_t h, const double *d_y);
int  shud_rhs_eval_compute(shud_rhs_t h, double t, const double *d_y, double *d_ydot);
/* Test hook (no reference analogue; tests/test_gpu_partition.py): on every following device eval of a
 * partitioned handle the comm stream, after its pack (and RCCL exchange), spins spin_us microseconds, then copies
 * the ghost states from d_ele_src (3 x #ghost elements, recv order) / d_riv_src (#ghost reaches) into the ghost
 * buffers with a kernel (NULL: no copy), then publishes the halo flag unless publish == 0 (the folded launch's
 * boundary workgroups then time out: SHUD_EF_HALO_WAIT).  timeout_ms > 0 sets their poll bound (else
 * SHUD_HALO_TIMEOUT_MS or 5000).  spin_us 0, NULL sources and publish 1 disarm the hook. */
int  shud_rhs_debug_halo(shud_rhs_t h, double spin_us, const double *d_ele_src, const double *d_riv_src,
                         int publish, double timeout_ms);

int  shud_rhs_nccl_unique_id(char out[128]);
int  shud_rhs_create_partitioned(const ShudMeshSoA *mesh, const ShudParamsSoA *par,
                                 const ShudRhsOptions *opt, const ShudPartition *part,
                                 shud_rhs_t *out);

#ifdef __cplusplus
}
#endif
#endif /* SHUD_RHS_H */
