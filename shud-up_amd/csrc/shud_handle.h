// shud_handle.h — internal: the shud_rhs handle shared by the host runtime translation units
// (shud_rhs.cpp: RHS; shud_et.cpp: ET-step prelude).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <vector>

#include "shud_dev.h"
#include "shud_rhs.h"

// records the message for shud_rhs_last_error_string() and returns code
int shud_fail(int code, const char *fmt, ...);


#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return shud_fail(SHUD_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                               \
    } while (0)
#define NCCL_TRY(expr)                                                                      \
    do {                                                                                    \
        ncclResult_t r_ = (expr);                                                           \
        if (r_ != ncclSuccess)                                                              \
            return shud_fail(SHUD_ERR_NCCL, "%s failed: %s", #expr, ncclGetErrorString(r_));     \
    } while (0)


using namespace shud;
struct EtState;                           // shud_et.cpp

struct shud_rhs {
    int NE = 0, NR = 0, NS = 0;          // local totals (incl. ghosts)
    int n_own = 0, n_segghost = 0, n_own_riv = 0;
    bool lakeon = false;                 // lakes: any iLake > 0; serial, packed
    int NL = 0;
    DevLake lk{};
    int n_int = 0;                       // partitioned: owned prefix independent of ghost data
    int mode = SHUD_MODE_SERIAL;
    bool open = false;
    bool check_errors = true;
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::vector<void *> allocs;

    DevMesh dm{};
    DevDiag dd{};
    bool have_diag = false;
    int cur = 0, cur_e = 0;
    long long ncalls = 0;
    bool packed = false;                 // class-table / 16-byte-record layout in use (DevPacked)
    DevPacked dp{};
    int n_classes = 0;
    int n_shared = 0;       // interior edges evaluated once (in-tile edge sharing, build_packed)
    bool fu_unit[2] = {true, true};      // fu_Surf / fu_Sub are all 1.0 (cryosphere off): not read
    bool qd_now = false;                 // this eval's element launch wrote DevPacked::qdown (river kernel reads it)

    // host-pointer eval staging
    double *d_y = nullptr, *d_ydot = nullptr, *d_scratch_dy = nullptr;
    // replay info of the last eval
    bool have_last = false;
    const double *last_y = nullptr;
    int last_cur = 0, last_cur_e = 0;

    std::vector<int> seg_perm;           // element-sorted position -> reference segment index
    int max_col[4] = {0, 0, 0, 0};       // highest BC column referenced: eyBC, eqBC, ryBC, rqBC
    double *d_tab[4] = {nullptr, nullptr, nullptr, nullptr};
    int tab_len[4] = {0, 0, 0, 0};

    EtState *et = nullptr;               // ET-step prelude (shud_et_attach), owned
    // output path (shud_out.h): Model_Data::summary arrays and the derived ET sums, allocated on first use
    double *d_sum[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};   // yEleSurf/Unsat/GW, yRivStg, yLakeStg
    double *d_trans = nullptr, *d_evapo = nullptr;                      // qEleTrans, qEleEvapo
    double *d_zero_lake = nullptr;                                      // QLakeRivOut (always 0)

    DevErr *d_err = nullptr;
    DevErr *h_err = nullptr;             // pinned
    unsigned long long *d_warn = nullptr;   // DevErr::warn slots
    unsigned long long *h_warn = nullptr;   // pinned

    // partition / halo
    bool partitioned = false;
    int rank = 0, nranks = 1;
    bool use_nccl = false;
    ncclComm_t comm = nullptr;
    hipStream_t s_comm = nullptr;        // RCCL halo exchange, overlapped with the interior element kernel
    hipEvent_t ev_pack = nullptr, ev_comm = nullptr;
    // boundary + ghost elements folded into the interior launch (launch_element_kernel_packed_fold): the comm stream
    // publishes halo_epoch into d_halo_flag after the exchange; SHUD_RHS_FOLD=0 keeps two launches (A/B)
    bool fold = false;
    bool fold_join = false;              // main stream joins ev_comm after the folded eval (SHUD_RHS_FOLD_JOIN=1)
    unsigned long long *d_halo_flag = nullptr, halo_epoch = 0;
    unsigned long long halo_timeout = 0; // poll bound in wall_clock64 ticks (SHUD_HALO_TIMEOUT_MS, default 5000)
    double wall_khz = 100000.0;          // hipDeviceAttributeWallClockRate
    long long n_exch = 0;                // exchanges enqueued (an RCCL handle's first one takes the split path)
    // test hook (shud_rhs_debug_halo): a late or missing halo on the comm stream
    bool dbg_armed = false, dbg_publish = true;
    unsigned long long dbg_spin = 0;
    const double *dbg_gele = nullptr, *dbg_griv = nullptr;
    // in-loop kernel timing (shud_rhs_timing): 3 events per device eval {start, after element kernel(s),
    // after river (+lake) kernel}, recorded on the handle's stream while enabled
    int tm_cap = 0, tm_n = 0, tm_stride = 1;
    long long tm_seen = 0;
    std::vector<hipEvent_t> tm_ev;
    std::vector<int> esend_off, erecv_off, rsend_off, rrecv_off;
    int *d_esend_idx = nullptr, *d_rsend_idx = nullptr;
    int n_esend = 0, n_rsend = 0, n_eghost = 0, n_rghost = 0;
    double *d_esend = nullptr, *d_rsend = nullptr, *d_gele = nullptr, *d_griv = nullptr;

    template <class T>
    int dalloc(T **p, size_t n) {
        void *q = nullptr;
        size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
        hipError_t e = hipMalloc(&q, bytes);
        if (e != hipSuccess) return shud_fail(SHUD_ERR_HIP, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
        allocs.push_back(q);
        *p = (T *)q;
        return 0;
    }
    template <class T>
    int upload(T **p, const T *src, size_t n) {
        int rc = dalloc(p, n);
        if (rc) return rc;
        if (n && src) HIP_TRY(hipMemcpy(*p, src, n * sizeof(T), hipMemcpyHostToDevice));
        else if (n) HIP_TRY(hipMemset(*p, 0, n * sizeof(T)));
        return 0;
    }
    template <class T>
    int upload_fill(T **p, const T *src, size_t n, T fill) {
        if (src) return upload(p, src, n);
        std::vector<T> tmp(n, fill);
        return upload(p, tmp.data(), n);
    }
};

int shud_reset_err(shud_rhs *h);
int shud_read_err(shud_rhs *h);          // h_err = the device error word (warning slots summed); synchronises
int shud_diag_replay(shud_rhs *h);       // shud_rhs.cpp: last eval again with diagnostic stores (device only)
int shud_ensure_diag(shud_rhs *h);       // shud_rhs.cpp: allocate the DevDiag arrays (zeros) once
void shud_et_free(shud_rhs *h);          // shud_et.cpp
const double *shud_et_array(shud_rhs *h, int which);   // shud_et.cpp: SHUD_ARR_Y_ELE_IS.. (NULL if not attached)
