// shud_out.hip — output path on the device (include/shud_out.h).
//
// The reference keeps one host buffer per Print_Ctrl and, at every solver step, adds each selected
// Model_Data value into it (Print_Ctrl::PrintData, src/classes/Model_Control.cpp:926-960); the mean over the
// interval goes to a binary .dat (fun_printBINARY :893-899) and/or ASCII .csv (:900-909) file.  Here the values
// already live in HBM, so the buffers do too: every export adds all registered variables with ONE batched
// kernel (blockIdx.y = control; a control's selected columns are a device index list when flag_IO masks some),
// and only the controls whose interval ends scale their buffer on the device (buffer *= tau / NumUpdate, the
// reference's expression) and come back over PCIe to be written with the reference's byte layout.
//
// Finished intervals leave the compute stream at once: one kernel per control writes the scaled mean into a
// snapshot buffer and zeroes the accumulator; the snapshot goes device->host on a copy stream into one of two
// pinned banks, and writer threads (controls dealt round-robin, so each file keeps one writer and its row order)
// append the rows once that copy's event has fired.  The time loop only waits when both banks are still being
// written (the reference writes synchronously inside ExportResults; the bytes written are the same, in the
// same order).
#include <hip/hip_runtime.h>

#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "shud_handle.h"
#include "shud_out.h"

namespace {

struct PrintSlot {                       // one Print_Ctrl on the device (POD, copied to a device table)
    const double *src;
    const int *sel;                      // selected column -> source index; nullptr = identity
    double *buf;
    int nvar;
};

__global__ void __launch_bounds__(256) k_accumulate(const PrintSlot *__restrict__ slots) {
    const PrintSlot s = slots[blockIdx.y];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < s.nvar; i += gridDim.x * blockDim.x)
        s.buf[i] += s.src[s.sel ? s.sel[i] : i];                 // buffer[i] += *(PrintVar[i])
}

// buffer[i] *= tau / NumUpdate (the reference's expression, into the snapshot), then buffer[i] = 0
__global__ void __launch_bounds__(256) k_snap(double *__restrict__ buf, double *__restrict__ snap, int n, double f) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        snap[i] = buf[i] * f;
        buf[i] = 0.0;
    }
}

// Model_Data::summary (MD_update.cpp:190-216): element storages and river stage from a state vector, BC
// values where the element / reach has a head boundary condition
__global__ void __launch_bounds__(256) k_summary(DevMesh m, const double *__restrict__ y, int ne, int nr, int nl,
                                                 double *ysf, double *yus, double *ygw, double *yriv, double *ylake) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < ne) {
        ysf[i] = y[i];
        yus[i] = y[ne + i];
        const int ibc = (int)(int16_t)(m.eflags[i] & 0xffff);
        ygw[i] = ibc > 0 ? m.eybc[ibc] : y[2 * ne + i];
    }
    if (i < nr) {
        const int bc = m.riv_bc[i];
        yriv[i] = bc > 0 ? m.rybc[bc] : y[3 * ne + i];
    }
    if (i < nl) ylake[i] = y[3 * ne + nr + i];                   // yLakeStg = Y[iLAKE] (MD_update.cpp:175)
}

// qEleTrans = Tg + Tu, qEleEvapo = Eu + Eg + Es (MD_ET.cpp:388-389), from the replayed diagnostics
__global__ void __launch_bounds__(256) k_et_sums(DevDiag d, int ne, double *trans, double *evapo) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ne) return;
    trans[i] = d.q_tg[i] + d.q_tu[i];
    evapo[i] = d.q_eu[i] + d.q_eg[i] + d.q_es[i];
}

}  // namespace

struct PrintCtrl {
    std::string filename;
    long long start_time = 0;
    int interval = 0, numvar = 0, numall = 0, num_update = 0;
    double tau = 1.0;
    std::vector<double> icol;
    int *d_sel = nullptr;
    double *d_buf = nullptr;
    double *d_snap = nullptr;            // the finished interval's mean, on its way to the host
    double *h_buf[2] = {nullptr, nullptr};   // pinned banks for the interval mean
    FILE *fb = nullptr, *fa = nullptr;
    int64_t rows = 0;
};

struct OutTask {                         // one row of one control: (bank, control, left endpoint of the interval)
    int bank, ctrl;
    double tq;
};
constexpr int kWriters = 4;

struct shud_out {
    int device = 0;
    hipStream_t stream = nullptr;        // compute stream (accumulate / snapshot kernels)
    hipStream_t s_copy = nullptr;        // device->host copies of the snapshots
    hipEvent_t ev_snap = nullptr, ev_copied[2] = {nullptr, nullptr};
    bool copy_pending = false;           // a snapshot copy is in flight (the next snapshot waits for it)
    int bank = 0;
    std::vector<PrintCtrl> pc;
    std::vector<PrintSlot> slots;        // host mirror of d_slots, index-aligned with pc
    PrintSlot *d_slots = nullptr;
    int n_slots_alloc = 0;
    int max_nvar = 0;
    // writer threads: writer w owns the controls k with k % kWriters == w
    std::thread writer[kWriters];
    std::mutex mu;
    std::condition_variable cv;
    std::deque<OutTask> tasks[kWriters];
    int bank_left[2] = {0, 0};           // rows of the bank's event not yet written
    bool stop = false;
    // first writer-side failure (the snapshot copy's event or a file write): reported by shud_out_flush /
    // shud_out_rows / shud_out_destroy; rows whose copy failed are never written (no stale bank reaches a file)
    int werr = 0;
    std::string werr_msg;
};
static void writer_fail(shud_out *o, int code, const std::string &msg) {
    std::lock_guard<std::mutex> lk(o->mu);
    if (!o->werr) { o->werr = code; o->werr_msg = msg; }
}

static void writer_loop(shud_out *o, int w) {
    (void)hipSetDevice(o->device);
    for (;;) {
        OutTask job;
        {
            std::unique_lock<std::mutex> lk(o->mu);
            o->cv.wait(lk, [&] { return o->stop || !o->tasks[w].empty(); });
            if (o->tasks[w].empty()) return;
            job = o->tasks[w].front();
            o->tasks[w].pop_front();
        }
        const hipError_t he = hipEventSynchronize(o->ev_copied[job.bank]);
        PrintCtrl &p = o->pc[job.ctrl];
        const double *hb = p.h_buf[job.bank];
        if (he != hipSuccess) {
            writer_fail(o, SHUD_ERR_HIP, std::string("output snapshot copy failed (") + hipGetErrorString(he) +
                                             "): row of " + p.filename + " not written");
        } else {
            if (p.fa) {                                              // fun_printASCII
                fprintf(p.fa, "%.1f\t", job.tq);
                for (int i = 0; i < p.numvar; i++) fprintf(p.fa, "%e\t", hb[i]);
                fprintf(p.fa, "\n");
                if (ferror(p.fa)) writer_fail(o, SHUD_ERR_ARG, "write error on " + p.filename + ".csv");
            }
            if (p.fb) {                                              // fun_printBINARY
                const size_t w1 = fwrite(&job.tq, sizeof(double), 1, p.fb);
                const size_t w2 = fwrite(hb, sizeof(double), p.numvar, p.fb);
                if (w1 != 1 || w2 != (size_t)p.numvar) writer_fail(o, SHUD_ERR_ARG, "write error on " + p.filename + ".dat");
            }
        }
        {
            std::lock_guard<std::mutex> lk(o->mu);
            o->bank_left[job.bank]--;
        }
        o->cv.notify_all();
    }
}

// wait until every queued row is in the files (flushed to the C library); returns the first writer failure
static int out_drain(shud_out *o) {
    std::unique_lock<std::mutex> lk(o->mu);
    o->cv.wait(lk, [&] { return o->bank_left[0] == 0 && o->bank_left[1] == 0; });
    for (PrintCtrl &p : o->pc) {
        if (p.fb && fflush(p.fb) != 0 && !o->werr) { o->werr = SHUD_ERR_ARG; o->werr_msg = "flush error on " + p.filename + ".dat"; }
        if (p.fa && fflush(p.fa) != 0 && !o->werr) { o->werr = SHUD_ERR_ARG; o->werr_msg = "flush error on " + p.filename + ".csv"; }
    }
    return o->werr;
}
static int out_report(shud_out *o) {
    return o->werr ? shud_fail(o->werr, "shud_out: %s", o->werr_msg.c_str()) : SHUD_OK;
}

static int out_fail_io(const char *what, const std::string &f) {
    return shud_fail(SHUD_ERR_ARG, "%s: cannot open %s", what, f.c_str());
}

extern "C" int shud_out_create(int device, void *stream, shud_out_t *out) {
    if (!out) return shud_fail(SHUD_ERR_ARG, "null argument");
    *out = nullptr;
    HIP_TRY(hipSetDevice(device));
    shud_out *o = new shud_out;
    o->device = device;
    o->stream = (hipStream_t)stream;
    HIP_TRY(hipStreamCreateWithFlags(&o->s_copy, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&o->ev_snap, hipEventDisableTiming));
    for (int b = 0; b < 2; b++) HIP_TRY(hipEventCreateWithFlags(&o->ev_copied[b], hipEventDisableTiming));
    for (int w = 0; w < kWriters; w++) o->writer[w] = std::thread(writer_loop, o, w);
    *out = o;
    return SHUD_OK;
}

// Print_Ctrl::Init / InitIJ (Model_Control.cpp:759-858) + open_file (:683-758)
extern "C" int shud_out_add(shud_out_t o, const ShudPrintSpec *s) {
    if (!o || !s || !s->basename || !s->d_src) return shud_fail(SHUD_ERR_ARG, "null argument");
    if (s->interval == 0) return shud_fail(SHUD_ERR_ARG, "Print_Ctrl %s: interval 0 (reference: myexit(ERRCONSIS))",
                                           s->basename);
    if (s->n_all < 0 || s->interval < 0) return shud_fail(SHUD_ERR_ARG, "bad n_all / interval");
    HIP_TRY(hipSetDevice(o->device));
    if (out_drain(o)) return out_report(o);   // the writer indexes pc: no rows in flight while it grows
    PrintCtrl p;
    p.filename = s->basename;
    p.start_time = (long long)s->start_time;
    p.interval = s->interval;
    p.numall = s->n_all;
    p.tau = s->iflux ? 1440. : 1.;
    std::vector<int> sel;
    for (int i = 0; i < s->n_all; i++) {
        if (s->flag_io && !s->flag_io[i]) continue;
        sel.push_back(i);
        p.icol.push_back((double)(i + 1));                       // icol[k] = (double)(i + 1)
    }
    p.numvar = (int)sel.size();
    if (p.numvar <= 0) fprintf(stderr, "WARNING: Empty columns in %s.\n;", p.filename.c_str());
    const size_t nb = std::max(p.numvar, 1);
    HIP_TRY(hipMalloc(&p.d_buf, nb * sizeof(double)));
    HIP_TRY(hipMalloc(&p.d_snap, nb * sizeof(double)));
    HIP_TRY(hipMemsetAsync(p.d_buf, 0, nb * sizeof(double), o->stream));   // buffer[k] = 0.0
    for (int b = 0; b < 2; b++) HIP_TRY(hipHostMalloc(&p.h_buf[b], nb * sizeof(double), hipHostMallocDefault));
    if (s->flag_io && p.numvar < s->n_all) {
        HIP_TRY(hipMalloc(&p.d_sel, nb * sizeof(int)));
        HIP_TRY(hipMemcpy(p.d_sel, sel.data(), sel.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    // open_file: fixed 1024-byte header, StartTime, NumVar, icol (binary); the ASCII twin's preamble
    char header[1024];
    memset(header, 0, sizeof(header));
    const char *mode = s->solar_lonlat_mode ? s->solar_lonlat_mode : "";
    snprintf(header, sizeof(header),
             "# SHUD output\n"
             "# Radiation input mode: %s\n"
             "# Terrain radiation (TSR): %s\n"
             "# Solar lon/lat mode: %s\n"
             "# Solar lon/lat (deg): lon=%.6f, lat=%.6f\n",
             s->radiation_input_mode == 1 ? "SWNET" : "SWDOWN", s->terrain_radiation ? "ON" : "OFF", mode,
             s->solar_lon_deg, s->solar_lat_deg);
    if (s->binary) {
        const std::string fb = p.filename + ".dat";
        p.fb = fopen(fb.c_str(), "wb");
        if (!p.fb) return out_fail_io("shud_out_add", fb);
        fwrite(header, sizeof(char), 1024, p.fb);
        double tmp = (double)p.start_time;
        fwrite(&tmp, sizeof(tmp), 1, p.fb);
        tmp = (double)p.numvar;
        fwrite(&tmp, sizeof(tmp), 1, p.fb);
        fwrite(p.icol.data(), sizeof(double), p.icol.size(), p.fb);
    }
    if (s->ascii) {
        const std::string fa = p.filename + ".csv";
        p.fa = fopen(fa.c_str(), "w");
        if (!p.fa) return out_fail_io("shud_out_add", fa);
        fprintf(p.fa, "# Timestamp semantics: left endpoint (t-Interval)\n");
        fprintf(p.fa, "%d\t %d\t %ld\n", 0, p.numvar, (long)p.start_time);
        fprintf(p.fa, "# Radiation input mode: %s\n", s->radiation_input_mode == 1 ? "SWNET" : "SWDOWN");
        fprintf(p.fa, "# Terrain radiation (TSR): %s\n", s->terrain_radiation ? "ON" : "OFF");
        fprintf(p.fa, "# Solar lon/lat mode: %s\n", mode);
        fprintf(p.fa, "# Solar lon/lat (deg): lon=%.6f, lat=%.6f\n", s->solar_lon_deg, s->solar_lat_deg);
        fprintf(p.fa, "%s", "Time_min");
        for (int i = 0; i < p.numvar; i++) fprintf(p.fa, " \tX%d", i + 1);
        fprintf(p.fa, "\n");
    }
    o->max_nvar = std::max(o->max_nvar, p.numvar);
    o->slots.push_back(PrintSlot{s->d_src, p.d_sel, p.d_buf, p.numvar});
    o->pc.push_back(p);
    // the device slot table (tiny): re-uploaded whole on every add
    if ((int)o->slots.size() > o->n_slots_alloc) {
        if (o->d_slots) HIP_TRY(hipFree(o->d_slots));
        o->n_slots_alloc = std::max(16, 2 * (int)o->slots.size());
        HIP_TRY(hipMalloc(&o->d_slots, o->n_slots_alloc * sizeof(PrintSlot)));
    }
    HIP_TRY(hipMemcpyAsync(o->d_slots, o->slots.data(), o->slots.size() * sizeof(PrintSlot), hipMemcpyHostToDevice,
                           o->stream));
    HIP_TRY(hipStreamSynchronize(o->stream));
    return SHUD_OK;
}

// Control_Data::ExportResults (Model_Control.cpp:123-127) -> Print_Ctrl::PrintData (:926-960) for every control
extern "C" int shud_out_export(shud_out_t o, double t) {
    if (!o) return shud_fail(SHUD_ERR_ARG, "null argument");
    if (o->pc.empty()) return SHUD_OK;
    HIP_TRY(hipSetDevice(o->device));
    if (o->max_nvar > 0) {
        const int gx = std::min((o->max_nvar + 255) / 256, 2048);
        hipLaunchKernelGGL(k_accumulate, dim3(gx, (unsigned)o->pc.size()), dim3(256), 0, o->stream, o->d_slots);
        HIP_TRY(hipGetLastError());
    }
    // OUTPUT_TRIGGER_EPSILON = 0.001 min (:939)
    const long long t_floor = (long long)floor(t + 0.001);
    std::vector<OutTask> rows;
    const int bank = o->bank;
    for (size_t k = 0; k < o->pc.size(); k++) {
        PrintCtrl &p = o->pc[k];
        p.num_update++;
        if (t_floor % p.interval != 0) continue;
        rows.push_back(OutTask{bank, (int)k, (double)(t_floor - (long long)p.interval)});   // left endpoint
    }
    if (rows.empty()) return SHUD_OK;
    // a free host bank (the writers may still be writing the one used two events ago)
    {
        std::unique_lock<std::mutex> lk(o->mu);
        o->cv.wait(lk, [&] { return o->bank_left[bank] == 0; });
    }
    // the snapshots are free once the previous copy has finished
    if (o->copy_pending) HIP_TRY(hipStreamWaitEvent(o->stream, o->ev_copied[bank ^ 1], 0));
    for (const auto &r : rows) {
        PrintCtrl &p = o->pc[r.ctrl];
        const double f = p.tau / p.num_update;
        if (p.numvar > 0)
            hipLaunchKernelGGL(k_snap, dim3((p.numvar + 255) / 256), dim3(256), 0, o->stream, p.d_buf, p.d_snap,
                               p.numvar, f);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(o->ev_snap, o->stream));
    HIP_TRY(hipStreamWaitEvent(o->s_copy, o->ev_snap, 0));
    for (const auto &r : rows) {
        PrintCtrl &p = o->pc[r.ctrl];
        if (p.numvar > 0)
            HIP_TRY(hipMemcpyAsync(p.h_buf[bank], p.d_snap, p.numvar * sizeof(double), hipMemcpyDeviceToHost,
                                   o->s_copy));
    }
    HIP_TRY(hipEventRecord(o->ev_copied[bank], o->s_copy));
    // every launch and copy is enqueued: only now are the rows committed (a failure above returns with the
    // intervals still open and nothing queued for the writers)
    for (const auto &r : rows) {
        PrintCtrl &p = o->pc[r.ctrl];
        p.num_update = 0;
        p.rows++;
    }
    o->bank ^= 1;
    o->copy_pending = true;
    {
        std::lock_guard<std::mutex> lk(o->mu);
        o->bank_left[bank] = (int)rows.size();
        for (const auto &r : rows) o->tasks[r.ctrl % kWriters].push_back(r);
    }
    o->cv.notify_all();
    return SHUD_OK;
}

extern "C" int shud_out_flush(shud_out_t o) {
    if (!o) return shud_fail(SHUD_ERR_ARG, "null argument");
    out_drain(o);
    return out_report(o);
}

extern "C" int64_t shud_out_rows(shud_out_t o, int k) {
    if (!o || k < 0 || k >= (int)o->pc.size()) return -1;
    if (out_drain(o)) return out_report(o);          // a writer failure: its (negative) error code
    return o->pc[k].rows;
}

extern "C" int shud_out_destroy(shud_out_t o) {
    if (!o) return SHUD_OK;
    (void)hipSetDevice(o->device);
    out_drain(o);
    const int rc = out_report(o);
    {
        std::lock_guard<std::mutex> lk(o->mu);
        o->stop = true;
    }
    o->cv.notify_all();
    for (int w = 0; w < kWriters; w++)
        if (o->writer[w].joinable()) o->writer[w].join();
    (void)hipStreamSynchronize(o->stream);
    (void)hipStreamSynchronize(o->s_copy);
    for (PrintCtrl &p : o->pc) {
        if (p.fb) fclose(p.fb);
        if (p.fa) fclose(p.fa);
        if (p.d_buf) (void)hipFree(p.d_buf);
        if (p.d_snap) (void)hipFree(p.d_snap);
        if (p.d_sel) (void)hipFree(p.d_sel);
        for (int b = 0; b < 2; b++)
            if (p.h_buf[b]) (void)hipHostFree(p.h_buf[b]);
    }
    if (o->d_slots) (void)hipFree(o->d_slots);
    if (o->ev_snap) (void)hipEventDestroy(o->ev_snap);
    for (int b = 0; b < 2; b++)
        if (o->ev_copied[b]) (void)hipEventDestroy(o->ev_copied[b]);
    if (o->s_copy) (void)hipStreamDestroy(o->s_copy);
    delete o;
    return rc;
}

// ---------------------------------------------------------------------------------------------
// device sources on the RHS handle
// ---------------------------------------------------------------------------------------------
extern "C" int shud_rhs_prepare_outputs(shud_rhs_t h) {
    if (!h) return shud_fail(SHUD_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(h->device));
    const size_t len[5] = {(size_t)h->n_own, (size_t)h->n_own, (size_t)h->n_own, (size_t)h->n_own_riv,
                           (size_t)h->NL};
    int rc;
    for (int k = 0; k < 5; k++)
        if (!h->d_sum[k] && (rc = h->upload(&h->d_sum[k], (const double *)nullptr, len[k]))) return rc;
    if ((rc = shud_ensure_diag(h))) return rc;
    if (!h->d_zero_lake && (rc = h->upload(&h->d_zero_lake, (const double *)nullptr, std::max(h->NL, 1)))) return rc;
    if (!h->d_trans && ((rc = h->upload(&h->d_trans, (const double *)nullptr, h->NE)) ||
                        (rc = h->upload(&h->d_evapo, (const double *)nullptr, h->NE))))
        return rc;
    return SHUD_OK;
}

extern "C" int shud_rhs_summary(shud_rhs_t h, const double *d_y) {
    if (!h || !d_y) return shud_fail(SHUD_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(h->device));
    const int ne = h->n_own, nr = h->n_own_riv, nl = h->NL;
    const size_t len[5] = {(size_t)ne, (size_t)ne, (size_t)ne, (size_t)nr, (size_t)nl};
    for (int k = 0; k < 5; k++)
        if (!h->d_sum[k]) {
            int rc = h->dalloc(&h->d_sum[k], len[k]);
            if (rc) return rc;
        }
    const int n = std::max(ne, std::max(nr, nl));
    if (n > 0)
        hipLaunchKernelGGL(k_summary, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->dm, d_y, ne, nr, nl,
                           h->d_sum[0], h->d_sum[1], h->d_sum[2], h->d_sum[3], h->d_sum[4]);
    HIP_TRY(hipGetLastError());
    return SHUD_OK;
}

extern "C" int shud_rhs_refresh_diagnostics(shud_rhs_t h) {
    if (!h) return shud_fail(SHUD_ERR_ARG, "null argument");
    int rc = shud_diag_replay(h);
    if (rc) return rc;
    const int ne = h->NE;
    if (!h->d_trans && ((rc = h->dalloc(&h->d_trans, ne)) || (rc = h->dalloc(&h->d_evapo, ne)))) return rc;
    if (ne > 0)
        hipLaunchKernelGGL(k_et_sums, dim3((ne + 255) / 256), dim3(256), 0, h->stream, h->dd, ne, h->d_trans,
                           h->d_evapo);
    HIP_TRY(hipGetLastError());
    return SHUD_OK;
}

extern "C" const double *shud_rhs_device_array(shud_rhs_t h, int which, int64_t *n) {
    if (!h) return nullptr;
    const int64_t ne = h->n_own, nr = h->n_own_riv, nl = h->NL;
    const double *p = nullptr;
    int64_t len = 0;
    const DevDiag &d = h->dd;
    switch (which) {
        case SHUD_ARR_Y_ELE_SURF: p = h->d_sum[0]; len = ne; break;
        case SHUD_ARR_Y_ELE_UNSAT: p = h->d_sum[1]; len = ne; break;
        case SHUD_ARR_Y_ELE_GW: p = h->d_sum[2]; len = ne; break;
        case SHUD_ARR_Y_RIV_STG: p = h->d_sum[3]; len = nr; break;
        case SHUD_ARR_Y_LAKE_STG: p = h->d_sum[4]; len = nl; break;
        case SHUD_ARR_QELE_SURF_TOT: p = d.qele_surf_tot; len = ne; break;
        case SHUD_ARR_QELE_SUB_TOT: p = d.qele_sub_tot; len = ne; break;
        case SHUD_ARR_QELE_SURF: p = d.qele_surf; len = 3 * (int64_t)h->NE; break;
        case SHUD_ARR_QELE_SUB: p = d.qele_sub; len = 3 * (int64_t)h->NE; break;
        case SHUD_ARR_QE2R_SURF: p = d.qe2r_surf; len = ne; break;
        case SHUD_ARR_QE2R_SUB: p = d.qe2r_sub; len = ne; break;
        case SHUD_ARR_Q_INFIL: p = d.q_infil; len = ne; break;
        case SHUD_ARR_Q_EXFIL: p = d.q_exfil; len = ne; break;
        case SHUD_ARR_Q_RECHARGE: p = d.q_recharge; len = ne; break;
        case SHUD_ARR_Q_ETA: p = d.q_eta; len = ne; break;
        case SHUD_ARR_Q_E_IC: p = d.e_ic; len = ne; break;
        case SHUD_ARR_Q_TRANS: p = h->d_trans; len = ne; break;
        case SHUD_ARR_Q_EVAPO: p = h->d_evapo; len = ne; break;
        case SHUD_ARR_QRIV_DOWN: p = d.qriv_down; len = nr; break;
        case SHUD_ARR_QRIV_UP: p = d.qriv_up; len = nr; break;
        case SHUD_ARR_QRIV_SURF: p = d.qriv_surf; len = nr; break;
        case SHUD_ARR_QRIV_SUB: p = d.qriv_sub; len = nr; break;
        case SHUD_ARR_Q_PRCP: p = h->dm.prcp; len = ne; break;
        case SHUD_ARR_Q_NET_PRCP: p = h->dm.net_prep; len = ne; break;
        case SHUD_ARR_Q_ETP: p = h->dm.etp; len = ne; break;
        case SHUD_ARR_Y_ELE_IS: p = shud_et_array(h, which); len = ne; break;
        case SHUD_ARR_Y_ELE_SNOW: p = shud_et_array(h, which); len = ne; break;
        case SHUD_ARR_RN_H: p = shud_et_array(h, which); len = ne; break;
        case SHUD_ARR_RN_T: p = shud_et_array(h, which); len = ne; break;
        case SHUD_ARR_RN_FACTOR: p = shud_et_array(h, which); len = ne; break;
        case SHUD_ARR_LAKE_TOPAREA: p = nl ? d.lake_toparea : nullptr; len = nl; break;
        case SHUD_ARR_Q_LAKE_EVAP: p = nl ? d.q_lake_evap : nullptr; len = nl; break;
        case SHUD_ARR_Q_LAKE_PRCP: p = nl ? d.q_lake_prcp : nullptr; len = nl; break;
        case SHUD_ARR_Q_LAKE_RIVIN: p = nl ? d.q_lake_rivin : nullptr; len = nl; break;
        case SHUD_ARR_Q_LAKE_RIVOUT: p = nl ? h->d_zero_lake : nullptr; len = nl; break;
        case SHUD_ARR_Q_LAKE_SURF: p = nl ? d.q_lake_surf : nullptr; len = nl; break;
        case SHUD_ARR_Q_LAKE_SUB: p = nl ? d.q_lake_sub : nullptr; len = nl; break;
        default: break;
    }
    if (n) *n = p ? len : 0;
    return p;
}
