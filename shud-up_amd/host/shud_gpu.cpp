// shud_gpu.cpp — C++ host of the device path: SHUD() (src/Model/shud.cpp:32-170) with the RHS, the ET-step
// prelude, the integrator and the outputs on one MI355X, driven through the C-ABIs of include/.
//
//   shud_gpu [-o outdir] [-e end_day] [-n num_steps] [-C cwd] [-q] <input_dir> <project>
//   shud_gpu --rhs-check K | --rhs-bench [--evals N] ...   partitioned RHS modes (shud_gpu_part.cpp)
//
// input_dir/<project>.* are the reference's input files (FileIn, IO.cpp:53-91); forcing csv paths in
// <project>.tsd.forc resolve against -C (default: the process cwd, as the reference runs from its repository
// root), then against input_dir.  Outputs: <outdir>/<project>.<suffix>.dat in Print_Ctrl's byte layout
// (default outdir: output/<project>.out, IO.cpp:54).  Exit codes: 0, or the reference's myexit codes for
// physics errors (10/13) and 1 for input / solver / device errors.
//
// The loop below is shud.cpp:86-140 line by line:
//   for i < NumSteps:  tnext += SolverStep
//     while t + ZERO < tnext:  tout = ET sub-step ? min(t + ETStep, tnext) : tnext
//        updateAllTimeSeries(t); updateforcing(t); ET(t, tout)   -> shud_project_forcing + shud_et_step
//        [CVodeSetStopTime(tout)]; CVode(mem, tout, udata, &t, CV_NORMAL)  -> shud_ode_solve (y in HBM)
//     summary(udata); ExportResults(t)   -> shud_rhs_summary + shud_rhs_refresh_diagnostics + shud_out_export
// Not restated (out of the device path's scope): water-balance diagnostics (SHUD_WB_DIAG), flood alerts,
// the screen print / .cfg.ic.update snapshots, NetCDF forcing and outputs, the uncoupled -g mode.
#include <sys/stat.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "shud_et.h"
#include "shud_host.h"
#include "shud_ode.h"
#include "shud_out.h"
#include "shud_rhs.h"

static constexpr double kZero = 1.0e-10;          // ZERO (Macros.hpp:32)

static void usage() {
    fprintf(stderr, "usage: shud_gpu [-o outdir] [-e end_day] [-n num_steps] [-C cwd] [-q] <input_dir> <project>\n"
                    "       shud_gpu --rhs-check K | --rhs-bench [--evals N] [-o outdir] [-C cwd] <input_dir> <project>\n");
}

int shud_gpu_rhs_partition(shud_project_t p, int nparts_check, bool bench, int nevals, const std::string &outdir,
                           bool quiet);

static int mkdirs(const std::string &d) {
    std::string cur;
    for (size_t i = 0; i <= d.size(); i++) {
        if (i == d.size() || d[i] == '/') {
            if (!cur.empty()) mkdir(cur.c_str(), 0755);
        }
        if (i < d.size()) cur += d[i];
    }
    struct stat st;
    return stat(d.c_str(), &st) == 0 ? 0 : -1;
}

static const char *lonlat_name(int m) { return m == 1 ? "FORCING_MEAN" : (m == 2 ? "FIXED" : "FORCING_FIRST"); }

int main(int argc, char **argv) {
    std::string outdir, cwd;
    double end_day = -1.0;
    long long max_steps = -1;
    bool quiet = false;
    int rhs_check = 0, evals = 0;
    bool rhs_bench = false;
    std::vector<const char *> pos;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "-o" && i + 1 < argc) outdir = argv[++i];
        else if (a == "-e" && i + 1 < argc) end_day = atof(argv[++i]);
        else if (a == "-n" && i + 1 < argc) max_steps = atoll(argv[++i]);
        else if (a == "-C" && i + 1 < argc) cwd = argv[++i];
        else if (a == "-q") quiet = true;
        else if (a == "--rhs-check" && i + 1 < argc) rhs_check = atoi(argv[++i]);
        else if (a == "--rhs-bench") rhs_bench = true;
        else if (a == "--evals" && i + 1 < argc) evals = atoi(argv[++i]);
        else if (a == "-h" || a == "--help") { usage(); return 0; }
        else pos.push_back(argv[i]);
    }
    if (pos.size() != 2) { usage(); return 1; }
    const char *indir = pos[0], *prj = pos[1];
    if (outdir.empty()) outdir = std::string("output/") + prj + ".out";
    const auto wall0 = std::chrono::steady_clock::now();

    // ---- loadinput + initialize + LoadIC (shud.cpp:49-64) ----
    shud_project_t p = nullptr;
    if (shud_project_load(indir, prj, cwd.empty() ? nullptr : cwd.c_str(), end_day, &p)) {
        fprintf(stderr, "%s\n", shud_project_error());
        return 1;
    }
    if (rhs_check > 0 || rhs_bench) {
        const int rc = shud_gpu_rhs_partition(p, rhs_check, rhs_bench, evals > 0 ? evals : (rhs_bench ? 100 : 6),
                                              outdir, quiet);
        shud_project_free(p);
        return rc;
    }
    ShudControl c;
    shud_project_control(p, &c);
    ShudMeshSoA mesh;
    ShudParamsSoA par;
    shud_project_mesh(p, &mesh, &par);
    int64_t ny = 0;
    const double *y0 = shud_project_array(p, "y0", &ny);
    const double *y_is = shud_project_array(p, "y_is", nullptr);
    const double *y_snow = shud_project_array(p, "y_snow", nullptr);
    if (!quiet)
        printf("* \t Project: %s  NumEle %d  NumRiv %d  NumSeg %d  NumLake %d  NY %lld\n"
               "* \t StartTime %.1f  EndTime %.1f [min]  SolverStep %.1f  ETStep %.1f  NumSteps %lld\n",
               prj, mesh.num_ele, mesh.num_riv, mesh.num_seg, mesh.num_lake, (long long)ny, c.start_time,
               c.end_time, c.solver_step, c.et_step, (long long)c.num_steps);

    // ---- the device side: RHS handle, ET prelude, integrator (SetCVODE, cvode_config.cpp:149-197) ----
    ShudRhsOptions ro = {SHUD_MODE_SERIAL, 0, nullptr, 1};
    shud_rhs_t h = nullptr;
    if (shud_rhs_create(&mesh, &par, &ro, &h)) {
        fprintf(stderr, "shud_rhs_create: %s\n", shud_rhs_last_error_string());
        return 1;
    }
    ShudEtMeshSoA etm;
    ShudEtParams etp;
    shud_project_et(p, &etm, &etp);
    if (shud_et_attach(h, &etm, &etp) || shud_et_set_state(h, y_is, y_snow)) {
        fprintf(stderr, "shud_et_attach: %s\n", shud_rhs_last_error_string());
        return 1;
    }
    // carried u_satn before the first RHS: updateforcing's updateElement on f_update's globals, which are
    // freshly allocated (zero) before the first f() call -> u_satn = 0 (satn of an empty column)
    std::vector<double> zeros(mesh.num_ele, 0.0);
    ShudStepInputs si = {};
    si.u_satn = zeros.data();
    if (shud_rhs_set_step_inputs(h, &si)) {
        fprintf(stderr, "shud_rhs_set_step_inputs: %s\n", shud_rhs_last_error_string());
        return 1;
    }
    ShudOdeOptions oo = {c.reltol, c.abstol, c.init_step, c.max_step, 1e-6, 1000000, 0, 0};
    shud_ode_t ode = nullptr;
    if (shud_ode_create(h, c.start_time, y0, SHUD_WHERE_HOST, &oo, &ode)) {
        fprintf(stderr, "shud_ode_create: %s\n", shud_rhs_last_error_string());
        return 1;
    }
    double *d_y = nullptr;
    if (shud_rhs_device_alloc(h, (size_t)ny * sizeof(double), (void **)&d_y) ||
        shud_rhs_memcpy(h, d_y, y0, (size_t)ny * sizeof(double), 1)) {
        fprintf(stderr, "device alloc: %s\n", shud_rhs_last_error_string());
        return 1;
    }

    // ---- initialize_output (MD_initialize.cpp:246-345) with device sources ----
    if (mkdirs(outdir)) {
        fprintf(stderr, "cannot create output directory %s\n", outdir.c_str());
        return 1;
    }
    shud_rhs_prepare_outputs(h);
    shud_rhs_summary(h, d_y);
    shud_out_t out = nullptr;
    shud_out_create(0, shud_rhs_stream(h), &out);
    const int nd = shud_project_outputs(p, outdir.c_str(), nullptr, 0);
    std::vector<ShudOutputDecl> decl(nd);
    shud_project_outputs(p, outdir.c_str(), decl.data(), nd);
    int nprint = 0;
    for (const auto &d : decl) {
        int64_t n = 0;
        const double *src = shud_rhs_device_array(h, d.array, &n);
        if (!src) {
            fprintf(stderr, "no device source for %s\n", d.basename);
            return 1;
        }
        if (d.column >= 0) src += (size_t)d.column * mesh.num_ele;
        ShudPrintSpec ps = {d.basename, src, d.n_all, d.flag_io, d.interval, d.iflux, (int64_t)c.forc_start_time,
                            c.binary, c.ascii, c.radiation_input_mode, c.terrain_radiation,
                            lonlat_name(c.solar_lonlat_mode), c.solar_lon_deg, c.solar_lat_deg};
        if (shud_out_add(out, &ps)) {
            fprintf(stderr, "shud_out_add(%s): %s\n", d.basename, shud_rhs_last_error_string());
            return 1;
        }
        nprint++;
    }

    // ---- the time loop (shud.cpp:86-140) ----
    shud_rhs_synchronize(h);
    const auto loop0 = std::chrono::steady_clock::now();
    const bool et_sub = c.et_step > kZero && c.et_step + kZero < c.solver_step;
    double t = c.start_time, tnext = t;
    const long long nsteps = max_steps >= 0 && max_steps < c.num_steps ? max_steps : c.num_steps;
    int rc = 0;
    // wall time per phase of the loop (host view: includes waiting on the device where a phase synchronizes)
    double ph[5] = {0, 0, 0, 0, 0};         // forcing+BC rows, ET step, CVode, summary+diagnostics, export
    auto tick = std::chrono::steady_clock::now();
    auto lap = [&](int k) {
        const auto now = std::chrono::steady_clock::now();
        ph[k] += std::chrono::duration<double>(now - tick).count();
        tick = now;
    };
    for (long long i = 0; i < nsteps && !rc; i++) {
        tnext += c.solver_step;
        while (t + kZero < tnext) {
            const double tout = et_sub ? std::fmin(t + c.et_step, tnext) : tnext;
            ShudEtForcing f;
            if (shud_project_forcing(p, t, tout, &f)) {
                fprintf(stderr, "%s\n", shud_project_error());
                rc = 1;
                break;
            }
            ShudStepInputs bc = {};                 // tsd_eyBC .. tsd_rqBC rows (f_update's getX)
            if (shud_project_bc_rows(p, &bc) == 1 && shud_rhs_set_step_inputs(h, &bc)) {
                fprintf(stderr, "shud_rhs_set_step_inputs (BC rows): %s\n", shud_rhs_last_error_string());
                rc = 1;
                break;
            }
            lap(0);
            if (shud_et_step(h, &f)) {
                ShudErr e;
                shud_rhs_get_error(h, &e);
                fprintf(stderr, "%s\n", e.message[0] ? e.message : shud_rhs_last_error_string());
                rc = e.exit_code ? e.exit_code : 1;
                break;
            }
            lap(1);
            if (et_sub) shud_ode_set_stop_time(ode, tout);
            const int flag = shud_ode_solve(ode, tout, d_y, SHUD_WHERE_DEVICE, &t, SHUD_ODE_NORMAL);
            if (flag < 0) {
                ShudErr e;
                shud_rhs_get_error(h, &e);
                if (flag == SHUD_ODE_RHSFUNC_FAIL && e.exit_code) {
                    printf("\n%s\n", e.message);
                    fprintf(stderr, "\nEXIT with error code %d\n", e.exit_code);
                    rc = e.exit_code;
                } else {
                    fprintf(stderr, "CVode failed with flag %d at t = %f (%s)\n", flag, t, shud_rhs_last_error_string());
                    rc = 1;
                }
                break;
            }
            lap(2);
        }
        if (rc) break;
        shud_rhs_summary(h, d_y);                 // Model_Data::summary(udata)
        shud_rhs_refresh_diagnostics(h);          // the flux arrays of CVODE's last f() call
        lap(3);
        if (shud_out_export(out, t)) {            // Control_Data::ExportResults(t)
            fprintf(stderr, "shud_out_export: %s\n", shud_rhs_last_error_string());
            rc = 1;
        }
        lap(4);
        if (!quiet && c.verbose) printf("step %lld  t = %.3f min\n", i + 1, t);
    }
    shud_rhs_synchronize(h);
    const double loop_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - loop0).count();
    shud_out_destroy(out);
    ShudOdeStats st;
    shud_ode_get_stats(ode, &st);
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - wall0).count();
    if (!quiet)
        printf("* \t t = %.3f min  steps %lld  RHS %lld  Newton %lld  Krylov %lld  err-test fails %lld  "
               "%d outputs  wall %.2f s (time loop %.2f s)\n",
               t, (long long)st.nst, (long long)(st.nfe + st.nfe_ls), (long long)st.nni, (long long)st.nli,
               (long long)st.netf, nprint, wall, loop_s);
    // one machine-readable line (tools/e2e.sh)
    printf("{\"shud_gpu\": {\"num_ele\": %d, \"t_end_min\": %.6f, \"solver_steps\": %lld, \"cvode_steps\": %lld, "
           "\"rhs_evals\": %lld, \"newton_iters\": %lld, \"krylov_iters\": %lld, \"outputs\": %d, "
           "\"wall_s\": %.4f, \"loop_s\": %.4f, \"loop_phases_s\": {\"forcing\": %.4f, \"et_step\": %.4f, "
           "\"cvode\": %.4f, \"summary_diag\": %.4f, \"export\": %.4f}, \"host_syncs\": %lld, \"exit\": %d}}\n",
           mesh.num_ele, t, nsteps, (long long)st.nst, (long long)(st.nfe + st.nfe_ls), (long long)st.nni,
           (long long)st.nli, nprint, wall, loop_s, ph[0], ph[1], ph[2], ph[3], ph[4], (long long)st.n_sync, rc);
    shud_ode_destroy(ode);
    shud_rhs_device_free(h, d_y);
    shud_rhs_destroy(h);
    shud_project_free(p);
    return rc;
}
