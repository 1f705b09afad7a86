// shud_gpu_part.cpp — the partitioned RHS modes of shud_gpu (include/shud_partition.h).
//
//   shud_gpu --rhs-check K [--evals N] [-C cwd] <input_dir> <project>
//       one process, one GPU: the project's mesh split K ways by the C++ partitioner, one partitioned RHS handle
//       per part (local mesh + ghosts gathered by the C++ planner), the halo moved between the handles' device
//       buffers by D2D copies (the bytes RCCL would move), step inputs from the device ET prelude run on every
//       local mesh.  Every eval's owned DY of every part must equal the unpartitioned handle's bit for bit.
//   shud_gpu --rhs-bench [--evals N] [-o outdir] [-C cwd] <input_dir> <project>
//       one process per GPU (RANK / WORLD_SIZE / LOCAL_RANK from the environment, e.g.
//       `torchrun --no-python --nproc-per-node 8 shud-up_amd/shud_gpu --rhs-bench ...`): the rank's part on
//       device LOCAL_RANK with the RCCL halo exchange (rank 0 publishes the RCCL unique id in
//       <outdir>/.shud_nccl_id); N device-resident RHS evals timed per rank, one JSON line per rank.
// The reference evaluates the same RHS as one OpenMP loop over the whole mesh (src/ModelData/MD_f_omp.cpp:12-66,
// MD_f.cpp:9-50); a partitioned handle computes the owned part of it exactly (global reduction orders).
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <ctime>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "shud_et.h"
#include "shud_host.h"
#include "shud_partition.h"
#include "shud_rhs.h"

namespace {

struct Rank {
    shud_plan_t plan = nullptr;
    ShudPartition part{};
    ShudMeshSoA lmesh{};
    ShudParamsSoA lpar{};
    shud_rhs_t h = nullptr;
    int n_own = 0, n_own_riv = 0, ne = 0;
    std::vector<double> y_own, dy_own, ref_own;
    double *d_y = nullptr, *d_dy = nullptr;
    double *esend = nullptr, *rsend = nullptr, *gele = nullptr, *griv = nullptr;
    // local ET statics (gathered)
    std::vector<int32_t> iforc, ilc, imf, ilake;
    std::vector<double> z_surf, albedo, fix_p, wind_h, veg, nx, ny, nz, y_is, y_snow;
};

int fail(const char *what) {
    fprintf(stderr, "%s: %s %s\n", what, shud_rhs_last_error_string(), shud_partition_error());
    return 1;
}

// the project's ET statics gathered to a rank's local elements
ShudEtMeshSoA local_et(Rank &r, const ShudEtMeshSoA &g) {
    const int ne = r.ne;
    auto gi = [&](const int32_t *src, std::vector<int32_t> &dst) -> const int32_t * {
        if (!src) return nullptr;
        dst.resize(ne);
        shud_plan_gather_ele_i32(r.plan, src, dst.data());
        return dst.data();
    };
    auto gd = [&](const double *src, std::vector<double> &dst) -> const double * {
        if (!src) return nullptr;
        dst.resize(ne);
        shud_plan_gather_ele(r.plan, src, dst.data());
        return dst.data();
    };
    ShudEtMeshSoA l = g;
    l.num_ele = ne;
    l.iforc = gi(g.iforc, r.iforc);
    l.ilc = gi(g.ilc, r.ilc);
    l.imf = gi(g.imf, r.imf);
    l.ilake = gi(g.ilake, r.ilake);
    l.z_surf = gd(g.z_surf, r.z_surf);
    l.albedo = gd(g.albedo, r.albedo);
    l.fix_pressure = gd(g.fix_pressure, r.fix_p);
    l.wind_h = gd(g.wind_h, r.wind_h);
    l.veg_frac = gd(g.veg_frac, r.veg);
    l.nx = gd(g.nx, r.nx);
    l.ny = gd(g.ny, r.ny);
    l.nz = gd(g.nz, r.nz);
    return l;
}

// attach the ET prelude, IC storages and u_satn = 0 (as the driver does before the first RHS), run one ET step
int prepare_handle(shud_rhs_t h, const ShudEtMeshSoA &etm, const ShudEtParams &etp, const double *y_is,
                   const double *y_snow, int ne, ShudEtForcing *f) {
    if (shud_et_attach(h, &etm, &etp) || shud_et_set_state(h, y_is, y_snow)) return fail("shud_et_attach");
    std::vector<double> zeros(ne, 0.0);
    ShudStepInputs si = {};
    si.u_satn = zeros.data();
    if (shud_rhs_set_step_inputs(h, &si)) return fail("shud_rhs_set_step_inputs");
    if (shud_et_step(h, f)) return fail("shud_et_step");
    return 0;
}

// a deterministic state near the IC: surface water, unsaturated storage and heads perturbed per entity
std::vector<double> test_state(const double *y0, int64_t ny, int ne, int k) {
    std::vector<double> y(y0, y0 + ny);
    for (int64_t i = 0; i < ny; i++) {
        const double u = 0.5 + 0.5 * std::sin(0.7 * (double)i + 1.3 * k);
        if (i < ne) y[i] = 0.02 * u;                          // surface water depth
        else y[i] = y[i] * (0.9 + 0.2 * u);
    }
    return y;
}

// the RCCL id file of one job: "<token>\n" + 128 id bytes.  The token names the job, from the most specific source
// the environment offers: SHUD_JOB_ID when the caller sets it (any launcher, several nodes sharing the outdir, per-rank
// wrapper scripts); else torchrun's run id when it is a real one (static rendezvous leaves it at "none"), with the
// rendezvous address and port; else that address and port with the launcher's pid (every local rank of one job is a
// direct child of the same launcher process — torchrun's agent or bench.py — and a later job's launcher is another
// process; address and port alone would accept an earlier job's file).  The last form needs single-node ranks that
// are direct children of one launcher: a rank that finds a fresh id file under another token says so and stops.
std::string job_token() {
    const char *run = getenv("TORCHELASTIC_RUN_ID"), *ma = getenv("MASTER_ADDR"), *mp = getenv("MASTER_PORT");
    const char *jid = getenv("SHUD_JOB_ID");
    if (jid && *jid) return std::string("job:") + jid;
    const std::string addr = std::string(ma ? ma : "-") + ":" + (mp ? mp : "-");
    if (run && *run && strcmp(run, "none") != 0) return std::string("run:") + run + ":" + addr;
    return "ppid:" + addr + ":" + std::to_string((long)getppid());
}

// the token of a fresh id file (written after `not_before`), "" if there is none
std::string id_file_token(const std::string &f, time_t not_before) {
    struct stat st;
    if (stat(f.c_str(), &st) != 0 || st.st_mtime < not_before) return "";
    FILE *fp = fopen(f.c_str(), "rb");
    if (!fp) return "";
    char buf[512];
    const size_t n = fread(buf, 1, sizeof buf - 1, fp);
    fclose(fp);
    buf[n] = 0;
    const char *nl = strchr(buf, '\n');
    return nl ? std::string(buf, nl - buf) : "";
}

// the 128 id bytes of `f` if it carries `token` and was written after `not_before` (seconds since the epoch)
std::string read_id_file(const std::string &f, const std::string &token, time_t not_before) {
    struct stat st;
    if (stat(f.c_str(), &st) != 0 || st.st_mtime < not_before) return "";
    FILE *fp = fopen(f.c_str(), "rb");
    if (!fp) return "";
    std::string s(token.size() + 1 + 128, '\0');
    const size_t n = fread(&s[0], 1, s.size(), fp);
    fclose(fp);
    if (n != s.size() || s.compare(0, token.size(), token) != 0 || s[token.size()] != '\n') return "";
    return s.substr(token.size() + 1);
}

int mkdirs(const std::string &d) {
    std::string cur;
    for (size_t i = 0; i <= d.size(); i++) {
        if ((i == d.size() || d[i] == '/') && !cur.empty()) mkdir(cur.c_str(), 0755);
        if (i < d.size()) cur += d[i];
    }
    struct stat st;
    return stat(d.c_str(), &st) == 0 ? 0 : -1;
}

}  // namespace

int shud_gpu_rhs_partition(shud_project_t p, int nparts_check, bool bench, int nevals, const std::string &outdir,
                           bool quiet) {
    ShudControl c;
    shud_project_control(p, &c);
    ShudMeshSoA mesh;
    ShudParamsSoA par;
    shud_project_mesh(p, &mesh, &par);
    int64_t ny = 0;
    const double *y0 = shud_project_array(p, "y0", &ny);
    const double *y_is = shud_project_array(p, "y_is", nullptr);
    const double *y_snow = shud_project_array(p, "y_snow", nullptr);
    const double *cx = shud_project_array(p, "x", nullptr);
    const double *cy = shud_project_array(p, "y", nullptr);
    ShudEtMeshSoA etm;
    ShudEtParams etp;
    shud_project_et(p, &etm, &etp);
    ShudEtForcing f;
    if (shud_project_forcing(p, c.start_time, c.start_time + c.et_step, &f)) {
        fprintf(stderr, "%s\n", shud_project_error());
        return 1;
    }
    const int NE = mesh.num_ele;
    const int rank = bench ? atoi(getenv("RANK") ? getenv("RANK") : "0") : 0;
    const int world = bench ? atoi(getenv("WORLD_SIZE") ? getenv("WORLD_SIZE") : "1") : nparts_check;
    const int local = bench ? atoi(getenv("LOCAL_RANK") ? getenv("LOCAL_RANK") : "0") : 0;
    const int K = world;
    if (K < 1 || K > SHUD_PART_MAX_PARTS) { fprintf(stderr, "bad part count %d\n", K); return 1; }

    // ---- partition (every rank computes the same one: deterministic) ----
    std::vector<int32_t> ele_part(NE, 0);
    ShudPartStats st{};
    const auto tp = std::chrono::steady_clock::now();
    if (K > 1 && shud_partition_mesh(&mesh, cx, cy, K, SHUD_PART_AUTO, 12345, ele_part.data(), &st))
        return fail("shud_partition_mesh");
    const double part_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tp).count();

    if (!bench) {
        // ======== --rhs-check K: all parts in this process on one GPU, D2D halo ========
        ShudRhsOptions ro = {SHUD_MODE_SERIAL, 0, nullptr, 1};
        shud_rhs_t g = nullptr;
        if (shud_rhs_create(&mesh, &par, &ro, &g)) return fail("shud_rhs_create");
        if (prepare_handle(g, etm, etp, y_is, y_snow, NE, &f)) return 1;
        std::vector<Rank> R(K);
        for (int r = 0; r < K; r++) {
            Rank &q = R[r];
            if (shud_plan_build(&mesh, ele_part.data(), K, r, &q.plan) || shud_plan_partition(q.plan, &q.part) ||
                shud_plan_local_mesh(q.plan, &mesh, &par, &q.lmesh, &q.lpar))
                return fail("shud_plan");
            q.ne = q.lmesh.num_ele;
            q.n_own = q.part.n_own_ele;
            q.n_own_riv = q.part.n_own_riv;
            if (shud_rhs_create_partitioned(&q.lmesh, &q.lpar, &ro, &q.part, &q.h)) return fail("create_partitioned");
            std::vector<double> lis(q.ne), lsn(q.ne);
            shud_plan_gather_ele(q.plan, y_is, lis.data());
            shud_plan_gather_ele(q.plan, y_snow, lsn.data());
            const ShudEtMeshSoA le = local_et(q, etm);
            if (prepare_handle(q.h, le, etp, lis.data(), lsn.data(), q.ne, &f)) return 1;
            ShudPlanInfo I;
            shud_plan_info(q.plan, &I);
            const size_t no = 3 * (size_t)q.n_own + q.n_own_riv + I.n_own_lake;   // [sf|us|gw|riv|lake]
            q.y_own.resize(no);
            q.dy_own.resize(no);
            q.ref_own.resize(no);
            if (shud_rhs_device_alloc(q.h, no * 8, (void **)&q.d_y) || shud_rhs_device_alloc(q.h, no * 8, (void **)&q.d_dy) ||
                shud_rhs_halo_buffers(q.h, &q.esend, &q.rsend, &q.gele, &q.griv))
                return fail("device buffers");
        }
        std::vector<double> dy(ny);
        long long mismatched = 0;
        double t_part = 0., t_one = 0.;
        for (int e = 0; e < nevals; e++) {
            const std::vector<double> y = test_state(y0, ny, NE, e / 3);   // 3 successive calls per state
            auto t0 = std::chrono::steady_clock::now();
            if (shud_rhs_eval(g, 0.0, y.data(), dy.data(), SHUD_WHERE_HOST)) return fail("shud_rhs_eval");
            t_one += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            t0 = std::chrono::steady_clock::now();
            for (auto &q : R) {
                shud_plan_owned_state(q.plan, y.data(), NE, q.y_own.data());
                shud_rhs_memcpy(q.h, q.d_y, q.y_own.data(), q.y_own.size() * 8, 1);
                if (shud_rhs_eval_pack(q.h, q.d_y)) return fail("eval_pack");
                shud_rhs_synchronize(q.h);
            }
            for (int r = 0; r < K; r++) {                     // the all-to-all-v as D2D copies
                Rank &q = R[r];
                for (int s = 0; s < K; s++) {
                    if (s == r) continue;
                    const Rank &src = R[s];
                    const int e0 = src.part.ele_send_off[r], e1 = src.part.ele_send_off[r + 1];
                    const int d0 = q.part.ele_recv_off[s];
                    if (e1 > e0 && shud_rhs_memcpy(q.h, q.gele + 3 * (size_t)d0, src.esend + 3 * (size_t)e0,
                                                   24 * (size_t)(e1 - e0), 3)) return fail("halo copy");
                    const int r0 = src.part.riv_send_off[r], r1 = src.part.riv_send_off[r + 1];
                    const int q0 = q.part.riv_recv_off[s];
                    if (r1 > r0 && shud_rhs_memcpy(q.h, q.griv + q0, src.rsend + r0, 8 * (size_t)(r1 - r0), 3))
                        return fail("halo copy");
                }
            }
            for (auto &q : R) {
                if (shud_rhs_eval_compute(q.h, 0.0, q.d_y, q.d_dy)) return fail("eval_compute");
                shud_rhs_memcpy(q.h, q.dy_own.data(), q.d_dy, q.dy_own.size() * 8, 2);
                shud_rhs_synchronize(q.h);
            }
            t_part += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            for (auto &q : R) {
                shud_plan_owned_state(q.plan, dy.data(), NE, q.ref_own.data());
                for (size_t k = 0; k < q.ref_own.size(); k++)
                    if (memcmp(&q.ref_own[k], &q.dy_own[k], 8) != 0) mismatched++;
            }
        }
        int64_t max_ge = 0, max_gr = 0;
        for (auto &q : R) {
            ShudPlanInfo I;
            shud_plan_info(q.plan, &I);
            max_ge = std::max<int64_t>(max_ge, I.n_ghost_ele);
            max_gr = std::max<int64_t>(max_gr, I.n_ghost_riv);
        }
        printf("{\"shud_gpu_rhs_check\": {\"num_ele\": %d, \"parts\": %d, \"evals\": %d, \"mismatched_entries\": %lld, "
               "\"method\": \"%s\", \"edge_cut\": %lld, \"segment_cut\": %lld, \"imbalance\": %.4f, "
               "\"max_ghost_ele\": %lld, \"max_ghost_riv\": %lld, \"partition_s\": %.3f, \"host_eval_s_single\": %.4f, "
               "\"host_eval_s_parts\": %.4f}}\n",
               NE, K, nevals, mismatched, K > 1 ? (st.method_used == SHUD_PART_RCB ? "rcb" : "multilevel") : "none",
               (long long)st.edge_cut, (long long)st.segment_cut, st.imbalance, (long long)max_ge, (long long)max_gr,
               part_s, t_one, t_part);
        for (auto &q : R) {
            shud_rhs_device_free(q.h, q.d_y);
            shud_rhs_device_free(q.h, q.d_dy);
            shud_rhs_destroy(q.h);
            shud_plan_free(q.plan);
        }
        shud_rhs_destroy(g);
        return mismatched ? 2 : 0;
    }

    // ======== --rhs-bench: one process per GPU, RCCL halo ========
    ShudRhsOptions ro = {SHUD_MODE_SERIAL, local, nullptr, 1};
    Rank q;
    std::string nccl_id;
    shud_rhs_t h = nullptr;
    if (K == 1) {
        if (shud_rhs_create(&mesh, &par, &ro, &h)) return fail("shud_rhs_create");
        if (prepare_handle(h, etm, etp, y_is, y_snow, NE, &f)) return 1;
        q.n_own = NE;
        q.n_own_riv = mesh.num_riv;
    } else {
        if (mkdirs(outdir)) { fprintf(stderr, "cannot create %s\n", outdir.c_str()); return 1; }
        const std::string idf = outdir + "/.shud_nccl_id";
        const std::string token = job_token();
        if (rank == 0) {
            unlink(idf.c_str());                              // never leave an earlier job's id in place
            char id[128];
            if (shud_rhs_nccl_unique_id(id)) return fail("nccl id");
            const std::string tmp = idf + ".tmp";
            FILE *fp = fopen(tmp.c_str(), "wb");
            if (!fp || fwrite(token.data(), 1, token.size(), fp) != token.size() || fputc('\n', fp) == EOF ||
                fwrite(id, 1, 128, fp) != 128) {
                fprintf(stderr, "cannot write %s\n", tmp.c_str());
                return 1;
            }
            fclose(fp);
            rename(tmp.c_str(), idf.c_str());
            nccl_id.assign(id, 128);
        } else {
            const time_t not_before = time(nullptr) - 60;     // a file older than this job's start is stale
            for (int w = 0; w < 1200 && nccl_id.empty(); w++) {   // up to 120 s
                nccl_id = read_id_file(idf, token, not_before);
                if (nccl_id.empty()) std::this_thread::sleep_for(std::chrono::milliseconds(100));
            }
            if (nccl_id.empty()) {
                const std::string other = id_file_token(idf, not_before);
                if (!other.empty() && other != token)
                    fprintf(stderr, "rank %d: %s holds the RCCL id of job '%s', not this job '%s' (ranks of one job "
                                    "must share SHUD_JOB_ID, or be direct children of one launcher on one node)\n",
                            rank, idf.c_str(), other.c_str(), token.c_str());
                else
                    fprintf(stderr, "rank %d: no RCCL id in %s\n", rank, idf.c_str());
                return 1;
            }
        }
        if (shud_plan_build(&mesh, ele_part.data(), K, rank, &q.plan) || shud_plan_partition(q.plan, &q.part) ||
            shud_plan_local_mesh(q.plan, &mesh, &par, &q.lmesh, &q.lpar))
            return fail("shud_plan");
        q.part.nccl_unique_id = nccl_id.data();
        q.ne = q.lmesh.num_ele;
        q.n_own = q.part.n_own_ele;
        q.n_own_riv = q.part.n_own_riv;
        if (shud_rhs_create_partitioned(&q.lmesh, &q.lpar, &ro, &q.part, &h)) return fail("create_partitioned");
        std::vector<double> lis(q.ne), lsn(q.ne);
        shud_plan_gather_ele(q.plan, y_is, lis.data());
        shud_plan_gather_ele(q.plan, y_snow, lsn.data());
        const ShudEtMeshSoA le = local_et(q, etm);
        if (prepare_handle(h, le, etp, lis.data(), lsn.data(), q.ne, &f)) return 1;
    }
    size_t no = (size_t)ny;                                  // K = 1: the whole y, lakes included
    if (K > 1) {
        ShudPlanInfo I;
        shud_plan_info(q.plan, &I);
        no = 3 * (size_t)q.n_own + q.n_own_riv + I.n_own_lake;   // owned [sf|us|gw|riv|lake]
    }
    const std::vector<double> y = test_state(y0, ny, NE, 0);
    std::vector<double> yo(no);
    if (K == 1) yo = y;
    else shud_plan_owned_state(q.plan, y.data(), NE, yo.data());
    double *d_y = nullptr, *d_dy = nullptr;
    if (shud_rhs_device_alloc(h, no * 8, (void **)&d_y) || shud_rhs_device_alloc(h, no * 8, (void **)&d_dy) ||
        shud_rhs_memcpy(h, d_y, yo.data(), no * 8, 1))
        return fail("device buffers");
    for (int w = 0; w < 5; w++)
        if (shud_rhs_eval(h, 0.0, d_y, d_dy, SHUD_WHERE_DEVICE)) return fail("eval");
    shud_rhs_synchronize(h);
    shud_rhs_timing(h, nevals, nevals >= 20 ? 5 : 1);
    const auto t0 = std::chrono::steady_clock::now();
    for (int e = 0; e < nevals; e++)
        if (shud_rhs_eval(h, 0.0, d_y, d_dy, SHUD_WHERE_DEVICE)) return fail("eval");
    shud_rhs_synchronize(h);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    double me = 0, mr = 0, mv = 0;
    int nt = 0;
    shud_rhs_timing_read(h, &me, &mr, &mv, &nt);
    ShudErr err;
    shud_rhs_get_error(h, &err);
    printf("{\"shud_gpu_rhs_bench\": {\"rank\": %d, \"world\": %d, \"num_ele\": %d, \"own_ele\": %d, \"local_ele\": %d, "
           "\"evals\": %d, \"s\": %.6f, \"ms_per_eval\": %.5f, \"ele_kernel_ms\": %.5f, \"riv_kernel_ms\": %.5f, "
           "\"element_updates_per_s_rank\": %.4e, \"partition_s\": %.3f, \"exit_code\": %d}}\n",
           rank, K, NE, q.n_own, K == 1 ? NE : q.ne, nevals, dt, dt / nevals * 1e3, me, mr,
           (double)q.n_own * nevals / dt, part_s, err.exit_code);
    (void)quiet;
    shud_rhs_device_free(h, d_y);
    shud_rhs_device_free(h, d_dy);
    shud_rhs_destroy(h);
    if (q.plan) shud_plan_free(q.plan);
    return 0;
}
