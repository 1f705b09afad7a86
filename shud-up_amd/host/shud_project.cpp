// shud_project.cpp — SHUD project readers and Model_Data::initialize, restated in C++ for the device path's
// host (include/shud_host.h).  Every function cites the reference routine it follows; the derived arrays are
// checked bit for bit against the Python restatement (shud_rhs/shudio.py) by tests/test_host.py.
#include <strings.h>

#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <set>

#include "shud_host_impl.hpp"
#include "shud_out.h"

namespace shudhost {

static thread_local std::string g_err;

int fail(Project *p, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    if (p) p->err = buf;
    return -1;
}
const char *last_error() { return g_err.c_str(); }

static constexpr int kMaxLen = 2048;             // MAXLEN (Macros.hpp:30)
static constexpr double kMinRivSlope = 4e-4;     // MINRIVSLOPE (Macros.hpp:47)
static constexpr double kZero = 1.0e-10;         // ZERO (Macros.hpp:32)
static constexpr double kHeightWind = 10;        // HeightWindMeasure (Macros.hpp:71)

// TabularData::read(FILE*, int*) (TabularData.cpp:27-50)
bool read_table(FILE *fp, Table &t) {
    char str[kMaxLen];
    t = Table{};
    if (!fgets(str, kMaxLen, fp)) return false;
    if (sscanf(str, "%d %d", &t.nrow, &t.ncol) != 2 || t.nrow < 0 || t.ncol < 0) return false;
    t.x.assign((size_t)t.nrow * t.ncol, 0.0);
    if (!fgets(str, kMaxLen, fp)) return t.nrow == 0;
    t.header = str;
    for (int i = 0; i < t.nrow && fgets(str, kMaxLen, fp); i++) {
        char *ps = str;
        for (int j = 0; j < t.ncol; j++) t.x[(size_t)i * t.ncol + j] = (double)strtold(ps, &ps);
    }
    return true;
}

static std::string path_of(const Project &p, const char *ext) { return p.indir + "/" + p.prj + "." + ext; }

static int read_table_file(Project &p, const std::string &fn, Table &t) {
    FILE *fp = fopen(fn.c_str(), "r");
    if (!fp) return fail(&p, "Fatal Error: %s is in use or does not exist!", fn.c_str());
    const bool ok = read_table(fp, t);
    fclose(fp);
    return ok ? 0 : fail(&p, "cannot parse table %s", fn.c_str());
}

static std::string upper(const char *s) {
    std::string u(s);
    for (auto &c : u) c = (char)toupper((unsigned char)c);
    return u;
}

// globalCal::read (ModelConfigure.cpp:443-459): "KEY value" lines, '#', blank and space-led lines skipped.
// Defaults: calib_* members (ModelConfigure.hpp:12-41, 117-131; River.hpp:15-25).
static int read_calib(Project &p) {
    static const char *ones[] = {"GEOL_KSATH", "GEOL_KSATV", "GEOL_KMACSATH", "GEOL_DMAC", "GEOL_THETAS",
                                 "GEOL_THETAR", "GEOL_MACVF", "SOIL_KINF", "SOIL_KMACSATV", "SOIL_DINF",
                                 "SOIL_ALPHA", "SOIL_BETA", "SOIL_MACHF", "LC_VEGFRAC", "LC_ALBEDO", "LC_ROUGH",
                                 "LC_SOILDGD", "LC_DROOT", "LC_IMPAF", "LC_ISMAX", "RIV_ROUGH", "RIV_KH",
                                 "RIV_CWR", "RIV_DPTH+", "RIV_WDTH+", "RIV_BSLOPE+", "RIV_SINU", "RIV_BEDTHICK",
                                 "TS_PRCP", "TS_LAI", "TS_MF", "ET_ETP", "ET_IC", "ET_TR", "ET_SOIL"};
    for (const char *k : ones) p.cal[k] = 1.0;
    p.cal["AQ_DEPTH+"] = 0.0;
    p.cal["TS_SFCTMP+"] = 0.0;
    p.cal["IC_GW+"] = 0.0;
    p.cal["IC_RIV+"] = 0.0;
    const std::string fn = path_of(p, "cfg.calib");
    FILE *fp = fopen(fn.c_str(), "r");
    if (!fp) return fail(&p, "Fatal Error: %s is in use or does not exist!", fn.c_str());
    char str[kMaxLen], key[kMaxLen];
    while (fgets(str, kMaxLen, fp)) {
        if (str[0] == '#' || str[0] == '\n' || str[0] == '\0' || str[0] == ' ') continue;
        double v = 0.0;
        if (sscanf(str, "%s %lf", key, &v) != 2) continue;
        const std::string k = upper(key);
        if (k == "FZN_SUBMAX") p.fz_sub_max = v;
        else if (k == "FZN_SUBMIN") p.fz_sub_min = v;
        else if (k == "FZN_SUBDAY") p.fz_sub_day = v;
        else if (k == "FZN_SURFMAX") p.fz_surf_max = v;
        else if (k == "FZN_SURFMIN") p.fz_surf_min = v;
        else if (k == "FZN_SURFDAY") p.fz_surf_day = v;
        else p.cal[k] = v;
    }
    fclose(fp);
    return 0;
}

// Control_Data::read (Model_Control.cpp:141-502) for the keys the device path uses, then updateSimPeriod
// (:132-137).  Output intervals: PrintOutDt (Model_Control.hpp:116-147).
static int read_para(Project &p, double end_day) {
    ShudControl &c = p.ctl;
    c.close_boundary = 1; c.ascii = 0; c.binary = 1; c.init_type = 3; c.cryosphere = 0; c.verbose = 0;
    c.abstol = 1.0e-4; c.reltol = 1.0e-3; c.init_step = 1.e-2; c.max_step = 30; c.et_step = 60;
    c.radiation_input_mode = 0; c.solar_lonlat_mode = 0; c.terrain_radiation = 1;
    c.rad_factor_cap = 5.0; c.rad_cosz_min = 0.05; c.tsr_integration_step_min = 60;
    double day_start = 0, day_end = 10;
    const std::string fn = path_of(p, "cfg.para");
    FILE *fp = fopen(fn.c_str(), "r");
    if (!fp) return fail(&p, "Fatal Error: %s is in use or does not exist!", fn.c_str());
    char str[kMaxLen], opt[kMaxLen], mode[kMaxLen];
    double val = 0.0;                            // sscanf leaves it unchanged when the value does not parse
    struct { const char *k; int *v; } dts[] = {
        {"dt_ye_ic", &p.dt_ye_ic}, {"dt_ye_SNOW", &p.dt_ye_snow}, {"dt_ye_SURF", &p.dt_ye_surf},
        {"dt_ye_UNSAT", &p.dt_ye_unsat}, {"dt_ye_GW", &p.dt_ye_gw}, {"dt_qe_PRCP", &p.dt_qe_prcp},
        {"dt_qe_rech", &p.dt_qe_rech}, {"dt_qe_infil", &p.dt_qe_infil}, {"dt_Qe_sub", &p.dt_Qe_sub},
        {"dt_Qe_subx", &p.dt_Qe_subx}, {"dt_Qe_surf", &p.dt_Qe_surf}, {"dt_Qe_surfx", &p.dt_Qe_surfx},
        {"dt_Qe_rsub", &p.dt_Qe_rsub}, {"dt_Qe_rsurf", &p.dt_Qe_rsurf}, {"dt_yr_stage", &p.dt_yr_stage},
        {"dt_Qr_Surf", &p.dt_Qr_surf}, {"dt_Qr_Sub", &p.dt_Qr_sub}, {"dt_Qr_down", &p.dt_Qr_down},
        {"dt_Qr_up", &p.dt_Qr_up}, {"dt_lake", &p.dt_lake}};
    while (fgets(str, kMaxLen, fp)) {
        if (str[0] == '#' || str[0] == '\n' || str[0] == '\0' || str[0] == ' ') continue;
        opt[0] = '\0';
        sscanf(str, "%s %lf", opt, &val);
        auto is = [&](const char *k) { return strcasecmp(k, opt) == 0; };
        bool done = false;
        for (auto &d : dts)
            if (is(d.k)) { *d.v = (int)val; done = true; }
        if (done) continue;
        if (is("dt_qe_ET")) { p.dt_qe_et = p.dt_qe_etp = p.dt_qe_eta = (int)val; }
        else if (is("ASCII_OUTPUT")) c.ascii = (int)val;
        else if (is("BINARY_OUTPUT")) c.binary = (int)val;
        else if (is("VERBOSE")) c.verbose = (int)val;
        else if (is("CloseBoundary")) c.close_boundary = (int)val;
        else if (is("INIT_MODE")) c.init_type = (int)val;
        else if (is("ABSTOL")) c.abstol = val;
        else if (is("RELTOL")) c.reltol = val;
        else if (is("INIT_SOLVER_STEP")) c.init_step = val;
        else if (is("MAX_SOLVER_STEP")) c.max_step = val;
        else if (is("ET_STEP") || is("LSM_STEP")) c.et_step = val;
        else if (is("START")) day_start = val;
        else if (is("END")) day_end = val;
        else if (is("cryosphere")) c.cryosphere = (int)val;
        else if (is("SOLAR_LON_DEG")) p.solar_lon_fixed = val;
        else if (is("SOLAR_LAT_DEG")) p.solar_lat_fixed = val;
        else if (is("TERRAIN_RADIATION")) { if ((int)val == 0 || (int)val == 1) c.terrain_radiation = (int)val; }
        else if (is("SOLAR_UPDATE_INTERVAL")) { if ((int)val > 0) c.tsr_integration_step_min = (int)val; }
        else if (is("TSR_INTEGRATION_STEP_MIN")) { if ((int)val > 0) c.tsr_integration_step_min = (int)val; }
        else if (is("RAD_FACTOR_CAP")) { if (std::isfinite(val) && val > 0.0) c.rad_factor_cap = val; }
        else if (is("RAD_COSZ_MIN")) { if (std::isfinite(val) && val >= 0.0) c.rad_cosz_min = val > 1.0 ? 1.0 : val; }
        else if (is("RADIATION_INPUT_MODE")) {
            c.radiation_input_mode = 0;
            if (sscanf(str, "%s %s", opt, mode) == 2) {
                if (strcasecmp(mode, "SWNET") == 0) c.radiation_input_mode = 1;
                else if (strcasecmp(mode, "SWDOWN") != 0) {
                    char *e = nullptr;
                    const double mv = strtod(mode, &e);
                    if (e && *e == '\0' && (mv == 0.0 || mv == 1.0)) c.radiation_input_mode = mv == 1.0;
                }
            }
        } else if (is("SOLAR_LONLAT_MODE")) {
            c.solar_lonlat_mode = 0;
            if (sscanf(str, "%s %s", opt, mode) == 2) {
                if (strcasecmp(mode, "FORCING_MEAN") == 0) c.solar_lonlat_mode = 1;
                else if (strcasecmp(mode, "FIXED") == 0) c.solar_lonlat_mode = 2;
                else if (strcasecmp(mode, "FORCING_FIRST") != 0) {
                    char *e = nullptr;
                    const double mv = strtod(mode, &e);
                    if (e && *e == '\0' && (mv == 0.0 || mv == 1.0 || mv == 2.0)) c.solar_lonlat_mode = (int)mv;
                }
            }
        } else if (is("FORCING_MODE")) {
            if (sscanf(str, "%s %s", opt, mode) == 2 && strcasecmp(mode, "NETCDF") == 0) {
                fclose(fp);
                return fail(&p, "FORCING_MODE NETCDF is out of scope (NetCDF forcing provider); use CSV forcing");
            }
        }
        // other keys (SCR_INTV, NUM_OPENMP, SpinupDay, OUTPUT_MODE, ...) do not reach the device path
    }
    fclose(fp);
    if (end_day >= 0) day_end = end_day;
    c.solver_step = c.max_step;                                             // Model_Control.cpp:502
    c.start_time = day_start * 1440;                                        // updateSimPeriod
    c.end_time = day_end * 1440;
    c.num_steps = (int64_t)(unsigned long)((double)(unsigned long)(c.end_time - c.start_time) / c.solver_step);
    return 0;
}

static double eudist(double x1, double y1, double x2, double y2) {           // functions.hpp Eudist
    const double dx = x2 - x1, dy = y2 - y1;
    return sqrt(dx * dx + dy * dy);
}
static void perp_on_line(double *xx, double *yy, double x, double y, double x1, double y1, double x2,
                         double y2) {                                        // functions.cpp:259-288
    const double A = x - x1, B = y - y1, C = x2 - x1, D = y2 - y1;
    const double dot = A * C + B * D;
    const double len_sq = C * C + D * D;
    double param = -1.;
    if (len_sq != 0) param = dot / len_sq;
    if (param < 0.) { *xx = x1; *yy = y1; }
    else if (param > 1.) { *xx = x2; *yy = y2; }
    else { *xx = x1 + param * C; *yy = y1 + param * D; }
}
static inline double rmin(double a, double b) { return a > b ? b : a; }     // functions.hpp min/max
static inline double rmax(double a, double b) { return a < b ? b : a; }

int load(Project &p, const char *indir, const char *prj, const char *cwd, double end_day) {
    p.indir = indir;
    p.prj = prj;
    int rc;
    if ((rc = read_para(p, end_day)) || (rc = read_calib(p))) return rc;
    auto cal = [&](const char *k) { return p.cal.at(k); };

    // ---- read_mesh (MD_readin.cpp:192-236): elements [index, node1..3, nabr1..3], then nodes ----
    Table mesh, nodes, att, soil, geol, lc, riv, rtype, seg;
    {
        const std::string fn = path_of(p, "sp.mesh");
        FILE *fp = fopen(fn.c_str(), "r");
        if (!fp) return fail(&p, "Fatal Error: %s is in use or does not exist!", fn.c_str());
        const bool ok = read_table(fp, mesh) && read_table(fp, nodes);
        fclose(fp);
        if (!ok || mesh.ncol < 7 || nodes.ncol < 5) return fail(&p, "bad mesh file %s", fn.c_str());
    }
    if ((rc = read_table_file(p, path_of(p, "sp.att"), att))) return rc;
    if ((rc = read_table_file(p, path_of(p, "para.soil"), soil))) return rc;
    if ((rc = read_table_file(p, path_of(p, "para.geol"), geol))) return rc;
    if ((rc = read_table_file(p, path_of(p, "para.lc"), lc))) return rc;
    {
        const std::string fn = path_of(p, "sp.riv");
        FILE *fp = fopen(fn.c_str(), "r");
        if (!fp) return fail(&p, "Fatal Error: %s is in use or does not exist!", fn.c_str());
        const bool ok = read_table(fp, riv) && read_table(fp, rtype);
        fclose(fp);
        if (!ok) return fail(&p, "bad river file %s", fn.c_str());
    }
    if ((rc = read_table_file(p, path_of(p, "sp.rivseg"), seg))) return rc;
    if (att.ncol != 9) return fail(&p, "%s: %d columns, the reference requires 9", path_of(p, "sp.att").c_str(), att.ncol);
    const int NE = p.NE = mesh.nrow, NR = p.NR = riv.nrow, NS = p.NS = seg.nrow, NN = p.NumNode = nodes.nrow;
    p.NumLC = lc.nrow;
    if (att.nrow < NE) return fail(&p, "sp.att has %d rows for %d elements", att.nrow, NE);

    // ---- calibrated parameter tables: applyCalib (ModelConfigure.cpp:79-139, River.cpp:23-45) ----
    const int nso = soil.nrow, nge = geol.nrow, nlc = lc.nrow, nrt = rtype.nrow;
    std::vector<double> S_infK(nso), S_thS(nso), S_thR(nso), S_infD(nso), S_beta(nso), S_hA(nso), S_macKV(nso);
    for (int r = 0; r < nso; r++) {
        S_infK[r] = soil.at(r, 1) / 1440.0 * cal("SOIL_KINF");
        S_thS[r] = soil.at(r, 2);
        S_thR[r] = soil.at(r, 3);
        S_infD[r] = soil.at(r, 4) * cal("SOIL_DINF");
        const double b = soil.at(r, 6) * cal("SOIL_BETA");
        S_beta[r] = b < 1.1 ? 1.1 : b;
        S_hA[r] = soil.at(r, 7) * cal("SOIL_MACHF");
        S_macKV[r] = soil.at(r, 8) / 1440.0 * cal("SOIL_KMACSATV");
    }
    std::vector<double> G_KH(nge), G_KV(nge), G_vA(nge), G_macKH(nge), G_macD(nge), G_Sy(nge);
    for (int r = 0; r < nge; r++) {
        G_KH[r] = geol.at(r, 1) / 1440.0 * cal("GEOL_KSATH");
        G_KV[r] = geol.at(r, 2) / 1440.0 * cal("GEOL_KSATV");
        G_vA[r] = geol.at(r, 5) * cal("GEOL_MACVF");
        G_macKH[r] = geol.at(r, 6) / 1440.0 * cal("GEOL_KMACSATH");
        G_macD[r] = geol.at(r, 7) * cal("GEOL_DMAC");
        G_Sy[r] = cal("GEOL_THETAS") * geol.at(r, 3) - cal("GEOL_THETAR") * geol.at(r, 4);
    }
    std::vector<double> L_alb(nlc), L_veg(nlc), L_rough(nlc), L_rzd(nlc), L_sdg(nlc), L_imp(nlc);
    for (int r = 0; r < nlc; r++) {
        L_alb[r] = lc.at(r, 1) * cal("LC_ALBEDO");
        L_veg[r] = lc.at(r, 2) * cal("LC_VEGFRAC");
        L_rough[r] = lc.at(r, 3) / 60.0 * cal("LC_ROUGH");
        L_rzd[r] = lc.at(r, 4) * cal("LC_DROOT");
        L_sdg[r] = lc.at(r, 5) * cal("LC_SOILDGD");
        L_imp[r] = lc.at(r, 6) * cal("LC_IMPAF");
    }
    std::vector<double> R_depth(nrt), R_bs(nrt), R_bw(nrt), R_rough(nrt), R_cwr(nrt), R_kh(nrt), R_bt(nrt);
    for (int r = 0; r < nrt; r++) {
        R_depth[r] = rtype.at(r, 1) + cal("RIV_DPTH+");
        R_bs[r] = rtype.at(r, 2) + cal("RIV_BSLOPE+");
        R_bw[r] = rtype.at(r, 3) + cal("RIV_WDTH+");
        R_rough[r] = rtype.at(r, 5) / 60.0 * cal("RIV_ROUGH");
        R_cwr[r] = rtype.at(r, 6) * cal("RIV_CWR");
        R_kh[r] = rtype.at(r, 7) / 1440.0 * cal("RIV_KH");
        R_bt[r] = rtype.at(r, 8) * cal("RIV_BEDTHICK");
    }

    // ---- Node::Init (Node.cpp:13-20) and _Element::applyGeometry (Element.cpp:62-217) ----
    const double caqd = cal("AQ_DEPTH+");
    std::vector<double> zmin(NN);
    for (int k = 0; k < NN; k++) zmin[k] = nodes.at(k, 4) - (nodes.at(k, 3) + caqd);
    p.area.resize(NE); p.z_surf.resize(NE); p.z_bottom.resize(NE); p.cx.resize(NE); p.cy.resize(NE);
    p.edge.resize(3 * (size_t)NE); p.d2e.resize(3 * (size_t)NE); p.d2n.resize(3 * (size_t)NE);
    p.avg_rough.resize(3 * (size_t)NE); p.nabr.resize(3 * (size_t)NE);
    p.nx.resize(NE); p.ny.resize(NE); p.nz.resize(NE); p.slope_angle.resize(NE); p.aspect.resize(NE);
    for (int i = 0; i < NE; i++) {
        int nd[3];
        for (int j = 0; j < 3; j++) {
            nd[j] = (int)mesh.at(i, 1 + j) - 1;                               // Node[node[k] - 1]: positional
            if (nd[j] < 0 || nd[j] >= NN) return fail(&p, "element %d: node %d out of range", i + 1, nd[j] + 1);
            const int nb = (int)mesh.at(i, 4 + j) - 1;
            p.nabr[(size_t)j * NE + i] = nb < -1 ? -1 : nb;                   // file 0 -> -1; lake (<0) -> -1
        }
        const double x1 = nodes.at(nd[0], 1), x2 = nodes.at(nd[1], 1), x3 = nodes.at(nd[2], 1);
        const double y1 = nodes.at(nd[0], 2), y2 = nodes.at(nd[1], 2), y3 = nodes.at(nd[2], 2);
        const double zx1 = nodes.at(nd[0], 4), zx2 = nodes.at(nd[1], 4), zx3 = nodes.at(nd[2], 4);
        p.area[i] = 0.5 * ((x2 - x1) * (y3 - y1) - (y2 - y1) * (x3 - x1));
        p.z_surf[i] = (zx1 + zx2 + zx3) / 3.0;
        p.z_bottom[i] = (zmin[nd[0]] + zmin[nd[1]] + zmin[nd[2]]) / 3.0;
        const double x = (x1 + x2 + x3) / 3.0, y = (y1 + y2 + y3) / 3.0;
        p.cx[i] = x; p.cy[i] = y;
        p.edge[0 * (size_t)NE + i] = eudist(x2, y2, x3, y3);
        p.edge[1 * (size_t)NE + i] = eudist(x3, y3, x1, y1);
        p.edge[2 * (size_t)NE + i] = eudist(x1, y1, x2, y2);
        double px, py;
        perp_on_line(&px, &py, x, y, x2, y2, x3, y3); p.d2e[0 * (size_t)NE + i] = eudist(px, py, x, y);
        perp_on_line(&px, &py, x, y, x3, y3, x1, y1); p.d2e[1 * (size_t)NE + i] = eudist(px, py, x, y);
        perp_on_line(&px, &py, x, y, x1, y1, x2, y2); p.d2e[2 * (size_t)NE + i] = eudist(px, py, x, y);
        // terrain normal (Element.cpp:148-217): surface points (x, y, zmax)
        const double v1x = x2 - x1, v1y = y2 - y1, v1z = zx2 - zx1;
        const double v2x = x3 - x1, v2y = y3 - y1, v2z = zx3 - zx1;
        const double nxr = v1y * v2z - v1z * v2y, nyr = v1z * v2x - v1x * v2z, nzr = v1x * v2y - v1y * v2x;
        const double nlen = sqrt(nxr * nxr + nyr * nyr + nzr * nzr);
        double nx = 0.0, ny = 0.0, nz = 1.0;
        if (!(nlen <= kZero)) {
            nx = nxr / nlen; ny = nyr / nlen; nz = nzr / nlen;
            if (nz < 0.0) { nx = -nx; ny = -ny; nz = -nz; }
        }
        p.nx[i] = nx; p.ny[i] = ny; p.nz[i] = nz;
        const double nzc = rmin(1.0, rmax(0.0, nz));
        const double sa = atan2(hypot(nx, ny), nzc);
        p.slope_angle[i] = sa;
        double asp = 0.0;
        if (!(sa < 1e-6)) {
            const double PI = 3.1415926;                                     // Macros.hpp:46 (truncated)
            asp = atan2(nx, ny);
            if (asp < 0.0) asp += 2.0 * PI;
            if (asp >= 2.0 * PI) asp -= 2.0 * PI;
        }
        p.aspect[i] = asp;
    }

    // ---- copyGeol/Soil/Landc, InitElement, SoilDgrd/ImpAF (MD_initialize.cpp:176-186; Element.cpp:218-237) ----
    p.aq.resize(NE); p.macD.resize(NE); p.macKsatH.resize(NE); p.vAreaF.resize(NE); p.KsatH.resize(NE);
    p.KsatV.resize(NE); p.infKsatV.resize(NE); p.hAreaF.resize(NE); p.macKsatV.resize(NE); p.ThetaS.resize(NE);
    p.ThetaR.resize(NE); p.Beta.resize(NE); p.infD.resize(NE); p.Sy.resize(NE); p.RzD.resize(NE);
    p.VegFrac.resize(NE); p.ImpAF.resize(NE); p.rough.resize(NE); p.albedo.resize(NE);
    p.ibc.resize(NE); p.iss.resize(NE); p.ilake.resize(NE); p.iforc.resize(NE); p.ilc.resize(NE); p.imf.resize(NE);
    for (int i = 0; i < NE; i++) {
        const int s = (int)att.at(i, 1) - 1, g = (int)att.at(i, 2) - 1, l = (int)att.at(i, 3) - 1;
        if (s < 0 || s >= nso || g < 0 || g >= nge || l < 0 || l >= nlc)
            return fail(&p, "element %d: soil/geol/lc index out of range", i + 1);
        p.KsatH[i] = G_KH[g]; p.KsatV[i] = G_KV[g]; p.vAreaF[i] = G_vA[g]; p.macKsatH[i] = G_macKH[g];
        p.Sy[i] = G_Sy[g];
        double macD = G_macD[g];
        p.infKsatV[i] = S_infK[s]; p.ThetaS[i] = S_thS[s]; p.ThetaR[i] = S_thR[s]; p.Beta[i] = S_beta[s];
        p.hAreaF[i] = S_hA[s]; p.macKsatV[i] = S_macKV[s]; p.infD[i] = S_infD[s];
        p.rough[i] = L_rough[l]; p.RzD[i] = L_rzd[l]; p.ImpAF[i] = L_imp[l]; p.albedo[i] = L_alb[l];
        const double aq = p.z_surf[i] - p.z_bottom[i];
        if (aq < macD) macD = aq;
        p.macD[i] = macD;
        p.infKsatV[i] = p.infKsatV[i] * (1 - L_sdg[l]);
        p.macKsatV[i] = p.macKsatV[i] * (1 - L_sdg[l]);
        p.VegFrac[i] = L_veg[l] * (1 - p.ImpAF[i]);
        p.ilc[i] = (int32_t)att.at(i, 3);
        p.iforc[i] = (int32_t)att.at(i, 4) - 1;
        p.imf[i] = (int32_t)att.at(i, 5);
        p.ibc[i] = (int32_t)att.at(i, 6);
        p.iss[i] = (int32_t)att.at(i, 7);
        p.ilake[i] = (int32_t)att.at(i, 8);
    }
    // segments -> RivID (MD_initialize.cpp:188-191), rmSinks (Model_Data.cpp:238-266): one pass in element
    // order, a raised element is seen raised by the later ones; then InitElement again
    std::vector<int> riv_id(NE, 0);
    p.seg_ele.resize(NS); p.seg_riv.resize(NS); p.seg_length.resize(NS); p.seg_cwr.resize(NS);
    for (int s = 0; s < NS; s++) {
        p.seg_riv[s] = (int32_t)seg.at(s, 1) - 1;
        p.seg_ele[s] = (int32_t)seg.at(s, 2) - 1;
        p.seg_length[s] = seg.at(s, 3);
        if (p.seg_ele[s] < 0 || p.seg_ele[s] >= NE || p.seg_riv[s] < 0 || p.seg_riv[s] >= NR)
            return fail(&p, "river segment %d: element/reach out of range", s + 1);
        riv_id[p.seg_ele[s]] = p.seg_riv[s] + 1;
    }
    for (int i = 0; i < NE; i++) p.aq[i] = p.z_surf[i] - p.z_bottom[i];
    for (int i = 0; i < NE; i++) {
        double zn = 1.0e200;
        for (int j = 0; j < 3; j++) {
            const int nb = p.nabr[(size_t)j * NE + i];
            if (nb >= 0) zn = rmin(zn, p.z_surf[nb]);
        }
        if (zn > p.z_surf[i] && riv_id[i] <= 0) {
            p.z_surf[i] = zn;
            p.z_bottom[i] = zn - p.aq[i];
        }
    }
    p.fixp.resize(NE); p.windh.assign(NE, kHeightWind); p.depression.assign(NE, 0.0002);
    for (int i = 0; i < NE; i++) {
        const double aq = p.z_surf[i] - p.z_bottom[i];                        // InitElement inside rmSinks
        p.aq[i] = aq;
        if (aq < p.macD[i]) p.macD[i] = aq;
        p.fixp[i] = 101.325 * pow((293. - 0.0065 * p.z_surf[i]) / 293, 5.26);  // PressureElevation
    }
    // applyNabor (Element.cpp:238-270)
    for (int j = 0; j < 3; j++)
        for (int i = 0; i < NE; i++) {
            const int nb = p.nabr[(size_t)j * NE + i];
            if (nb >= 0) {
                p.d2n[(size_t)j * NE + i] = eudist(p.cx[i], p.cy[i], p.cx[nb], p.cy[nb]);
                p.avg_rough[(size_t)j * NE + i] = 0.5 * (p.rough[i] + p.rough[nb]);
            } else {
                p.d2n[(size_t)j * NE + i] = 0.0;
                p.avg_rough[(size_t)j * NE + i] = p.rough[i];
            }
        }

    // ---- rivers: initialRiver/applyParameter, BedSlope >= MINRIVSLOPE, updateFrDownstream, segments ----
    p.riv_down.resize(NR); p.riv_bc.resize(NR); p.riv_length.resize(NR); p.riv_slope.resize(NR);
    p.riv_d2d.resize(NR); p.riv_avg_rough.resize(NR); p.riv_depth.resize(NR); p.riv_bw.resize(NR);
    p.riv_bs.resize(NR); p.riv_ksath.resize(NR); p.riv_bedthick.resize(NR);
    std::vector<double> rrough(NR);
    std::vector<int> rt(NR);
    for (int r = 0; r < NR; r++) {
        const int down = (int)riv.at(r, 1);
        if (down == 0) return fail(&p, "river reach %d with down == 0: the reference exits (MD_RiverFlux.cpp:55-57)", r + 1);
        rt[r] = (int)riv.at(r, 2) - 1;
        if (rt[r] < 0 || rt[r] >= nrt) return fail(&p, "river reach %d: type out of range", r + 1);
        p.riv_down[r] = down > 0 ? down - 1 : down;
        p.riv_bc[r] = (int32_t)riv.at(r, 5);
        p.riv_length[r] = riv.at(r, 4);
        p.riv_slope[r] = rmax(kMinRivSlope, riv.at(r, 3));
        rrough[r] = R_rough[rt[r]];
        p.riv_depth[r] = R_depth[rt[r]]; p.riv_bw[r] = R_bw[rt[r]]; p.riv_bs[r] = R_bs[rt[r]];
        p.riv_ksath[r] = R_kh[rt[r]]; p.riv_bedthick[r] = R_bt[rt[r]];
    }
    for (int r = 0; r < NR; r++) {
        const int d = p.riv_down[r];
        if (d >= 0) {
            if (d >= NR) return fail(&p, "river reach %d: down %d out of range", r + 1, d + 1);
            p.riv_avg_rough[r] = 0.5 * (rrough[r] + rrough[d]);
            p.riv_d2d[r] = 0.5 * (p.riv_length[r] + p.riv_length[d]);
        } else {
            p.riv_avg_rough[r] = rrough[r];
            p.riv_d2d[r] = p.riv_length[r];
        }
    }
    for (int s = 0; s < NS; s++) p.seg_cwr[s] = R_cwr[rt[p.seg_riv[s]]];       // MD_initialize.cpp:220-226

    // ---- lakes: lakeon when any iLake > 0 (MD_readin.cpp:262-263); bathymetry (MD_Lake.cpp:147-168) ----
    std::set<int> lakes;
    for (int i = 0; i < NE; i++)
        if (p.ilake[i] > 0) lakes.insert(p.ilake[i]);
    p.NL = (int)lakes.size();
    p.bathy_off.assign(1, 0);
    if (p.NL) {
        const std::string fn = path_of(p, "lake.bathy");
        FILE *fp = fopen(fn.c_str(), "r");
        if (!fp) return fail(&p, "Fatal Error: %s is in use or does not exist!", fn.c_str());
        for (int l = 0; l < p.NL; l++) {
            Table tb;
            if (!read_table(fp, tb) || tb.ncol < 3) { fclose(fp); return fail(&p, "bad lake bathymetry %s", fn.c_str()); }
            for (int r = 0; r < tb.nrow; r++) { p.bathy_y.push_back(tb.at(r, 1)); p.bathy_a.push_back(tb.at(r, 2)); }
            p.bathy_off.push_back(p.bathy_off.back() + tb.nrow);
        }
        fclose(fp);
    }
    p.ctl.lakeon = p.NL > 0;
    p.ctl.num_lake = p.NL;

    // ---- LoadIC (MD_initialize.cpp:66-135) ----
    const size_t NY = 3 * (size_t)NE + NR + p.NL;
    p.y0.assign(NY, 0.0); p.y_is.assign(NE, 0.0); p.y_snow.assign(NE, 0.0);
    double *ysf = p.y0.data(), *yus = ysf + NE, *ygw = yus + NE, *yriv = ygw + NE, *ylake = yriv + NR;
    switch (p.ctl.init_type) {
        case 0: for (int i = 0; i < NE; i++) ygw[i] = p.aq[i]; break;
        case 1: break;
        case 2:
            for (int i = 0; i < NE; i++) { yus[i] = 0.3 * p.aq[i]; ygw[i] = 0.4 * p.aq[i]; }
            for (int r = 0; r < NR; r++) yriv[r] = 0.2 * p.riv_depth[r];
            for (int l = 0; l < p.NL; l++) {
                const int o = p.bathy_off[l];
                ylake[l] = 0.3 * (p.bathy_y[o + 1] - p.bathy_y[o]);
            }
            break;
        default: {
            const std::string fn = path_of(p, "cfg.ic");
            FILE *fp = fopen(fn.c_str(), "r");
            if (!fp) return fail(&p, "Fatal Error: %s is in use or does not exist!", fn.c_str());
            Table te, tr, tl;
            const bool ok = read_table(fp, te) && read_table(fp, tr);
            if (!ok || te.ncol < 6 || te.nrow < NE || tr.ncol < 2 || tr.nrow < NR) {
                fclose(fp);
                return fail(&p, "%s: element/river tables do not cover the mesh", fn.c_str());
            }
            for (int i = 0; i < NE; i++) {
                p.y_is[i] = te.at(i, 1); p.y_snow[i] = te.at(i, 2);
                ysf[i] = te.at(i, 3); yus[i] = te.at(i, 4); ygw[i] = te.at(i, 5);
            }
            for (int r = 0; r < NR; r++) yriv[r] = tr.at(r, 1);
            if (p.NL) {
                const bool okl = read_table(fp, tl);
                for (int l = 0; l < p.NL; l++) ylake[l] = (okl && tl.nrow == p.NL && tl.ncol >= 2) ? tl.at(l, 1) : 2.;
            }
            fclose(fp);
        }
    }
    // read_cfgout (MD_readin.cpp:25-104): all columns on unless <prj>.cfg.output lists them; each table's
    // header line sets the default (atoi of its text), then "index ON/OFF" rows
    p.io_ele.assign(NE, 1);
    p.io_riv.assign(NR, 1);
    p.io_lake.assign(p.NL, 1);
    {
        const std::string fn = path_of(p, "cfg.output");
        FILE *fp = fopen(fn.c_str(), "r");
        if (fp) {
            std::vector<int32_t> *io[3] = {&p.io_ele, &p.io_riv, &p.io_lake};
            const int n[3] = {NE, NR, p.NL};
            for (int k = 0; k < 3; k++) {
                if (k > 0 && n[k] == 0) continue;
                Table tb;
                if (!read_table(fp, tb) || tb.ncol != 2) {
                    fclose(fp);
                    return fail(&p, "%s: the tables must have 2 columns (index, OFF/ON)", fn.c_str());
                }
                io[k]->assign(n[k], atoi(tb.header.c_str()));
                for (int r = 0; r < tb.nrow; r++) {
                    const int idx = (int)tb.at(r, 0) - 1;
                    if (idx >= 0 && idx < n[k]) (*io[k])[idx] = (int)tb.at(r, 1) > 0 ? 1 : 0;
                }
            }
            fclose(fp);
        }
    }
    if (int rc2 = read_bc(p)) return rc2;
    return read_forcing(p, cwd);
}

}  // namespace shudhost

using namespace shudhost;

extern "C" {

const char *shud_project_error(void) { return last_error(); }

int shud_project_load(const char *indir, const char *prj, const char *cwd, double end_day, shud_project_t *out) {
    if (!indir || !prj || !out) return fail(nullptr, "null argument");
    auto *p = new Project();
    if (load(*p, indir, prj, cwd, end_day)) {
        delete p;
        return -1;
    }
    *out = reinterpret_cast<shud_project_t>(p);
    return 0;
}

void shud_project_free(shud_project_t h) { delete reinterpret_cast<Project *>(h); }

int shud_project_control(shud_project_t h, ShudControl *c) {
    if (!h || !c) return fail(nullptr, "null argument");
    *c = reinterpret_cast<Project *>(h)->ctl;
    return 0;
}

int shud_project_mesh(shud_project_t h, ShudMeshSoA *m, ShudParamsSoA *q) {
    if (!h || !m || !q) return fail(nullptr, "null argument");
    Project &p = *reinterpret_cast<Project *>(h);
    memset(m, 0, sizeof *m);
    m->num_ele = p.NE; m->num_riv = p.NR; m->num_seg = p.NS; m->close_boundary = p.ctl.close_boundary;
    m->nabr = p.nabr.data(); m->area = p.area.data(); m->z_surf = p.z_surf.data(); m->z_bottom = p.z_bottom.data();
    m->depression = p.depression.data(); m->edge = p.edge.data(); m->dist2nabor = p.d2n.data();
    m->dist2edge = p.d2e.data(); m->avg_rough = p.avg_rough.data(); m->rough = p.rough.data();
    m->ibc = p.ibc.data(); m->iss = p.iss.data(); m->ilake = p.ilake.data();
    m->riv_down = p.riv_down.data(); m->riv_bc = p.riv_bc.data(); m->riv_length = p.riv_length.data();
    m->riv_bed_slope = p.riv_slope.data(); m->riv_dist2down = p.riv_d2d.data();
    m->riv_avg_rough = p.riv_avg_rough.data(); m->riv_depth = p.riv_depth.data();
    m->riv_bottom_width = p.riv_bw.data(); m->riv_bankslope = p.riv_bs.data(); m->riv_ksath = p.riv_ksath.data();
    m->riv_bedthick = p.riv_bedthick.data();
    m->seg_ele = p.seg_ele.data(); m->seg_riv = p.seg_riv.data(); m->seg_length = p.seg_length.data();
    m->seg_cwr = p.seg_cwr.data();
    m->num_lake = p.NL;
    if (p.NL) { m->lake_bathy_off = p.bathy_off.data(); m->lake_bathy_y = p.bathy_y.data(); m->lake_bathy_a = p.bathy_a.data(); }
    q->aquifer_depth = p.aq.data(); q->macD = p.macD.data(); q->macKsatH = p.macKsatH.data();
    q->geo_vAreaF = p.vAreaF.data(); q->KsatH = p.KsatH.data(); q->KsatV = p.KsatV.data();
    q->infKsatV = p.infKsatV.data(); q->hAreaF = p.hAreaF.data(); q->macKsatV = p.macKsatV.data();
    q->ThetaS = p.ThetaS.data(); q->ThetaR = p.ThetaR.data(); q->Beta = p.Beta.data(); q->infD = p.infD.data();
    q->Sy = p.Sy.data(); q->RzD = p.RzD.data(); q->VegFrac = p.VegFrac.data(); q->ImpAF = p.ImpAF.data();
    return 0;
}

int shud_project_et(shud_project_t h, ShudEtMeshSoA *m, ShudEtParams *q) {
    if (!h || !m || !q) return fail(nullptr, "null argument");
    Project &p = *reinterpret_cast<Project *>(h);
    m->num_ele = p.NE;
    m->iforc = p.iforc.data(); m->ilc = p.ilc.data(); m->imf = p.imf.data(); m->z_surf = p.z_surf.data();
    m->albedo = p.albedo.data(); m->fix_pressure = p.fixp.data(); m->wind_h = p.windh.data();
    m->veg_frac = p.VegFrac.data(); m->ilake = p.ilake.data();
    m->nx = p.nx.data(); m->ny = p.ny.data(); m->nz = p.nz.data();
    q->cPrep = p.cal.at("TS_PRCP"); q->cTemp = p.cal.at("TS_SFCTMP+"); q->cLAItsd = p.cal.at("TS_LAI");
    q->cMF = p.cal.at("TS_MF"); q->cETP = p.cal.at("ET_ETP");
    q->cISmax = 1.0;                 // gc.cISmax: LC_ISMAX sets clandc.cISmax, never gc.cISmax (ModelConfigure.cpp:175)
    q->radiation_input_mode = p.ctl.radiation_input_mode;
    q->terrain_radiation = p.ctl.terrain_radiation;
    q->rad_factor_cap = p.ctl.rad_factor_cap;
    q->rad_cosz_min = p.ctl.rad_cosz_min;
    q->cryosphere = p.ctl.cryosphere;
    q->ft_surf_day = (int32_t)p.fz_surf_day; q->ft_sub_day = (int32_t)p.fz_sub_day;
    q->ft_surf_max = p.fz_surf_max; q->ft_surf_min = p.fz_surf_min;
    q->ft_sub_max = p.fz_sub_max; q->ft_sub_min = p.fz_sub_min;
    return 0;
}

const double *shud_project_array(shud_project_t h, const char *name, int64_t *n) {
    if (!h || !name) return nullptr;
    Project &p = *reinterpret_cast<Project *>(h);
    struct { const char *k; const std::vector<double> *v; } t[] = {
        {"y0", &p.y0}, {"y_is", &p.y_is}, {"y_snow", &p.y_snow}, {"x", &p.cx}, {"y", &p.cy},
        {"slope_angle", &p.slope_angle}, {"aspect", &p.aspect}, {"albedo", &p.albedo},
        {"fix_pressure", &p.fixp}, {"nx", &p.nx}, {"ny", &p.ny}, {"nz", &p.nz}};
    for (auto &e : t)
        if (strcmp(e.k, name) == 0) {
            if (n) *n = (int64_t)e.v->size();
            return e.v->data();
        }
    if (n) *n = 0;
    return nullptr;
}

// Model_Data::initialize_output (MD_initialize.cpp:246-345) + FileOut::updateFilePath names (IO.cpp:130-186)
int shud_project_outputs(shud_project_t h, const char *outdir, ShudOutputDecl *decl, int max) {
    if (!h || !outdir) return fail(nullptr, "null argument");
    Project &p = *reinterpret_cast<Project *>(h);
    struct D { std::string sfx; int arr, col, n, dt, flux; };   // n: NumEle / NumRiv / NumLake control
    std::vector<D> v;
    const int NE = p.NE, NR = p.NR, NL = p.NL;
    auto add = [&](const char *sfx, int arr, int n, int dt, int flux, int col = -1) {
        v.push_back({sfx, arr, col, n, dt, flux});
    };
    if (p.dt_ye_ic > 0) add("eleyic", SHUD_ARR_Y_ELE_IS, NE, p.dt_ye_ic, 0);
    if (p.dt_ye_snow > 0) add("eleysnow", SHUD_ARR_Y_ELE_SNOW, NE, p.dt_ye_snow, 0);
    if (p.dt_ye_surf > 0) add("eleysurf", SHUD_ARR_Y_ELE_SURF, NE, p.dt_ye_surf, 0);
    if (p.dt_ye_unsat > 0) add("eleyunsat", SHUD_ARR_Y_ELE_UNSAT, NE, p.dt_ye_unsat, 0);
    if (p.dt_ye_gw > 0) add("eleygw", SHUD_ARR_Y_ELE_GW, NE, p.dt_ye_gw, 0);
    if (p.dt_qe_prcp > 0) add("elevprcp", SHUD_ARR_Q_PRCP, NE, p.dt_qe_prcp, 1);
    if (p.dt_qe_prcp > 0) add("elevnetprcp", SHUD_ARR_Q_NET_PRCP, NE, p.dt_qe_prcp, 1);
    if (p.dt_qe_etp > 0) add("elevetp", SHUD_ARR_Q_ETP, NE, p.dt_qe_etp, 1);
    if (p.dt_qe_eta > 0) add("eleveta", SHUD_ARR_Q_ETA, NE, p.dt_qe_eta, 1);
    if (p.dt_qe_rech > 0) add("elevrech", SHUD_ARR_Q_RECHARGE, NE, p.dt_qe_rech, 1);
    if (p.dt_Qe_sub > 0) add("eleqsub", SHUD_ARR_QELE_SUB_TOT, NE, p.dt_Qe_sub, 1);
    if (p.dt_Qe_subx > 0)                    // InitIJ with CS.dt_Qe_sub, as the reference passes it
        for (int j = 0; j < 3; j++) {
            static const char *nm[3] = {"eleqsub1", "eleqsub2", "eleqsub3"};
            add(nm[j], SHUD_ARR_QELE_SUB, NE, p.dt_Qe_sub, 1, j);
        }
    if (p.dt_Qe_surf > 0) add("eleqsurf", SHUD_ARR_QELE_SURF_TOT, NE, p.dt_Qe_surf, 1);
    if (p.dt_Qe_surfx > 0)
        for (int j = 0; j < 3; j++) {
            static const char *nm[3] = {"eleqsurf1", "eleqsurf2", "eleqsurf3"};
            add(nm[j], SHUD_ARR_QELE_SURF, NE, p.dt_Qe_surf, 1, j);
        }
    if (p.dt_Qe_rsub > 0) add("eleqrsub", SHUD_ARR_QE2R_SUB, NE, p.dt_Qe_rsub, 1);
    if (p.dt_Qe_rsurf > 0) add("eleqrsurf", SHUD_ARR_QE2R_SURF, NE, p.dt_Qe_rsurf, 1);
    if (p.dt_qe_infil > 0) {
        add("elevinfil", SHUD_ARR_Q_INFIL, NE, p.dt_qe_infil, 1);
        add("elevexfil", SHUD_ARR_Q_EXFIL, NE, p.dt_qe_infil, 1);
    }
    if (p.dt_qe_et > 0) {
        add("elevetic", SHUD_ARR_Q_E_IC, NE, p.dt_qe_et, 1);
        add("elevettr", SHUD_ARR_Q_TRANS, NE, p.dt_qe_et, 1);
        add("elevetev", SHUD_ARR_Q_EVAPO, NE, p.dt_qe_et, 1);
        add("rn_h", SHUD_ARR_RN_H, NE, p.dt_qe_et, 0);
        add("rn_t", SHUD_ARR_RN_T, NE, p.dt_qe_et, 0);
        add("rn_factor", SHUD_ARR_RN_FACTOR, NE, p.dt_qe_et, 0);
    }
    if (p.dt_Qr_up > 0) add("rivqup", SHUD_ARR_QRIV_UP, NR, p.dt_Qr_up, 1);
    if (p.dt_Qr_down > 0) add("rivqdown", SHUD_ARR_QRIV_DOWN, NR, p.dt_Qr_down, 1);
    if (p.dt_Qr_sub > 0) add("rivqsub", SHUD_ARR_QRIV_SUB, NR, p.dt_Qr_sub, 1);
    if (p.dt_Qr_surf > 0) add("rivqsurf", SHUD_ARR_QRIV_SURF, NR, p.dt_Qr_surf, 1);
    if (p.dt_yr_stage > 0) add("rivystage", SHUD_ARR_Y_RIV_STG, NR, p.dt_yr_stage, 0);
    if (p.dt_lake > 0 && NL > 0) {
        add("lakystage", SHUD_ARR_Y_LAKE_STG, NL, p.dt_lake, 0);
        add("lakatop", SHUD_ARR_LAKE_TOPAREA, NL, p.dt_lake, 0);
        add("lakvevap", SHUD_ARR_Q_LAKE_EVAP, NL, p.dt_lake, 1);
        add("lakvprcp", SHUD_ARR_Q_LAKE_PRCP, NL, p.dt_lake, 1);
        add("lakqrivin", SHUD_ARR_Q_LAKE_RIVIN, NL, p.dt_lake, 1);
        add("lakqrivout", SHUD_ARR_Q_LAKE_RIVOUT, NL, p.dt_lake, 1);
        add("lakqsurf", SHUD_ARR_Q_LAKE_SURF, NL, p.dt_lake, 1);
        add("lakqsub", SHUD_ARR_Q_LAKE_SUB, NL, p.dt_lake, 1);
    }
    p.out_names.clear();
    for (auto &d : v) p.out_names.push_back(std::string(outdir) + "/" + p.prj + "." + d.sfx);
    const int n = (int)v.size();
    for (int k = 0; k < n && k < max && decl; k++) {
        decl[k].basename = p.out_names[k].c_str();
        decl[k].array = v[k].arr;
        decl[k].column = v[k].col;
        decl[k].n_all = v[k].n;
        decl[k].interval = v[k].dt;
        decl[k].iflux = v[k].flux;
        // io_ele / io_riv / io_lake by the control's size, as initialize_output passes them
        const int a = v[k].arr;
        const bool lake = a == SHUD_ARR_Y_LAKE_STG || (a >= SHUD_ARR_LAKE_TOPAREA && a <= SHUD_ARR_Q_LAKE_SUB);
        const bool riv = a == SHUD_ARR_Y_RIV_STG || (a >= SHUD_ARR_QRIV_DOWN && a <= SHUD_ARR_QRIV_SUB);
        const std::vector<int32_t> &io = lake ? p.io_lake : riv ? p.io_riv : p.io_ele;
        bool all = true;
        for (int32_t f : io) all = all && f;
        decl[k].flag_io = all ? nullptr : io.data();
    }
    return n;
}

int shud_project_forcing(shud_project_t h, double t, double tout, ShudEtForcing *f) {
    if (!h || !f) return fail(nullptr, "null argument");
    return step_forcing(*reinterpret_cast<Project *>(h), t, tout, f);
}

int shud_project_bc_rows(shud_project_t h, ShudStepInputs *in) {
    if (!h || !in) return fail(nullptr, "null argument");
    Project &p = *reinterpret_cast<Project *>(h);
    const double **rows[4] = {&in->ele_ybc, &in->ele_qbc, &in->riv_ybc, &in->riv_qbc};
    int32_t *ns[4] = {&in->n_ele_ybc, &in->n_ele_qbc, &in->n_riv_ybc, &in->n_riv_qbc};
    int any = 0;
    for (int k = 0; k < 4; k++) {
        if (!p.have_bc[k]) continue;
        p.bc_row[k].assign(p.bc_w[k], 0.0);
        memcpy(p.bc_row[k].data(), p.bc[k].row(), p.bc[k].ncol * sizeof(double));
        *rows[k] = p.bc_row[k].data();
        *ns[k] = p.bc_w[k] - 1;                      // data columns (x[0] is the time column)
        any = 1;
    }
    return any;
}

int shud_project_solar(shud_project_t h, double t_min, double lat, double lon, double tz, double *out5) {
    if (!h || !out5) return fail(nullptr, "null argument");
    solar_position(*reinterpret_cast<Project *>(h), t_min, lat, lon, tz, true, out5);
    return 0;
}

}  // extern "C"
