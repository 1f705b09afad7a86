// shud_host_impl.hpp — internal types of libshud_host (include/shud_host.h).
#pragma once
#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

#include "shud_host.h"

namespace shudhost {

// TabularData (src/classes/TabularData.cpp:27-55): "nrow ncol", a header line, nrow rows of ncol numbers
// parsed with strtold (an unparsable token leaves the pointer in place, so it and the rest of the row read 0)
struct Table {
    int nrow = 0, ncol = 0;
    std::string header;
    std::vector<double> x;                       // row-major [nrow][ncol]
    double at(int r, int c) const { return x[(size_t)r * ncol + c]; }
};

// _TimeSeriesData (src/classes/TimeSeriesData.cpp): rows read once in full (the reference streams MAXQUE-row
// chunks through a ring; for a monotonic time column the row it exposes is the same zero-order hold)
struct Series {
    std::string fn;
    int ncol = 0;                                // incl. the time column (minutes after read)
    long start_date = 0;                         // third header field ("nrow ncol yyyymmdd")
    std::vector<double> ts;                      // [n][ncol]
    int64_t n = 0, now = 0;
    double lon = -9999.0, lat = -9999.0, xyz[3] = {0, 0, 0};
    const double *row() const { return &ts[(size_t)now * ncol]; }
    double t_now() const { return ts[(size_t)now * ncol]; }
    // nextTimeMin: the ring slot after iNow; past the last row it never exceeds t_now (stale or duplicate)
    double t_next() const { return now + 1 < n ? ts[(size_t)(now + 1) * ncol] : -1.0e300; }
};

struct Project {
    std::string prj, indir, err;
    ShudControl ctl{};
    // print-control intervals (PrintOutDt, Model_Control.hpp:116-147) and calibration (globalCal)
    int dt_ye_gw = 0, dt_ye_surf = 0, dt_ye_snow = 0, dt_ye_ic = 0, dt_ye_unsat = 0;
    int dt_qe_prcp = 1440, dt_qe_infil = 0, dt_qe_et = 0, dt_qe_rech = 0, dt_qe_etp = 0, dt_qe_eta = 0;
    int dt_Qe_sub = 0, dt_Qe_subx = 0, dt_Qe_surf = 0, dt_Qe_surfx = 0, dt_Qe_rsub = 0, dt_Qe_rsurf = 0;
    int dt_yr_stage = 0, dt_Qr_up = 0, dt_Qr_down = 0, dt_Qr_sub = 0, dt_Qr_surf = 0, dt_lake = 1440;
    std::map<std::string, double> cal;           // globalCal keys (upper case) -> value, defaults applied
    double fz_sub_max = -3, fz_sub_min = -10, fz_sub_day = 28, fz_surf_max = -1, fz_surf_min = -5, fz_surf_day = 7;
    double solar_lon_fixed = -9999.0, solar_lat_fixed = -9999.0;

    int NE = 0, NR = 0, NS = 0, NL = 0, NumNode = 0, NumLC = 0;
    // mesh SoA (ShudMeshSoA), params (ShudParamsSoA), ET statics (ShudEtMeshSoA)
    std::vector<int32_t> nabr, ibc, iss, ilake, riv_down, riv_bc, seg_ele, seg_riv, bathy_off;
    std::vector<double> area, z_surf, z_bottom, depression, edge, d2n, d2e, avg_rough, rough;
    std::vector<double> riv_length, riv_slope, riv_d2d, riv_avg_rough, riv_depth, riv_bw, riv_bs, riv_ksath,
        riv_bedthick, seg_length, seg_cwr, bathy_y, bathy_a;
    std::vector<double> aq, macD, macKsatH, vAreaF, KsatH, KsatV, infKsatV, hAreaF, macKsatV, ThetaS, ThetaR,
        Beta, infD, Sy, RzD, VegFrac, ImpAF;
    std::vector<int32_t> iforc, ilc, imf;
    std::vector<double> albedo, fixp, windh, nx, ny, nz, cx, cy, slope_angle, aspect;
    std::vector<double> y0, y_is, y_snow;
    // forcing
    std::vector<Series> wx;
    Series lai, mf;
    bool have_lai = false, have_mf = false;
    // boundary-condition series (tsd.ebc1 / ebc2 / rbc1 / rbc2) and their padded rows, and cfg.output flags
    Series bc[4];
    bool have_bc[4] = {false, false, false, false};
    int bc_w[4] = {0, 0, 0, 0};
    std::vector<double> bc_row[4];
    std::vector<int32_t> io_ele, io_riv, io_lake;
    // TSR bucket (MD_ET.cpp:60-136)
    long long tsr_bucket = -1;
    double tsr_t0 = 0, tsr_t1 = 0;
    int tsr_dtint = 0, tsr_n = 0;
    double tsr_den = 0;
    std::vector<double> tsr_sx, tsr_sy, tsr_sz, tsr_wdt;
    // per-step scratch for shud_project_forcing
    std::vector<double> st_rows, st_z, lai_row, mf_row;
    int lai_w = 0, mf_w = 0;                     // row widths handed to the device (>= every iLC / iMF + 1)
    // TimeContext base date
    long long base_days = 0;
    bool base_ok = false;
    std::vector<std::string> out_names;
};

int fail(Project *p, const char *fmt, ...);
bool read_table(FILE *fp, Table &t);
int load(Project &p, const char *indir, const char *prj, const char *cwd, double end_day);
int read_forcing(Project &p, const char *cwd);
int step_forcing(Project &p, double t, double tout, ShudEtForcing *f);
int read_bc(Project &p);
int read_series_file(Project &p, Series &s);
int move_series(Project &p, Series &s, double t);
void solar_position(const Project &p, double t_min, double lat_deg, double lon_deg, double tz, bool tz_given,
                    double out[5]);

}  // namespace shudhost
