// shud_forcing.cpp — forcing time series, LAI/MF series and the TSR solar samples for the device ET prelude
// (include/shud_host.h shud_project_forcing).  Restates the reference's host side of tReadForcing:
//   read_forc (CSV list)            src/ModelData/MD_readin.cpp:555-729 (+ solar lon/lat selection :645-690)
//   _TimeSeriesData                 src/classes/TimeSeriesData.cpp (read_csv, movePointer, getX, *TimeMin)
//   updateAllTimeSeries             src/ModelData/MD_update.cpp:3-40
//   TSR forcing-interval bucket     src/ModelData/MD_ET.cpp:60-136
//   solarPosition / TimeContext     src/Equations/SolarRadiation.cpp:1-184, src/classes/TimeContext.cpp
#include <strings.h>
#include <sys/stat.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>

#include "shud_host_impl.hpp"

namespace shudhost {

static constexpr int kMaxLen = 2048;             // MAXLEN (Macros.hpp:30)
static constexpr int kNforc = 5;                  // Nforc (Macros.hpp:37): prcp, temp, rh, wind, rn

static bool exists(const std::string &f) {
    struct stat st;
    return stat(f.c_str(), &st) == 0;
}

// _TimeSeriesData::read_csv (TimeSeriesData.cpp:161-238) for the whole file: 2 header lines, then rows
// "time_day v1 .. v(ncol-1)" parsed with istream >> double; '#' and blank lines skipped; time -> minutes.
static int read_series(Project &p, Series &s) {
    std::ifstream file(s.fn);
    if (!file.is_open()) return fail(&p, "Fatal Error: %s is in use or does not exist!", s.fn.c_str());
    std::string line;
    std::getline(file, line);
    std::getline(file, line);
    long lineNo = 2;
    double prev = 0.0;
    bool has = false;
    s.ts.clear();
    while (std::getline(file, line)) {
        lineNo++;
        const size_t first = line.find_first_not_of(" \t\r\n");
        if (first == std::string::npos || line[first] == '#') continue;
        std::istringstream iss(line);
        double day = 0.0;
        if (!(iss >> day)) return fail(&p, "Fatal Error: Failed to parse time value. File: %s Line: %ld", s.fn.c_str(), lineNo);
        const double tmin = day * 1440.0;
        if (has && tmin + 1e-12 < prev)
            return fail(&p, "Fatal Error: Time column is not monotonic non-decreasing. File: %s Line: %ld", s.fn.c_str(), lineNo);
        s.ts.push_back(tmin);
        for (int j = 1; j < s.ncol; j++) {
            double v;
            if (!(iss >> v))
                return fail(&p, "Fatal Error: Failed to parse numeric column %d. File: %s Line: %ld", j + 1, s.fn.c_str(), lineNo);
            s.ts.push_back(v);
        }
        has = true;
        prev = tmin;
    }
    s.n = (int64_t)(s.ts.size() / s.ncol);
    s.now = 0;
    if (s.n <= 0) return fail(&p, "Reading fail, file = %s", s.fn.c_str());
    return 0;
}

// readDimensions (TimeSeriesData.cpp:239-249): "%d %d %ld" -> ncol, StartTime
static int read_dims(Project &p, Series &s) {
    FILE *fp = fopen(s.fn.c_str(), "r");
    if (!fp) return fail(&p, "Fatal Error: %s is in use or does not exist!", s.fn.c_str());
    int tmp = 0, nc = 0;
    long st = 0;
    const int k = fscanf(fp, "%d %d %ld", &tmp, &nc, &st);
    fclose(fp);
    if (k < 2 || nc < 1) return fail(&p, "bad time-series header in %s", s.fn.c_str());
    s.ncol = nc;
    s.start_date = st;
    return 0;
}

// _TimeSeriesData::movePointer (TimeSeriesData.cpp:285-307): advance while the next row's time <= t; past the
// last row with t more than a day beyond it the reference exits ("missing forcing data").
static int move_pointer(Project &p, Series &s, double t) {
    while (s.now + 1 < s.n && t >= s.ts[(size_t)(s.now + 1) * s.ncol] &&
           s.ts[(size_t)(s.now + 1) * s.ncol] >= s.t_now())
        s.now++;
    const double tn = s.t_now();
    if (s.now + 1 >= s.n && t - tn > 1 && tn + 1440 < t)
        return fail(&p, "Error in reading file: %s  Error: missing forcing data after t=%.3lf", s.fn.c_str(), tn / 1440. + 1);
    return 0;
}

// TimeContext (TimeContext.cpp): days_from_civil / civil_from_days (Howard Hinnant's algorithms, as written)
static long long days_from_civil(int y, unsigned m, unsigned d) {
    y -= m <= 2;
    const int era = (y >= 0 ? y : y - 399) / 400;
    const unsigned yoe = (unsigned)(y - era * 400);
    const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return (long long)era * 146097 + (long long)doe - 719468;
}
static void civil_from_days(long long z, int &y, unsigned &m, unsigned &d) {
    z += 719468;
    const long long era = (z >= 0 ? z : z - 146096) / 146097;
    const unsigned doe = (unsigned)(z - era * 146097);
    const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    y = (int)(yoe) + (int)(era * 400);
    const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const unsigned mp = (5 * doy + 2) / 153;
    d = doy - (153 * mp + 2) / 5 + 1;
    m = mp + (mp < 10 ? 3 : -9);
    y += (m <= 2);
}
static bool leap(int y) { return (y % 4) == 0 && ((y % 100) != 0 || (y % 400) == 0); }
static int days_in_month(int y, unsigned m) {
    static const int dim[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    if (m < 1 || m > 12) return 0;
    return (m == 2 && leap(y)) ? 29 : dim[m - 1];
}
static void set_base_date(Project &p, long yyyymmdd) {       // TimeContext::setBaseDate
    p.base_ok = false;
    p.base_days = 0;
    if (yyyymmdd <= 0) return;
    const int y = (int)(yyyymmdd / 10000);
    const long md = yyyymmdd % 10000;
    const unsigned m = (unsigned)(md / 100), d = (unsigned)(md % 100);
    if (m < 1 || m > 12) return;
    const int dim = days_in_month(y, m);
    if (dim <= 0 || d < 1 || (int)d > dim) return;
    p.base_ok = true;
    p.base_days = days_from_civil(y, m, d);
}
static int julian_day(const Project &p, double t_min) {      // TimeContext::julianDay via toCivil
    if (!p.base_ok) return 0;
    long long total = 0;
    if (!std::isnan(t_min) && !std::isinf(t_min)) total = (long long)t_min;
    long long day_off = total / 1440, mod = total % 1440;
    if (mod < 0) { mod += 1440; day_off -= 1; }
    int y; unsigned m, d;
    civil_from_days(p.base_days + day_off, y, m, d);
    if (y == 0 || m == 0 || d == 0) return 0;
    static const int cum[12] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334};
    if (m < 1 || m > 12) return 0;
    int doy = cum[m - 1] + (int)d;
    if (m > 2 && leap(y)) doy += 1;
    return doy;
}

// solarPositionImpl (SolarRadiation.cpp:92-176) and its helpers (:1-91)
void solar_position(const Project &p, double t_min, double lat_deg, double lon_deg, double tz, bool tz_given,
                    double out[5]) {
    constexpr double kPi = 3.141592653589793238462643383279502884;
    constexpr double kTwoPi = 2.0 * kPi;
    constexpr double kDeg2Rad = kPi / 180.0;
    auto fin = [](double x) { return std::isfinite(x) != 0; };
    auto clamp = [](double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); };
    auto wrap1440 = [&](double m) {
        if (!fin(m)) return 0.0;
        double r = std::fmod(m, 1440.0);
        if (r < 0.0) r += 1440.0;
        return r;
    };
    double cosZ = 0.0, zen = kPi / 2.0, az = 0.0, decl_o = 0.0, ha_o = 0.0;
    const double lat = fin(lat_deg) ? clamp(lat_deg, -90.0, 90.0) : 0.0;
    double lon = 0.0;
    if (fin(lon_deg)) {
        lon = std::fmod(lon_deg, 360.0);
        if (lon > 180.0) lon -= 360.0;
        else if (lon < -180.0) lon += 360.0;
    }
    if (!tz_given || !fin(tz)) tz = fin(lon) ? std::round(lon / 15.0) : 0.0;
    int doy = julian_day(p, t_min);
    if (doy < 1 || doy > 366) doy = 1;
    const double mod_min = wrap1440(t_min);
    const double hour = mod_min / 60.0;
    const double gamma = (kTwoPi / 365.0) * (static_cast<double>(doy - 1) + (hour - 12.0) / 24.0);
    const double sin_g = std::sin(gamma), cos_g = std::cos(gamma);
    const double sin_2g = std::sin(2.0 * gamma), cos_2g = std::cos(2.0 * gamma);
    const double sin_3g = std::sin(3.0 * gamma), cos_3g = std::cos(3.0 * gamma);
    const double eq_time_min =
        229.18 * (0.000075 + 0.001868 * cos_g - 0.032077 * sin_g - 0.014615 * cos_2g - 0.040849 * sin_2g);
    const double decl = 0.006918 - 0.399912 * cos_g + 0.070257 * sin_g - 0.006758 * cos_2g + 0.000907 * sin_2g -
                        0.002697 * cos_3g + 0.00148 * sin_3g;
    decl_o = decl;
    const double time_offset_min = eq_time_min + 4.0 * lon - 60.0 * tz;
    const double tst = wrap1440(mod_min + time_offset_min);
    const double ha_deg = tst / 4.0 - 180.0;
    const double ha = ha_deg * kDeg2Rad;
    ha_o = ha;
    const double lat_rad = lat * kDeg2Rad;
    const double sin_lat = std::sin(lat_rad), cos_lat = std::cos(lat_rad);
    const double sin_decl = std::sin(decl), cos_decl = std::cos(decl);
    const double sin_ha = std::sin(ha), cos_ha = std::cos(ha);
    const double cosz_raw = sin_lat * sin_decl + cos_lat * cos_decl * cos_ha;
    cosZ = clamp(cosz_raw, -1.0, 1.0);
    zen = std::acos(clamp(cosZ, -1.0, 1.0));
    const double east = -cos_decl * sin_ha;
    const double north = cos_lat * sin_decl - sin_lat * cos_decl * cos_ha;
    const double a = std::atan2(east, north);
    if (fin(a)) {
        az = std::fmod(a, kTwoPi);
        if (az < 0.0) az += kTwoPi;
    } else {
        az = 0.0;
    }
    if (!fin(cosZ) || !fin(zen) || !fin(az) || !fin(decl_o) || !fin(ha_o)) {
        cosZ = 0.0; zen = kPi / 2.0; az = 0.0; decl_o = 0.0; ha_o = 0.0;
    }
    out[0] = cosZ; out[1] = zen; out[2] = az; out[3] = decl_o; out[4] = ha_o;
}

// read_forc (MD_readin.cpp:555-729), read_lai / read_mf (:942-951)
int read_forcing(Project &p, const char *cwd) {
    const std::string fn = p.indir + "/" + p.prj + ".tsd.forc";
    FILE *fp = fopen(fn.c_str(), "r");
    if (!fp) return fail(&p, "Fatal Error: %s is in use or does not exist!", fn.c_str());
    char str[kMaxLen], path[kMaxLen] = "", shortname[kMaxLen];
    int nforc = 0;
    long fst = 0;
    if (!fgets(str, kMaxLen, fp) || sscanf(str, "%d %ld", &nforc, &fst) != 2 || nforc <= 0) {
        fclose(fp);
        return fail(&p, "Fatal Error: invalid forcing list header in %s (Expected: <NumForc> <ForcStartTime>)", fn.c_str());
    }
    p.ctl.num_forc = nforc;
    p.ctl.forc_start_time = fst;
    set_base_date(p, fst);
    if (!fgets(str, kMaxLen, fp)) { fclose(fp); return fail(&p, "Fatal Error: forcing list file missing path line: %s", fn.c_str()); }
    if (strlen(str) > 1) sscanf(str, "%s", path);
    if (!fgets(str, kMaxLen, fp)) { fclose(fp); return fail(&p, "Fatal Error: forcing list file missing header line: %s", fn.c_str()); }
    p.wx.assign(nforc, Series{});
    for (int i = 0; i < nforc;) {
        if (!fgets(str, kMaxLen, fp)) {
            fclose(fp);
            return fail(&p, "Fatal Error: forcing list file %s ended early (expected %d records, got %d)", fn.c_str(), nforc, i);
        }
        const char *q = str;
        while (*q == ' ' || *q == '\t' || *q == '\r' || *q == '\n') q++;
        if (*q == '\0' || *q == '#') continue;
        int id;
        double lon = -9999.0, lat = -9999.0;
        Series &s = p.wx[i];
        if (sscanf(str, "%d %lf %lf %lf %lf %lf %s", &id, &lon, &lat, s.xyz, s.xyz + 1, s.xyz + 2, shortname) != 7) {
            fclose(fp);
            return fail(&p, "Fatal Error: invalid forcing record in %s (Expected: ID Lon Lat X Y Z Filename)", fn.c_str());
        }
        s.lon = lon;
        s.lat = lat;
        // the reference opens "<path>/<file>" relative to its working directory; here relative to `cwd`
        // (default: the process cwd), then the project directory as a fallback
        std::string full = strlen(path) ? std::string(path) + "/" + shortname : std::string(shortname);
        std::string cand = (cwd && full[0] != '/') ? std::string(cwd) + "/" + full : full;
        if (!exists(cand)) cand = p.indir + "/" + shortname;
        s.fn = cand;
        s.ncol = kNforc + 1;
        i++;
    }
    fclose(fp);
    // solar lon/lat (MD_readin.cpp:645-690)
    ShudControl &c = p.ctl;
    c.solar_lon_deg = -9999.0;
    c.solar_lat_deg = -9999.0;
    if (c.solar_lonlat_mode == 2) {
        c.solar_lon_deg = p.solar_lon_fixed;
        c.solar_lat_deg = p.solar_lat_fixed;
        if (c.solar_lon_deg == -9999.0 || c.solar_lat_deg == -9999.0)
            return fail(&p, "Fatal Error: SOLAR_LONLAT_MODE=FIXED but SOLAR_LON_DEG/SOLAR_LAT_DEG is missing.");
    } else if (c.solar_lonlat_mode == 1) {
        double slo = 0.0, sla = 0.0;
        int n = 0;
        for (auto &s : p.wx) {
            if (s.lon == -9999.0 || s.lat == -9999.0) continue;
            if (s.lon < -180.0 || s.lon > 180.0 || s.lat < -90.0 || s.lat > 90.0) continue;
            slo += s.lon; sla += s.lat; n++;
        }
        if (n > 0) { c.solar_lon_deg = slo / n; c.solar_lat_deg = sla / n; }
    } else {
        c.solar_lon_deg = p.wx[0].lon;
        c.solar_lat_deg = p.wx[0].lat;
    }
    if (c.solar_lon_deg == -9999.0 || c.solar_lat_deg == -9999.0)
        return fail(&p, "Fatal Error: SOLAR_LONLAT_MODE selected Lon/Lat is missing");
    if (c.solar_lon_deg < -180.0 || c.solar_lon_deg > 180.0 || c.solar_lat_deg < -90.0 || c.solar_lat_deg > 90.0)
        return fail(&p, "Fatal Error: invalid solar Lon/Lat selected (lon=%.6f, lat=%.6f)", c.solar_lon_deg, c.solar_lat_deg);
    int rc;
    for (auto &s : p.wx)
        if ((rc = read_series(p, s))) return rc;
    p.lai.fn = p.indir + "/" + p.prj + ".tsd.lai";
    if ((rc = read_dims(p, p.lai)) || (rc = read_series(p, p.lai))) return rc;
    p.have_lai = true;
    p.mf.fn = p.indir + "/" + p.prj + ".tsd.mf";
    if ((rc = read_dims(p, p.mf)) || (rc = read_series(p, p.mf))) return rc;
    p.have_mf = true;
    // element indices into the series (iForc, iLC, iMF).  tsd_LAI.getX(t, iLC) / tsd_MF.getX(t, iMF) index the
    // row without a bound check (TimeSeriesData.cpp:270-273): a column past the table (heihe: iLC 13, 14 of a
    // 12-column LAI table) reads whatever follows the row on the reference's heap.  Here such columns read 0
    // (the rows handed to the device are padded), with a warning.
    p.lai_w = p.lai.ncol;
    p.mf_w = p.mf.ncol;
    for (int i = 0; i < p.NE; i++) {
        if (p.iforc[i] < 0 || p.iforc[i] >= nforc) return fail(&p, "element %d: forcing station %d out of range", i + 1, p.iforc[i] + 1);
        if (p.ilc[i] < 0 || p.imf[i] < 0) return fail(&p, "element %d: negative LAI/MF column", i + 1);
        if (p.ilc[i] >= p.lai_w) p.lai_w = p.ilc[i] + 1;
        if (p.imf[i] >= p.mf_w) p.mf_w = p.imf[i] + 1;
    }
    if (p.lai_w > p.lai.ncol)
        fprintf(stderr, "WARNING: %s has %d columns but elements use LAI column %d; the reference reads past the row "
                "(undefined), here those columns read 0\n", p.lai.fn.c_str(), p.lai.ncol, p.lai_w - 1);
    if (p.mf_w > p.mf.ncol)
        fprintf(stderr, "WARNING: %s has %d columns but elements use MF column %d; the reference reads past the row "
                "(undefined), here those columns read 0\n", p.mf.fn.c_str(), p.mf.ncol, p.mf_w - 1);
    if (p.ctl.terrain_radiation && nforc > 1) {
        // the device prelude takes one set of solar samples per step: every station must share one time column
        for (int k = 1; k < nforc; k++)
            if (p.wx[k].ts.size() / p.wx[k].ncol != p.wx[0].ts.size() / p.wx[0].ncol)
                return fail(&p, "TERRAIN_RADIATION with forcing stations on different time columns is not supported");
    }
    return 0;
}

int read_series_file(Project &p, Series &s) {
    int rc = read_dims(p, s);
    return rc ? rc : read_series(p, s);
}
int move_series(Project &p, Series &s, double t) { return move_pointer(p, s, t); }

// read_bcEle1/2, read_bcRiv1/2 (MD_readin.cpp:959-982) when the mesh references them (ieBC1/2, irBC1/2)
int read_bc(Project &p) {
    static const char *ext[4] = {"tsd.ebc1", "tsd.ebc2", "tsd.rbc1", "tsd.rbc2"};
    int maxc[4] = {0, 0, 0, 0};
    for (int i = 0; i < p.NE; i++) {
        if (p.ibc[i] > 0) maxc[0] = std::max(maxc[0], p.ibc[i]);
        if (p.ibc[i] < 0) maxc[1] = std::max(maxc[1], -p.ibc[i]);
    }
    for (int r = 0; r < p.NR; r++) {
        if (p.riv_bc[r] > 0) maxc[2] = std::max(maxc[2], p.riv_bc[r]);
        if (p.riv_bc[r] < 0) maxc[3] = std::max(maxc[3], -p.riv_bc[r]);
    }
    for (int k = 0; k < 4; k++) {
        if (!maxc[k]) continue;
        p.bc[k].fn = p.indir + "/" + p.prj + "." + ext[k];
        if (int rc = read_series_file(p, p.bc[k])) return rc;
        p.have_bc[k] = true;
        // getX(t, col) reads ts[iNow][col] unchecked: columns past the table read 0 here (warning)
        p.bc_w[k] = std::max(p.bc[k].ncol, maxc[k] + 1);
        if (p.bc_w[k] > p.bc[k].ncol)
            fprintf(stderr, "WARNING: %s has %d columns but column %d is referenced; those read 0 here\n",
                    p.bc[k].fn.c_str(), p.bc[k].ncol, maxc[k]);
    }
    return 0;
}

// One ET step: updateAllTimeSeries(t) (MD_update.cpp:3-40) and the shared part of tReadForcing (MD_ET.cpp:21-136)
int step_forcing(Project &p, double t, double tout, ShudEtForcing *f) {
    int rc;
    for (auto &s : p.wx)
        if ((rc = move_pointer(p, s, t))) return rc;
    if (p.NumLC > 0 && (rc = move_pointer(p, p.lai, t))) return rc;
    if (p.mf.ncol > 0 && (rc = move_pointer(p, p.mf, t))) return rc;
    for (int k = 0; k < 4; k++)                                        // tsd_eyBC .. tsd_rqBC (MD_update.cpp:25-40)
        if (p.have_bc[k] && (rc = move_pointer(p, p.bc[k], t))) return rc;
    const int ns = (int)p.wx.size();
    p.st_rows.resize((size_t)ns * 6);
    p.st_z.resize(ns);
    for (int k = 0; k < ns; k++) {
        memcpy(&p.st_rows[(size_t)k * 6], p.wx[k].row(), 6 * sizeof(double));
        p.st_z[k] = p.wx[k].xyz[2];
    }
    memset(f, 0, sizeof *f);
    f->t = t;
    f->t_next = tout;
    f->n_station = ns;
    f->station = p.st_rows.data();
    f->station_z = p.st_z.data();
    p.lai_row.assign(p.lai_w, 0.0);
    memcpy(p.lai_row.data(), p.lai.row(), p.lai.ncol * sizeof(double));
    p.mf_row.assign(p.mf_w, 0.0);
    memcpy(p.mf_row.data(), p.mf.row(), p.mf.ncol * sizeof(double));
    f->n_lai_col = p.lai_w;
    f->lai_row = p.lai_row.data();
    f->n_mf_col = p.mf_w;
    f->mf_row = p.mf_row.data();
    f->tsr_mode = SHUD_TSR_OFF;
    if (!p.ctl.terrain_radiation) return 0;
    // every station shares the forcing interval (checked at load): the bucket of station 0 is every element's
    const double t0 = p.wx[0].t_now();
    double t1 = p.wx[0].t_next();
    if (!std::isfinite(t0)) {
        f->tsr_mode = SHUD_TSR_NO_TIME;
        return 0;
    }
    if (!std::isfinite(t1) || !(t1 > t0)) t1 = t0 + p.ctl.solver_step;
    int dt_int_min = p.ctl.tsr_integration_step_min;
    if (dt_int_min <= 0) dt_int_min = 60;
    if (p.tsr_bucket < 0 || t0 != p.tsr_t0 || t1 != p.tsr_t1 || dt_int_min != p.tsr_dtint) {
        p.tsr_bucket += 1;
        p.tsr_t0 = t0;
        p.tsr_t1 = t1;
        p.tsr_dtint = dt_int_min;
        const double dt_forc = t1 - t0;
        double dt_int = (double)dt_int_min;
        if (dt_int > dt_forc) dt_int = dt_forc;
        int n = (int)std::ceil(dt_forc / dt_int);
        if (n < 1) n = 1;
        p.tsr_n = n;
        const double dt_seg = dt_forc / (double)n;
        p.tsr_sx.assign(n, 0.0); p.tsr_sy.assign(n, 0.0); p.tsr_sz.assign(n, 0.0); p.tsr_wdt.assign(n, 0.0);
        p.tsr_den = 0.0;
        for (int k = 0; k < n; k++) {
            const double tk = t0 + (k + 0.5) * dt_seg;
            double sp[5];
            solar_position(p, tk, p.ctl.solar_lat_deg, p.ctl.solar_lon_deg, 0.0, true, sp);
            const double cosz = sp[0];
            if (!(cosz > 0.0) || !std::isfinite(cosz) || !std::isfinite(sp[2])) continue;
            const double cc = std::min(1.0, std::max(-1.0, cosz));
            const double sinz = std::sqrt(std::max(0.0, 1.0 - cc * cc));
            const double sin_az = std::sin(sp[2]), cos_az = std::cos(sp[2]);
            const double wdt = std::max(0.0, cc) * dt_seg;
            if (!(wdt > 0.0) || !std::isfinite(wdt)) continue;
            p.tsr_sx[k] = sinz * sin_az;
            p.tsr_sy[k] = sinz * cos_az;
            p.tsr_sz[k] = cc;
            p.tsr_wdt[k] = wdt;
            p.tsr_den += wdt;
        }
        f->tsr_mode = SHUD_TSR_RECOMPUTE;
    } else {
        f->tsr_mode = SHUD_TSR_CACHED;
    }
    f->tsr_n = p.tsr_n;
    f->tsr_sx = p.tsr_sx.data();
    f->tsr_sy = p.tsr_sy.data();
    f->tsr_sz = p.tsr_sz.data();
    f->tsr_wdt = p.tsr_wdt.data();
    f->tsr_den = p.tsr_den;
    return 0;
}

}  // namespace shudhost
