"""Pure-Python restatement of the reference's solar geometry (test infrastructure: the checker of the C++ host's
TSR samples, include/shud_host.h).  Follows src/Equations/SolarRadiation.cpp:1-184 (solarPositionImpl and its
helpers) and src/classes/TimeContext.cpp (setBaseDate, toCivil, julianDay), and the TSR bucket sampling of
src/ModelData/MD_ET.cpp:86-133.  Python's math module calls the same glibc libm as the C++ host; a compiled
reference (g++ -O2/-O3) turns each sin(x)/cos(x) pair into one glibc sincos(x) call, whose cosine can differ
from cos(x) by an ulp, so the pairs here go through libm's sincos too."""
import ctypes
import math

_LIBM = ctypes.CDLL("libm.so.6")
_LIBM.sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
_LIBM.sincos.restype = None


def sincos(x):
    s, c = ctypes.c_double(), ctypes.c_double()
    _LIBM.sincos(float(x), ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value

K_PI = 3.141592653589793238462643383279502884
K_2PI = 2.0 * K_PI
K_D2R = K_PI / 180.0


def _cdiv(a, b):
    """C integer division (truncates toward zero)"""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _days_from_civil(y, m, d):
    y -= 1 if m <= 2 else 0
    era = _cdiv(y if y >= 0 else y - 399, 400)
    yoe = y - era * 400
    doy = (153 * (m + (-3 if m > 2 else 9)) + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def _civil_from_days(z):
    z += 719468
    era = _cdiv(z if z >= 0 else z - 146096, 146097)
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    y = yoe + era * 400
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = mp + (3 if mp < 10 else -9)
    return y + (1 if m <= 2 else 0), m, d


def _leap(y):
    return y % 4 == 0 and (y % 100 != 0 or y % 400 == 0)


def julian_day(base_yyyymmdd, t_min):
    y0, md = base_yyyymmdd // 10000, base_yyyymmdd % 10000
    base = _days_from_civil(y0, md // 100, md % 100)
    total = 0 if (math.isnan(t_min) or math.isinf(t_min)) else int(t_min)     # (long long) truncation
    day_off = _cdiv(total, 1440)
    mod = total - day_off * 1440
    if mod < 0:
        mod += 1440
        day_off -= 1
    y, m, d = _civil_from_days(base + day_off)
    cum = [0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334]
    doy = cum[m - 1] + d
    if m > 2 and _leap(y):
        doy += 1
    return doy


def _wrap1440(x):
    if not math.isfinite(x):
        return 0.0
    r = math.fmod(x, 1440.0)
    return r + 1440.0 if r < 0.0 else r


def solar_position(base_yyyymmdd, t_min, lat_deg, lon_deg, tz=0.0):
    """(cosZ, zenith, azimuth, declination, hourAngle) as solarPosition(t, lat, lon, Time, tz)."""
    lat = min(max(lat_deg, -90.0), 90.0) if math.isfinite(lat_deg) else 0.0
    lon = 0.0
    if math.isfinite(lon_deg):
        lon = math.fmod(lon_deg, 360.0)
        if lon > 180.0:
            lon -= 360.0
        elif lon < -180.0:
            lon += 360.0
    doy = julian_day(base_yyyymmdd, t_min)
    if doy < 1 or doy > 366:
        doy = 1
    mod_min = _wrap1440(t_min)
    hour = mod_min / 60.0
    gamma = (K_2PI / 365.0) * (float(doy - 1) + (hour - 12.0) / 24.0)
    sg, cg = sincos(gamma)
    s2, c2 = sincos(2.0 * gamma)
    s3, c3 = sincos(3.0 * gamma)
    eqt = 229.18 * (0.000075 + 0.001868 * cg - 0.032077 * sg - 0.014615 * c2 - 0.040849 * s2)
    decl = 0.006918 - 0.399912 * cg + 0.070257 * sg - 0.006758 * c2 + 0.000907 * s2 - 0.002697 * c3 + 0.00148 * s3
    tst = _wrap1440(mod_min + (eqt + 4.0 * lon - 60.0 * tz))
    ha = (tst / 4.0 - 180.0) * K_D2R
    lr = lat * K_D2R
    sl, cl = sincos(lr)
    sd, cd = sincos(decl)
    sh, ch = sincos(ha)
    cosz = min(max(sl * sd + cl * cd * ch, -1.0), 1.0)
    zen = math.acos(min(max(cosz, -1.0), 1.0))
    az = math.atan2(-cd * sh, cl * sd - sl * cd * ch)
    az = math.fmod(az, K_2PI)
    if az < 0.0:
        az += K_2PI
    return cosz, zen, az, decl, ha


def tsr_samples(base_yyyymmdd, t0, t1, dt_int_min, lat, lon):
    """MD_ET.cpp:86-133: solar samples (sx, sy, sz, wdt) of the forcing interval [t0, t1) and their sum."""
    dt_forc = t1 - t0
    dt_int = float(dt_int_min)
    if dt_int > dt_forc:
        dt_int = dt_forc
    n = max(1, int(math.ceil(dt_forc / dt_int)))
    dt_seg = dt_forc / float(n)
    sx, sy, sz, wd = [0.0] * n, [0.0] * n, [0.0] * n, [0.0] * n
    den = 0.0
    for k in range(n):
        tk = t0 + (k + 0.5) * dt_seg
        cosz, _, az, _, _ = solar_position(base_yyyymmdd, tk, lat, lon, 0.0)
        if not (cosz > 0.0) or not math.isfinite(cosz) or not math.isfinite(az):
            continue
        cc = min(1.0, max(-1.0, cosz))
        sinz = math.sqrt(max(0.0, 1.0 - cc * cc))
        w = max(0.0, cc) * dt_seg
        if not (w > 0.0) or not math.isfinite(w):
            continue
        sa, ca = sincos(az)
        sx[k], sy[k], sz[k], wd[k] = sinz * sa, sinz * ca, cc, w
        den += w
    return sx, sy, sz, wd, den
