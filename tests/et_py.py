"""Pure-Python restatement of the ET-step prelude (TEST INFRASTRUCTURE: second, independent restatement used to
check oracle/shud_oracle_et.c bit for bit on small cases).  Follows src/ModelData/MD_ET.cpp:21-341 line by
line with Python's math (glibc libm, like the reference build).  Elementwise loops: small meshes only."""
import math

import numpy as np

ZERO, NA = 1e-10, -9999.0


def rmin(a, b):
    return b if a > b else a


def rmax(a, b):
    return b if a < b else a


def frozen(T, high, low):                   # functions.hpp:191-201
    if T > high:
        return 0.
    if T < low:
        return 1.
    return rmin(1.0, rmax((high - T) / (high - low), 0.0))


class PyAcc:                                # AccTemperature.hpp
    def __init__(self, maxlen):
        self.ts, self.tacc, self.n, self.acc, self.q, self.maxlen = -9999., 0., 0, 0., [], maxlen

    def push(self, x, tnow):
        self.tacc += x
        self.n += 1
        if (tnow - self.ts) >= 1440.:
            v = self.tacc / self.n
            self.q.append(v)
            self.acc += v
            if len(self.q) > self.maxlen:
                self.acc -= self.q.pop(0)
            self.tacc, self.n, self.ts = 0., 0, tnow

    def get(self):
        return self.acc / len(self.q) if self.q else float("nan")


class PyEt:
    def __init__(self, etm):
        self.a = {k: (None if v is None else np.asarray(v)) for k, v in etm.arrays.items()}
        self.p = dict(etm.params)
        n = etm.num_ele
        self.n = n
        self.y_is, self.y_snow = np.zeros(n), np.zeros(n)
        self.factor_cache = [None] * n
        self.acc_s = [PyAcc(self.p["ft_surf_day"]) for _ in range(n)]
        self.acc_g = [PyAcc(self.p["ft_sub_day"]) for _ in range(n)]
        self.out = {}

    def step(self, f):
        a, p, n = self.a, self.p, self.n
        o = {k: np.zeros(n) for k in ["t_prcp", "t_temp", "t_lai", "t_mf", "t_rn", "t_wind", "t_rh", "qEleprep",
                                      "qPotEvap", "qPotTran", "qEleETP", "qEleNetPrep", "qEleE_IC", "fu_surf",
                                      "fu_sub", "rn_factor"]}
        for i in range(n):                                      # tReadForcing, MD_ET.cpp:21-281
            row = f.station[a["iforc"][i]]
            prcp = row[1] * p["cPrep"]
            zt = f.station_z[a["iforc"][i]]
            zi = a["z_surf"][i]
            t0 = row[2]
            temp = (t0 if (abs(zi - NA) < ZERO or abs(zt - NA) < ZERO) else t0 + (zt - zi) * 0.0065) + p["cTemp"]
            lai = f.lai_row[a["ilc"][i]] * p["cLAItsd"]
            mf = f.mf_row[a["imf"][i]] * p["cMF"] / 1440.
            dsw = row[5]
            factor = 1.0
            if p["terrain_radiation"]:
                if f.tsr_mode == 1:
                    factor = 0.0
                else:
                    if f.tsr_mode == 3 or self.factor_cache[i] is None:
                        num = 0.0
                        if f.tsr_den > 0.0 and f.tsr is not None and f.tsr.shape[1] > 0:
                            for k in range(f.tsr.shape[1]):
                                sx, sy, sz, w = f.tsr[:, k]
                                if not (w > 0.0):
                                    continue
                                cosi = a["nx"][i] * sx + a["ny"][i] * sy + a["nz"][i] * sz
                                if not (cosi > 0.0) or not math.isfinite(cosi):
                                    continue
                                den = p["rad_cosz_min"] if sz < p["rad_cosz_min"] else sz
                                if not (den > 0.0) or not math.isfinite(den):
                                    continue
                                fk = cosi / den
                                if not math.isfinite(fk) or not (fk > 0.0):
                                    continue
                                if fk > p["rad_factor_cap"]:
                                    fk = p["rad_factor_cap"]
                                num += w * fk
                        fe = 0.0
                        if f.tsr_den > 0.0:
                            fe = num / f.tsr_den
                            if not math.isfinite(fe) or not (fe > 0.0):
                                fe = 0.0
                            if fe > p["rad_factor_cap"]:
                                fe = p["rad_factor_cap"]
                        self.factor_cache[i] = fe
                    factor = self.factor_cache[i]
                dsw = dsw * factor
            rn = dsw if p["radiation_input_mode"] == 1 else dsw * (1 - a["albedo"][i])
            wind = abs(row[4]) + 0.001
            rh = row[3]
            prcp = prcp * 0.001 / 1440.
            rn = rn * 1.0e-6
            rh = rmin(rmax(rh, 0.01), 1.0)
            P = a["fix_pressure"][i]
            lam = 2.501 - 0.002361 * temp
            gam = 0.0016286 * P / lam
            es = 0.6108 * math.exp(17.27 * temp / (temp + 237.3))
            ed = es - es * rh
            tt = temp + 237.3
            delta = 4098. * es / (tt * tt)
            rho = 3.486 * P / (275. + temp)
            lake = a["ilake"][i] > 0
            G = 0. if lake else (0.4 * math.exp(-0.5 * lai) * rn if lai > 0 else 0.1 * rn)
            RG = rn - G
            U2 = wind * math.log((2.0 - 0.) / 0.00137) / math.log((a["wind_h"][i] - 0.) / 0.00137)
            pe = (delta * RG * 86400 + gam * 6.43 * (1.0 + 0.536 * U2) * ed) / (delta + gam)
            pe = pe / lam
            pe = pe * 0.001 / 86400
            qpet = p["cETP"] * pe * 60.
            if lake or lai <= 0.:
                qptr = p["cETP"] * 0.
                etp = qpet
            else:
                hc = lai * 0.5
                zm = hc * 1.3333
                d, zom, zov = 0.67 * hc, 0.123 * hc, 0.0123 * hc
                ra = math.log(abs(zm - d) / zom) * math.log(abs(zm - d) / zov) / (0.4 * 0.4 * wind)
                if ra <= 0.0 or math.isnan(ra) or math.isinf(ra) or abs(ra - NA) < ZERO:
                    return 10, i
                rs = 200. / lai
                e_air = rho * 1.013e-3 * ed / ra
                pt = (delta * RG + e_air) / (delta + gam * (1 + rs / ra))
                pt = pt / lam
                pt = pt * 0.001
                qptr = p["cETP"] * pt * 60.
                etp = qptr * a["veg_frac"][i] + qpet * (1. - a["veg_frac"][i])
                if math.isnan(qptr) or math.isinf(qptr):
                    return 10, i
            for k, v in [("t_prcp", prcp), ("t_temp", temp), ("t_lai", lai), ("t_mf", mf), ("t_rn", rn),
                         ("t_wind", wind), ("t_rh", rh), ("qEleprep", prcp), ("qPotEvap", qpet), ("qPotTran", qptr),
                         ("qEleETP", etp), ("rn_factor", factor)]:
                o[k][i] = v
        DT = f.t_next - f.t
        for i in range(n):                                      # ET, MD_ET.cpp:282-341
            T, prcp, MF = o["t_temp"][i], o["t_prcp"][i], o["t_mf"][i]
            sn = self.y_snow[i]
            snf = frozen(T, 1.0, -3.0)
            if p["cryosphere"]:
                self.acc_s[i].push(T, f.t)
                self.acc_g[i].push(T, f.t)
                o["fu_sub"][i] = 1. - frozen(self.acc_g[i].get(), p["ft_sub_max"], p["ft_sub_min"])
                o["fu_surf"][i] = 1. - frozen(self.acc_s[i].get(), p["ft_surf_max"], p["ft_surf_min"])
            else:
                o["fu_sub"][i] = o["fu_surf"][i] = 1.
            sacc = snf * prcp
            melt = (T - 0.0) * MF if T > 0.0 else 0.
            melt = rmin(rmax(0., sn / DT), rmax(0., melt))
            sn += (sacc - melt) * DT
            LAI, vg = o["t_lai"][i], a["veg_frac"][i]
            ic = self.y_is[i] / vg if vg > ZERO else 0.0
            if LAI > ZERO:
                icmax = p["cISmax"] * 0.0002 * LAI
                iacc = rmin(prcp - sacc, rmax(0., (icmax - ic) / DT))
                iev = rmin(rmax(0., ic / DT), o["qPotEvap"][i])
            else:
                iacc = iev = 0.
            ic += (iacc - iev) * DT
            self.y_is[i] = ic * vg
            self.y_snow[i] = sn
            o["qEleE_IC"][i] = iev * vg
            o["qEleNetPrep"][i] = (1. - snf) * prcp + melt - iacc * vg
        o["yEleIS"], o["yEleSnow"] = self.y_is.copy(), self.y_snow.copy()
        self.out = o
        return 0, -1
