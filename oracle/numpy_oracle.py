"""TEST INFRASTRUCTURE ONLY — second, independent restatement of the SHUD RHS in vectorised numpy.

Written separately from shud_oracle.c (different code shape: whole-array expressions instead of the
reference's per-element loops) so the two restatements cross-check each other; the reference itself
cannot be compiled here (no SUNDIALS headers) and ships no golden vectors ("parity unpinned").
Same fp64 operation order as the reference, so on identical inputs it must agree with shud_oracle.c
bit for bit.  Citations are to /root/reference/src.  Serial (`make shud`) and OMP semantics.
Pure-numpy; sized for meshes up to ~1e5 elements in tests.
"""
import ctypes
import ctypes.util

import numpy as np

# glibc libm (the library the reference links): numpy's SIMD cbrt/power/cos differ by an ulp
_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
for _f in ("cbrt", "cos"):
    getattr(_libm, _f).restype = ctypes.c_double
    getattr(_libm, _f).argtypes = [ctypes.c_double]
_libm.pow.restype = ctypes.c_double
_libm.pow.argtypes = [ctypes.c_double, ctypes.c_double]
_vcbrt = np.vectorize(_libm.cbrt, otypes=[np.float64])
_vcos = np.vectorize(_libm.cos, otypes=[np.float64])
_vpow = np.vectorize(_libm.pow, otypes=[np.float64])


def cbrt(x):
    return _vcbrt(np.asarray(x, dtype=np.float64))


def cos(x):
    return _vcos(np.asarray(x, dtype=np.float64))


def power(a, b):
    a, b = np.broadcast_arrays(np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64))
    return _vpow(a, b)


ZERO = 1.0e-10
EPSILON = 0.005
EPS_SLOPE = 0.05e-6
PI = 3.1415926          # Macros.hpp:46 (truncated)
GRAV = 9.8


def rmin(a, b):          # functions.hpp:117-119
    return np.where(a > b, b, a)


def rmax(a, b):          # functions.hpp:120-123
    return np.where(a < b, b, a)


def manning(A, n, R, S):  # Equations.hpp:54-63, pow23 :36-39
    t = cbrt(R)
    p23 = t * t
    with np.errstate(invalid="ignore", divide="ignore"):
        pos = np.sqrt(np.where(S > 0, S, 0.0)) * A * p23 / n
        neg = -1.0 * np.sqrt(np.where(S > 0, 0.0, -S)) * A * p23 / n
    return np.where(S > 0, pos, neg)


class NumpyRhs:
    def __init__(self, m, mode=0):
        self.m = m
        self.mode = mode
        NE = m.num_ele
        self.u_satn = np.zeros(NE)
        self.e_ic = np.zeros(NE)
        self.ugw_stale = np.zeros(NE)
        st = {"fu_surf": np.ones(NE), "fu_sub": np.ones(NE)}
        for k in ["net_prep", "pot_evap", "pot_tran", "etp", "lai"]:
            st[k] = np.zeros(NE)
        self.st = st
        self.tabs = {k: np.zeros(1) for k in ["ele_ybc", "ele_qbc", "riv_ybc", "riv_qbc"]}

    def set_step_inputs(self, step=None, bc_tables=None):
        step = self.m.step if step is None else step
        for k, v in step.items():
            if k == "u_satn":
                self.u_satn = np.array(v, dtype=float)
            elif k == "e_ic":
                self.e_ic = np.array(v, dtype=float)
            elif k == "ugw_stale":
                self.ugw_stale = np.array(v, dtype=float)
            else:
                self.st[k] = np.array(v, dtype=float)
        bct = self.m.bc_tables if bc_tables is None else bc_tables
        for k, v in bct.items():
            self.tabs[k] = np.array(v, dtype=float)

    def eval(self, t, Y):
        m, omp = self.m, self.mode == 1
        NE, NR = m.num_ele, m.num_riv
        P, E, st = m.par, m.ele, self.st
        Y = np.asarray(Y, dtype=float)
        ibc = m.ibc.astype(np.int64)
        # ---- f_update / f_update_omp (MD_update.cpp:102-189, MD_f_omp.cpp:104-170)
        ysf, yus, ygw = Y[:NE], Y[NE:2 * NE], Y[2 * NE:3 * NE]
        if omp:
            ysf = np.where(ysf >= 0.0, ysf, 0.0)
            yus = np.where(yus >= 0.0, yus, 0.0)
            ygw0 = rmax(0.0, ygw)
        else:
            ygw0 = ygw
        ugw = np.where(ibc == 0, ygw0, np.where(ibc > 0, self.tabs["ele_ybc"][np.clip(ibc, 0, None)], self.ugw_stale))
        qbc = np.where(ibc < 0, self.tabs["ele_qbc"][np.clip(-ibc, 0, None)], 0.0)
        yr = Y[3 * NE:3 * NE + NR]
        if omp:
            yr = np.where(yr >= 0.0, yr, 0.0)
        rbc = m.riv_bc.astype(np.int64)
        w0, bs, L = m.riv["riv_bottom_width"], m.riv["riv_bankslope"], m.riv["riv_length"]
        topw = yr * bs * 2.0 + w0                      # River.hpp:115-127, River.cpp:49-62
        csa = yr * (w0 + yr * bs)
        ys = yr * bs
        per = 2.0 * np.sqrt(yr * yr + ys * ys) + w0
        eqw = 0.5 * ((yr * bs * 2.0 + w0) + w0)
        tarea = eqw * L
        topw, csa, per, tarea = [np.where(v < 0.0, 0.0, v) for v in (topw, csa, per, tarea)]
        uriv = np.where(rbc > 0, self.tabs["riv_ybc"][np.clip(rbc, 0, None)], yr)
        rqbc = np.where(rbc < 0, self.tabs["riv_qbc"][np.clip(-rbc, 0, None)], 0.0)
        aq, infD, ThS, ThR = P["aquifer_depth"], P["infD"], P["ThetaS"], P["ThetaR"]
        # ---- f_etFlux (MD_ET.cpp:343-404)
        Es = Eu = Eg = Tu = Tg = np.zeros(NE)
        if not omp:
            va, vb, pj = P["VegFrac"], 1.0 - P["VegFrac"], 1.0 - P["ImpAF"]
            pet, ptr, eic = st["pot_evap"], st["pot_tran"], self.e_ic.copy()
            fc = ThS * 0.75
            b = rmin(rmax(0.0, (self.u_satn * (ThS - ThR) - ThR) / (fc - ThR)), 1.0)
            beta = 0.5 * (1 - cos(PI * b))
            Es = rmin(rmax(0.0, ysf), pet) * vb
            wet = ugw > aq - infD
            Eg = np.where((Es < pet) & wet, rmin(rmax(0.0, ugw), pet - Es) * pj * vb, 0.0)
            Eu = np.where((Es < pet) & ~wet, rmin(rmax(0.0, yus), beta * (pet - Es)) * pj * vb, 0.0)
            lai = st["lai"] > ZERO
            full = eic >= ptr
            root = ugw > aq - P["RzD"]
            Tg = np.where(lai & ~full & root, rmin(rmax(0.0, ugw), ptr - eic) * pj * va, 0.0)
            Tu = np.where(lai & ~full & ~root, rmin(rmax(0.0, yus), beta * (ptr - eic)) * pj * va, 0.0)
            self.e_ic = np.where(lai, np.where(full, ptr * pj * va, eic), 0.0)
        # ---- updateElement / effKH / satKfun (Element.cpp:347-384, Equations.cpp:116-141)
        macd, kmac, af, kmx = P["macD"], P["macKsatH"], P["geo_vAreaF"], P["KsatH"]

        def effkh(g, a, md, km, f, kx):
            with np.errstate(invalid="ignore", divide="ignore"):
                return np.where((md <= ZERO) | (g < a - md), kx,
                                np.where(g > a, (km * md * f + kx * (a - md * f)) / a,
                                         (km * (g - (a - md)) * f + kx * (a - md + (g - (a - md)) * (1 - f))) / g))
        ekh = effkh(ugw, aq, macd, kmac, af, kmx)
        with np.errstate(invalid="ignore", divide="ignore"):
            deficit = aq - ugw
            dry = deficit <= 0.0
            theta = np.where(dry, ThS, yus / np.where(dry, 1.0, deficit) * ThS)
            satn = np.where(dry, 1.0, (theta - ThR) / (ThS - ThR))
            deficit = np.where(dry, 0.0, deficit)
            hi, lo = satn > 0.99, satn <= ZERO
            n = P["Beta"]
            s_ = np.where(hi | lo, 0.5, satn)
            tmp = -1.0 + power(1.0 - power(s_, n / (n - 1.0)), (n - 1.0) / n)
            satkr = np.where(hi, 1.0, np.where(lo, 0.0, np.sqrt(s_) * tmp * tmp))
            theta = np.where(hi, ThS, np.where(lo, ThR, theta))
            satn = np.where(hi, 1.0, np.where(lo, 0.0, satn))
        self.u_satn = satn
        infK, hA, macKV = P["infKsatV"], P["hAreaF"], P["macKsatV"]
        kmax = infK * (1.0 - hA) + macKV * hA
        # ---- Flux_Infiltration (Element.cpp:271-303)
        with np.errstate(invalid="ignore", divide="ignore"):
            av = ysf + st["net_prep"]
            exf = (ugw + yus > aq) | (deficit < yus)
            qex = np.where(exf, np.abs(ugw + yus - aq) / aq * kmax, 0.0)
            ek = np.where(av > kmax, infK * (1 - hA) + hA * macKV * satn,
                          np.where(av > infK, satkr * infK * (1 - hA) + hA * macKV * satn, satkr * infK * (1 - hA)))
            qi = np.where(~exf & (av > 0.0) & (deficit > infD), rmin(av, rmax(0.0, (1.0 + av / infD) * ek)), 0.0)
        q_infil, q_exfil = qi * st["fu_surf"], qex * st["fu_surf"]
        # ---- Flux_Recharge (Element.cpp:304-335), meanHarmonic (Equations.hpp:45-48)
        with np.errstate(invalid="ignore", divide="ignore"):
            skip = (ugw > aq - infD) & (yus < deficit)
            grad = np.where((theta > ThR) & ~(yus <= EPSILON), rmax((theta - ThR) / (ThS * 0.75 - ThR), 0.0), 0.0)
            ku = infK * satkr
            KV = P["KsatV"]
            ke = (ku * KV) * (deficit + ugw) / (deficit * KV + ugw * ku)
            qr = np.where(skip | (infK <= 0.0) | (KV <= 0.0), 0.0, grad * ke)
        q_rech = qr * st["fu_sub"]
        # ---- fun_Ele_surface / fun_Ele_sub (MD_ElementFlux.cpp:35-156)
        nab = m.nabr.reshape(3, NE)
        zs, zb, dep = E["z_surf"], E["z_bottom"], E["depression"]
        isf = np.where(ysf < 0.0, 0.0, ysf)
        QS = np.zeros((3, NE))
        QG = np.zeros((3, NE))
        for j in range(3):
            nb = nab[j]
            has = nb >= 0
            k = np.where(has, nb, 0)
            B = E["edge"].reshape(3, NE)[j]
            d2n = E["dist2nabor"].reshape(3, NE)[j]
            nsf = np.where(ysf[k] < 0.0, 0.0, ysf[k])
            with np.errstate(invalid="ignore", divide="ignore"):
                dh = (isf + zs) - (nsf + zs[k])
                ym = np.where((zs + isf) > (zs[k] + nsf), np.where(isf > dep, isf, 0.0), np.where(nsf > dep, nsf, 0.0))
                ym = rmin(ym, 0.5)
                s = dh / np.where(has, d2n, 1.0)
                guard = ((s > 0) & (isf <= 0)) | ((s < 0) & (nsf <= 0))
                q = np.where((ym <= 0.0) | guard, 0.0, manning(ym * B, E["avg_rough"].reshape(3, NE)[j], ym, s))
                ugn = ugw[k]
                dhg = (ugw + zb) - (ugn + zb[k])
                gg = ((dhg > 0.0) & (ugw <= 0.02)) | ((dhg < 0.0) & (ugn <= 0.02))
                ymg = (rmax(ugw, 0.0) + rmax(ugn, 0.0)) * 0.5
                qg = 0.5 * (ekh + ekh[k]) * (dhg / np.where(has, d2n, 1.0)) * ymg * B
                qg = np.where(gg, 0.0, qg)
            qb_s = np.zeros(NE)
            qb_g = np.zeros(NE)
            if m.close_boundary == 0:
                d2e = E["dist2edge"].reshape(3, NE)[j]
                with np.errstate(invalid="ignore", divide="ignore"):
                    sb = isf / d2e * 0.5
                    qb_s = np.where((isf > dep) & (sb > 0.0),
                                    np.sqrt(np.where(sb > 0, sb, 0.0)) * cbrt(isf * isf * isf * isf * isf) * B / E["rough"], 0.0)
                    gb = ugw / d2e * 0.5
                    qb_g = np.where((ugw > dep * 10.0) & (gb > 0.0), ekh * gb, 0.0)
            QS[j] = np.where(has, q, qb_s)
            QG[j] = np.where(has, qg, qb_g) * st["fu_sub"]
        # ---- segments (MD_RiverFlux.cpp:65-126, Flux_RiverElement.cpp:11-55)
        se, sr, sl, cw = m.seg_ele, m.seg_riv, m.seg_length, m.seg_cwr
        with np.errstate(invalid="ignore", divide="ignore"):
            yi = rmax(0.0, ysf[se] - q_infil[se] + q_exfil[se])
            zi = zs[se]
            zj = zs[se] - m.riv["riv_depth"][sr]
            yj = uriv[sr]
            zbank = zs[se] + 0.0
            hi_, hj_ = yi + zi, yj + zj
            dhw = hj_ - hi_
            yy = hi_ - zbank
            c1 = (yy > 0.0) & (yj > dep[se])
            yv1 = np.where(hi_ > zbank, dhw, yy)
            q1 = np.where(c1, cw * np.sqrt(2.0 * GRAV * np.where(c1, yv1, 0.0)) * sl * yv1 * 60.0, 0.0)
            c2 = (yy > 0.0) & (yi > dep[se])
            yv2 = np.where(hj_ > zbank, -dhw, yy)
            q2 = np.where(c2, -1.0 * cw * np.sqrt(2.0 * GRAV * np.where(c2, yv2, 0.0)) * sl * yv2 * 60.0, 0.0)
            qsurf = np.where(dhw > 0.0, q1, q2)
            ke_, kr = ekh[se], m.riv["riv_ksath"][sr]
            K = (ke_ * 1.0 + kr * 1.0) / (1.0 + 1.0)
            he, hr = ugw[se] + zb[se], yj + zj
            dhs = hr - he
            A1 = np.where(he > zj, (yj + (he - zj)) * 0.5 * sl, yj * sl)
            D = m.riv["riv_bedthick"][sr]
            qa = np.where(yj < EPSILON, 0.0, A1 * K * (dhs / D))
            qb = np.where(ugw[se] > ZERO, (yj + (he - zj)) * 0.5 * sl * K * (dhs / D), 0.0)
            qsub = np.where(dhs > ZERO, qa, np.where(dhs < -ZERO, qb, 0.0))
            qsub = np.where((ke_ < ZERO) | (kr < ZERO), 0.0, qsub) * st["fu_sub"][se]
        # ---- Flux_RiverDown (MD_RiverFlux.cpp:5-63)
        rd = m.riv_down.astype(np.int64)
        dn = np.where(rd >= 0, rd, 0)
        nrough = m.riv["riv_avg_rough"]
        slope, depth = m.riv["riv_bed_slope"], m.riv["riv_depth"]
        with np.errstate(invalid="ignore", divide="ignore"):
            sdn = ((uriv - depth) - (uriv[dn] - depth[dn])) / m.riv["riv_dist2down"] + (slope + slope[dn]) * 0.5
            R1 = np.where(per <= ZERO, 0.0, csa / np.where(per <= ZERO, 1.0, per))
            sout = slope + uriv * 2.0 / L
            R2 = np.where(per <= 0.0, 0.0, csa / np.where(per <= 0.0, 1.0, per))
            qdown = np.where(rd >= 0, manning(csa, nrough, R1, sdn),
                             np.where(rd >= -3, manning(csa, nrough, R2, sout),
                                      csa * np.sqrt(GRAV * uriv) * 60.0))
        # ---- PassValue (MD_f.cpp:217-257): ascending-index scatter sums
        qriv_surf = np.zeros(NR)
        qriv_sub = np.zeros(NR)
        qe2r_surf = np.zeros(NE)
        qe2r_sub = np.zeros(NE)
        np.add.at(qriv_surf, sr, qsurf)          # np.add.at applies in index order (unbuffered)
        np.add.at(qriv_sub, sr, qsub)
        np.add.at(qe2r_surf, se, -qsurf)
        np.add.at(qe2r_sub, se, -qsub)
        qup = np.zeros(NR)
        has_dn = rd >= 0
        np.add.at(qup, rd[has_dn], -qdown[has_dn])
        # ---- f_applyDY (MD_f.cpp:52-215) / _omp (MD_f_omp.cpp:9-67)
        tots = qe2r_surf + QS[0] + QS[1] + QS[2]
        totg = qe2r_sub + QG[0] + QG[1] + QG[2]
        area = E["area"]
        dsf = st["net_prep"] - q_infil + q_exfil - tots / area - Es
        dus = q_infil - q_rech - Eu - Tu
        dgw = q_rech - q_exfil - totg / area - Eg - Tg
        dgw = np.where(ibc > 0, 0.0, np.where(ibc < 0, dgw + qbc / area, dgw))
        iss = m.iss
        dsf = np.where(iss > 0, dsf + 0.0 / area, dsf)
        dgw = np.where(iss < 0, dgw + 0.0 / area, dgw)
        dus = dus / P["Sy"]
        dgw = dgw / P["Sy"]
        with np.errstate(invalid="ignore", divide="ignore"):
            flux = (-qup - qriv_surf - qriv_sub - qdown + rqbc)
            if omp:
                dr = flux / tarea
            else:
                dA = flux / L
                dA = np.where(dA < -1.0 * csa, -1.0 * csa, dA)
                sa = np.abs(bs)
                cc = topw * topw + 4 * sa * dA
                quad = np.where(cc < ZERO, -1.0 * topw / (2.0 * sa), (-topw + np.sqrt(np.where(cc < ZERO, 0.0, cc))) / (2 * sa))
                dr = np.where(dA == 0.0, 0.0, np.where(np.abs(bs) < EPS_SLOPE, dA / topw, quad))
            dr = np.where(rbc > 0, 0.0, dr)
        self.diag = dict(qele_surf=QS.reshape(-1), qele_sub=QG.reshape(-1), q_infil=q_infil, q_exfil=q_exfil,
                         q_recharge=q_rech, qseg_surf=qsurf, qseg_sub=qsub, qriv_down=qdown, qriv_up=qup,
                         qriv_surf=qriv_surf, qriv_sub=qriv_sub, eff_kh=ekh, u_satn=satn, e_ic=self.e_ic)
        return np.concatenate([dsf, dus, dgw, dr])
