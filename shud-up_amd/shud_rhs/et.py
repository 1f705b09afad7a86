"""ET-step prelude inputs (include/shud_et.h): per-element statics, calibration/config parameters and the
per-step forcing rows, with ctypes struct builders shared by the device handle (runtime.RhsHandle.et_*) and
the CPU oracle (oracle/oracle.py OracleEt), plus a seeded synthetic generator covering every branch of
tReadForcing/ET (MD_ET.cpp:21-341): lakes, LAI = 0, rain/snow/melt regimes, cryosphere, TSR modes."""
import ctypes as C
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import abi

ET_I = ["iforc", "ilc", "imf", "ilake"]
ET_D = ["z_surf", "albedo", "fix_pressure", "wind_h", "veg_frac", "nx", "ny", "nz"]
DEFAULT_PARAMS = dict(cPrep=1.0, cTemp=0.0, cLAItsd=1.0, cMF=1.0, cETP=1.0, cISmax=1.0, radiation_input_mode=0,
                      terrain_radiation=1, rad_factor_cap=5.0, rad_cosz_min=0.05, cryosphere=0, ft_surf_day=7,
                      ft_sub_day=28, ft_surf_max=-1.0, ft_surf_min=-5.0, ft_sub_max=-3.0, ft_sub_min=-10.0)


def _p(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype)) if a is not None else None


@dataclass
class EtModel:
    arrays: dict
    params: dict = field(default_factory=lambda: dict(DEFAULT_PARAMS))
    _keep: list = field(default_factory=list)

    @property
    def num_ele(self):
        return int(self.arrays["z_surf"].size)

    def mesh_struct(self):
        s = abi.ShudEtMeshSoA()
        s.num_ele = self.num_ele
        keep = []
        for k in ET_I:
            a = self.arrays.get(k)
            a = None if a is None else np.ascontiguousarray(a, dtype=np.int32)
            keep.append(a)
            setattr(s, k, _p(a, C.c_int32))
        for k in ET_D:
            a = self.arrays.get(k)
            a = None if a is None else np.ascontiguousarray(a, dtype=np.float64)
            keep.append(a)
            setattr(s, k, _p(a, C.c_double))
        self._keep = keep
        return s

    def params_struct(self):
        p = abi.ShudEtParams()
        for k, v in self.params.items():
            setattr(p, k, v)
        return p

    def subset(self, idx):
        """statics of the elements idx (a partition's local elements)"""
        return EtModel({k: (None if v is None else np.asarray(v)[idx]) for k, v in self.arrays.items()},
                       dict(self.params))


@dataclass
class EtForcing:
    t: float
    t_next: float
    station: np.ndarray          # [ns, 6]
    station_z: np.ndarray        # [ns]
    lai_row: np.ndarray
    mf_row: np.ndarray
    tsr_mode: int = abi.SHUD_TSR_OFF
    tsr: Optional[np.ndarray] = None   # [4, n]: sx, sy, sz, wdt
    tsr_den: float = 0.0
    _keep: list = field(default_factory=list)

    def struct(self):
        f = abi.ShudEtForcing()
        st = np.ascontiguousarray(self.station, dtype=np.float64)
        sz = np.ascontiguousarray(self.station_z, dtype=np.float64)
        lai = np.ascontiguousarray(self.lai_row, dtype=np.float64)
        mf = np.ascontiguousarray(self.mf_row, dtype=np.float64)
        f.t, f.t_next = self.t, self.t_next
        f.n_station, f.station, f.station_z = st.shape[0], _p(st, C.c_double), _p(sz, C.c_double)
        f.n_lai_col, f.lai_row = lai.size, _p(lai, C.c_double)
        f.n_mf_col, f.mf_row = mf.size, _p(mf, C.c_double)
        f.tsr_mode = self.tsr_mode
        keep = [st, sz, lai, mf]
        if self.tsr is not None:
            rows = [np.ascontiguousarray(self.tsr[k], dtype=np.float64) for k in range(4)]
            keep += rows
            f.tsr_n = rows[0].size
            f.tsr_sx, f.tsr_sy, f.tsr_sz, f.tsr_wdt = (_p(r, C.c_double) for r in rows)
        f.tsr_den = self.tsr_den
        self._keep = keep
        return f


def out_struct(n):
    arrs = {k: np.zeros(n) for k in abi.ET_OUT}
    o = abi.ShudEtOut()
    for k, a in arrs.items():
        setattr(o, k, _p(a, C.c_double))
    return o, arrs


def pressure_elevation(z):
    """PressureElevation (is_sm_et.hpp:91-96), as Element.cpp:222 sets FixPressure"""
    return 101.325 * np.power((293. - 0.0065 * z) / 293, 5.26)


def synth_et(num_ele, n_station=4, n_lc=6, n_mf=2, seed=3, lake_frac=0.02, terrain=True):
    rng = np.random.default_rng(seed)
    z = rng.uniform(200, 2500, num_ele)
    nrm = rng.normal(size=(3, num_ele))
    nrm[2] = np.abs(nrm[2]) + 2.0                      # mostly up-facing, some steep
    nrm /= np.linalg.norm(nrm, axis=0)
    a = dict(iforc=rng.integers(0, n_station, num_ele), ilc=rng.integers(1, n_lc + 1, num_ele),
             imf=rng.integers(1, n_mf + 1, num_ele), ilake=(rng.random(num_ele) < lake_frac).astype(np.int32),
             z_surf=z, albedo=rng.uniform(0.1, 0.3, num_ele), fix_pressure=pressure_elevation(z),
             wind_h=np.full(num_ele, 10.0), veg_frac=np.where(rng.random(num_ele) < 0.05, 0.0,
                                                              rng.uniform(0.1, 0.95, num_ele)),
             nx=nrm[0], ny=nrm[1], nz=nrm[2])
    p = dict(DEFAULT_PARAMS)
    p["terrain_radiation"] = 1 if terrain else 0
    return EtModel(a, p)


def synth_forcing(t, dt, n_station=4, n_lc=6, n_mf=2, seed=0, tsr_mode=abi.SHUD_TSR_OFF, n_tsr=24, temp=None):
    """Station rows (time, APCP mm/d, TMP C, RH, wind m/s, DSWRF W/m2): a cold, a melting, a warm and a
    station with NA elevation; LAI row with a zero column (bare soil); TSR samples with night entries."""
    rng = np.random.default_rng(seed)
    st = np.zeros((n_station, 6))
    st[:, 0] = t
    st[:, 1] = rng.choice([0.0, 0.5, 12.0, 40.0], n_station)
    base = np.array([-12.0, -1.5, 0.5, 18.0])
    st[:, 2] = (base[np.arange(n_station) % 4] if temp is None else temp) + rng.normal(0, 0.5, n_station)
    st[:, 3] = rng.choice([0.0, 0.005, 0.4, 0.95, 1.3], n_station)       # below CONST_RH and above 1 too
    st[:, 4] = rng.choice([-3.0, 0.0, 2.0, 8.0], n_station)              # fabs(wind) + 0.001
    st[:, 5] = rng.uniform(0, 900, n_station)
    sz = rng.uniform(0, 3000, n_station)
    sz[-1] = -9999.0                                                      # NA station elevation
    lai = np.concatenate([[t], rng.uniform(0.0, 6.0, n_lc)])
    lai[1] = 0.0                                                          # bare soil column
    mf = np.concatenate([[t], rng.uniform(0.0005, 0.003, n_mf)])
    f = EtForcing(t, t + dt, st, sz, lai, mf, tsr_mode)
    if tsr_mode == abi.SHUD_TSR_RECOMPUTE:
        ang = rng.uniform(0, 2 * np.pi, n_tsr)
        cz = rng.uniform(-0.3, 1.0, n_tsr)
        sinz = np.sqrt(np.maximum(0.0, 1 - cz * cz))
        wdt = np.where(cz > 0, cz * 60.0, 0.0)
        f.tsr = np.vstack([sinz * np.sin(ang), sinz * np.cos(ang), cz, wdt])
        f.tsr_den = float(wdt.sum())
    return f
