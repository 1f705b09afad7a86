"""ctypes front end of libshud_host.so (include/shud_host.h): the C++ host's SHUD project readers,
initialisation, forcing/TSR per ET step and print-control list.  Plain C++ (no HIP): loads on any machine.

`Project.load(indir, prj)` = Model_Data loadinput + initialize + LoadIC (MD_readin.cpp, MD_initialize.cpp);
`model()` wraps the derived SoA as a ShudModel (the same structure shudio.load_project builds);
`forcing(t, tout)` = updateAllTimeSeries(t) + the shared part of tReadForcing (MD_ET.cpp:21-136).
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .et import EtForcing, EtModel
from .model import ELE1, ELE3, RIV_D, ShudModel

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "libshud_host.so")
_LIB = None


class ShudControl(C.Structure):
    _fields_ = [("start_time", C.c_double), ("end_time", C.c_double), ("num_steps", C.c_int64),
                ("solver_step", C.c_double), ("et_step", C.c_double), ("reltol", C.c_double),
                ("abstol", C.c_double), ("init_step", C.c_double), ("max_step", C.c_double),
                ("init_type", C.c_int32), ("close_boundary", C.c_int32), ("ascii", C.c_int32),
                ("binary", C.c_int32), ("cryosphere", C.c_int32), ("verbose", C.c_int32),
                ("terrain_radiation", C.c_int32), ("radiation_input_mode", C.c_int32),
                ("solar_lonlat_mode", C.c_int32), ("solar_lon_deg", C.c_double), ("solar_lat_deg", C.c_double),
                ("rad_factor_cap", C.c_double), ("rad_cosz_min", C.c_double),
                ("tsr_integration_step_min", C.c_int32), ("forc_start_time", C.c_int64),
                ("num_forc", C.c_int32), ("lakeon", C.c_int32), ("num_lake", C.c_int32)]


class ShudOutputDecl(C.Structure):
    _fields_ = [("basename", C.c_char_p), ("array", C.c_int32), ("column", C.c_int32), ("n_all", C.c_int32),
                ("interval", C.c_int32), ("iflux", C.c_int32), ("flag_io", C.POINTER(C.c_int32))]


_H = C.c_void_p


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C shud-up_amd`")
        L = C.CDLL(LIB_PATH)
        sig = {
            "shud_project_load": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_double, C.POINTER(_H)]),
            "shud_project_error": (C.c_char_p, []),
            "shud_project_free": (None, [_H]),
            "shud_project_control": (C.c_int, [_H, C.POINTER(ShudControl)]),
            "shud_project_mesh": (C.c_int, [_H, C.POINTER(abi.ShudMeshSoA), C.POINTER(abi.ShudParamsSoA)]),
            "shud_project_et": (C.c_int, [_H, C.POINTER(abi.ShudEtMeshSoA), C.POINTER(abi.ShudEtParams)]),
            "shud_project_array": (C.POINTER(C.c_double), [_H, C.c_char_p, C.POINTER(C.c_int64)]),
            "shud_project_outputs": (C.c_int, [_H, C.c_char_p, C.POINTER(ShudOutputDecl), C.c_int]),
            "shud_project_forcing": (C.c_int, [_H, C.c_double, C.c_double, C.POINTER(abi.ShudEtForcing)]),
            "shud_project_bc_rows": (C.c_int, [_H, C.POINTER(abi.ShudStepInputs)]),
            "shud_project_solar": (C.c_int, [_H, C.c_double, C.c_double, C.c_double, C.c_double,
                                             C.POINTER(C.c_double)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _LIB = L
    return _LIB


def _arr(ptr, n, dtype):
    if not ptr or n == 0:
        return None
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


class Project:
    def __init__(self, indir, prj, cwd=None, end_day=-1.0):
        h = _H()
        rc = lib().shud_project_load(str(indir).encode(), str(prj).encode(),
                                     None if cwd is None else str(cwd).encode(), float(end_day), C.byref(h))
        if rc:
            raise RuntimeError(f"shud_project_load: {lib().shud_project_error().decode(errors='replace')}")
        self.h = h
        self.prj = prj

    def close(self):
        if self.h:
            lib().shud_project_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def control(self):
        c = ShudControl()
        lib().shud_project_control(self.h, C.byref(c))
        return {k: getattr(c, k) for k, _ in ShudControl._fields_}

    def array(self, name):
        n = C.c_int64()
        p = lib().shud_project_array(self.h, name.encode(), C.byref(n))
        return _arr(p, n.value, np.float64)

    def model(self):
        """ShudModel copy of the derived SoA (ShudMeshSoA / ShudParamsSoA)."""
        m, q = abi.ShudMeshSoA(), abi.ShudParamsSoA()
        lib().shud_project_mesh(self.h, C.byref(m), C.byref(q))
        NE, NR, NS = m.num_ele, m.num_riv, m.num_seg
        out = ShudModel(NE, NR, NS, m.close_boundary)
        for k in ELE1:
            out.ele[k] = _arr(getattr(m, k), NE, np.float64)
        for k in ELE3:
            out.ele[k] = _arr(getattr(m, k), 3 * NE, np.float64)
        out.nabr = _arr(m.nabr, 3 * NE, np.int32)
        out.ibc, out.iss = _arr(m.ibc, NE, np.int32), _arr(m.iss, NE, np.int32)
        out.ilake = _arr(m.ilake, NE, np.int32)
        for k in RIV_D:
            out.riv[k] = _arr(getattr(m, k), NR, np.float64)
        out.riv_down, out.riv_bc = _arr(m.riv_down, NR, np.int32), _arr(m.riv_bc, NR, np.int32)
        out.seg_ele, out.seg_riv = _arr(m.seg_ele, NS, np.int32), _arr(m.seg_riv, NS, np.int32)
        out.seg_length, out.seg_cwr = _arr(m.seg_length, NS, np.float64), _arr(m.seg_cwr, NS, np.float64)
        for k in abi.PARAM_NAMES:
            out.par[k] = _arr(getattr(q, k), NE, np.float64)
        if m.num_lake:
            out.num_lake = m.num_lake
            out.lake_bathy_off = _arr(m.lake_bathy_off, m.num_lake + 1, np.int32)
            nb = int(out.lake_bathy_off[-1])
            out.lake_bathy_y = _arr(m.lake_bathy_y, nb, np.float64)
            out.lake_bathy_a = _arr(m.lake_bathy_a, nb, np.float64)
        return out.finalize()

    def et_model(self):
        """EtModel (et.py) of the prelude statics and parameters (shud_et_attach inputs)."""
        m, q = abi.ShudEtMeshSoA(), abi.ShudEtParams()
        lib().shud_project_et(self.h, C.byref(m), C.byref(q))
        NE = m.num_ele
        arrays = {k: _arr(getattr(m, k), NE, np.int32) for k in ("iforc", "ilc", "imf", "ilake")}
        arrays.update({k: _arr(getattr(m, k), NE, np.float64)
                       for k in ("z_surf", "albedo", "fix_pressure", "wind_h", "veg_frac", "nx", "ny", "nz")})
        params = {k: getattr(q, k) for k, _ in abi.ShudEtParams._fields_}
        return EtModel(arrays, params)

    def outputs(self, outdir):
        outdir = str(outdir).encode()
        n = lib().shud_project_outputs(self.h, outdir, None, 0)
        arr = (ShudOutputDecl * max(n, 1))()
        lib().shud_project_outputs(self.h, outdir, arr, n)
        return [{"basename": d.basename.decode(), "array": d.array, "column": d.column, "n_all": d.n_all,
                 "interval": d.interval, "iflux": d.iflux,
                 "flag_io": None if not d.flag_io else _arr(d.flag_io, d.n_all, np.int32)} for d in arr[:n]]

    def bc_rows(self):
        """{ele_ybc, ele_qbc, riv_ybc, riv_qbc} rows at the current ET step (model.step_struct bc_tables form:
        x[0] = time, x[c] = column c), or {} without boundary conditions"""
        s = abi.ShudStepInputs()
        if lib().shud_project_bc_rows(self.h, C.byref(s)) != 1:
            return {}
        out = {}
        for k in ("ele_ybc", "ele_qbc", "riv_ybc", "riv_qbc"):
            n = getattr(s, "n_" + k)
            p = getattr(s, k)
            if p and n > 0:
                out[k] = _arr(p, n + 1, np.float64)
        return out

    def forcing(self, t, tout):
        """EtForcing for the ET step [t, tout) (advances the series pointers: call in time order)."""
        f = abi.ShudEtForcing()
        if lib().shud_project_forcing(self.h, float(t), float(tout), C.byref(f)):
            raise RuntimeError(lib().shud_project_error().decode(errors="replace"))
        ns = f.n_station
        st = np.ctypeslib.as_array(f.station, shape=(ns * 6,)).reshape(ns, 6).copy()
        sz = _arr(f.station_z, ns, np.float64)
        lai = _arr(f.lai_row, f.n_lai_col, np.float64)
        mf = _arr(f.mf_row, f.n_mf_col, np.float64)
        tsr = None
        if f.tsr_mode in (abi.SHUD_TSR_RECOMPUTE, abi.SHUD_TSR_CACHED) and f.tsr_n:
            tsr = np.stack([_arr(getattr(f, k), f.tsr_n, np.float64) for k in ("tsr_sx", "tsr_sy", "tsr_sz", "tsr_wdt")])
        return EtForcing(f.t, f.t_next, st, sz, lai, mf, tsr_mode=f.tsr_mode, tsr=tsr, tsr_den=f.tsr_den)

    def solar(self, t_min, lat, lon, tz=0.0):
        out = (C.c_double * 5)()
        lib().shud_project_solar(self.h, float(t_min), float(lat), float(lon), float(tz), out)
        return tuple(out)
