"""Host-side SoA model: the arrays a reference Model_Data holds for the RHS, in the C-ABI layout.

`ShudModel` is plain numpy (int32 / float64, contiguous).  It is filled either by the SHUD text-input
reader (shudio.py: MD_readin.cpp + MD_initialize.cpp semantics) or by the synthetic mesh generator
(synth.py), and turned into the ShudMeshSoA / ShudParamsSoA / ShudStepInputs structs of
include/shud_rhs.h by `mesh_struct()` / `params_struct()` / `step_struct()`.
"""
from dataclasses import dataclass, field
from typing import Dict, Optional
import ctypes as C

import numpy as np

from . import abi

ELE1 = ["area", "z_surf", "z_bottom", "depression", "rough"]
ELE3 = ["edge", "dist2nabor", "dist2edge", "avg_rough"]
RIV_D = ["riv_length", "riv_bed_slope", "riv_dist2down", "riv_avg_rough", "riv_depth", "riv_bottom_width",
         "riv_bankslope", "riv_ksath", "riv_bedthick"]


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _i(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _ptr(a, ctype):
    if a is None:
        return C.cast(None, C.POINTER(ctype))
    return a.ctypes.data_as(C.POINTER(ctype))


@dataclass
class ShudModel:
    num_ele: int
    num_riv: int
    num_seg: int
    close_boundary: int = 1
    ele: Dict[str, np.ndarray] = field(default_factory=dict)     # ELE1 [NE], ELE3 [3*NE] edge-major
    nabr: Optional[np.ndarray] = None                            # [3*NE] int32, -1 boundary
    ibc: Optional[np.ndarray] = None
    iss: Optional[np.ndarray] = None
    ilake: Optional[np.ndarray] = None
    riv: Dict[str, np.ndarray] = field(default_factory=dict)     # RIV_D [NR]
    riv_down: Optional[np.ndarray] = None
    riv_bc: Optional[np.ndarray] = None
    seg_ele: Optional[np.ndarray] = None
    seg_riv: Optional[np.ndarray] = None
    seg_length: Optional[np.ndarray] = None
    seg_cwr: Optional[np.ndarray] = None
    par: Dict[str, np.ndarray] = field(default_factory=dict)     # abi.PARAM_NAMES [NE]
    step: Dict[str, np.ndarray] = field(default_factory=dict)    # abi.STEP_ARRAYS [NE]
    bc_tables: Dict[str, np.ndarray] = field(default_factory=dict)  # ele_ybc, ele_qbc, riv_ybc, riv_qbc
    meta: Dict[str, object] = field(default_factory=dict)
    # lakes: bathymetry table per lake, rows [off[l], off[l+1])
    num_lake: int = 0
    lake_bathy_off: Optional[np.ndarray] = None
    lake_bathy_y: Optional[np.ndarray] = None
    lake_bathy_a: Optional[np.ndarray] = None

    @property
    def num_y(self):
        return 3 * self.num_ele + self.num_riv + self.num_lake

    def finalize(self):
        """Coerce dtypes / contiguity and fill defaults; returns self."""
        NE, NR = self.num_ele, self.num_riv
        for k in ELE1:
            if k in self.ele:
                self.ele[k] = _d(self.ele[k])
        for k in ELE3:
            if k in self.ele:
                self.ele[k] = _d(self.ele[k])
        if "depression" not in self.ele:
            self.ele["depression"] = np.full(NE, 0.0002)
        self.nabr = _i(self.nabr)
        self.ibc = _i(self.ibc if self.ibc is not None else np.zeros(NE))
        self.iss = _i(self.iss if self.iss is not None else np.zeros(NE))
        if self.ilake is not None:
            self.ilake = _i(self.ilake)
        for k in RIV_D:
            self.riv[k] = _d(self.riv[k]) if k in self.riv else np.zeros(NR)
        self.riv_down = _i(self.riv_down if self.riv_down is not None else np.full(NR, -3))
        self.riv_bc = _i(self.riv_bc if self.riv_bc is not None else np.zeros(NR))
        self.seg_ele = _i(self.seg_ele)
        self.seg_riv = _i(self.seg_riv)
        self.seg_length = _d(self.seg_length)
        self.seg_cwr = _d(self.seg_cwr)
        for k in abi.PARAM_NAMES:
            self.par[k] = _d(self.par[k])
        for k in list(self.step):
            self.step[k] = _d(self.step[k])
        for k in list(self.bc_tables):
            self.bc_tables[k] = _d(self.bc_tables[k])
        if self.num_lake:
            self.lake_bathy_off = _i(self.lake_bathy_off)
            self.lake_bathy_y = _d(self.lake_bathy_y)
            self.lake_bathy_a = _d(self.lake_bathy_a)
        return self

    # ---- C structs (the returned struct references arrays owned by self) ----
    def mesh_struct(self):
        m = abi.ShudMeshSoA()
        m.num_ele, m.num_riv, m.num_seg, m.close_boundary = self.num_ele, self.num_riv, self.num_seg, self.close_boundary
        m.nabr = _ptr(self.nabr, C.c_int32)
        for k in ELE1 + ELE3:
            setattr(m, k, _ptr(self.ele.get(k), C.c_double))
        m.ibc = _ptr(self.ibc, C.c_int32)
        m.iss = _ptr(self.iss, C.c_int32)
        m.ilake = _ptr(self.ilake, C.c_int32)
        m.riv_down = _ptr(self.riv_down, C.c_int32)
        m.riv_bc = _ptr(self.riv_bc, C.c_int32)
        for k in RIV_D:
            setattr(m, k, _ptr(self.riv[k], C.c_double))
        m.seg_ele = _ptr(self.seg_ele, C.c_int32)
        m.seg_riv = _ptr(self.seg_riv, C.c_int32)
        m.seg_length = _ptr(self.seg_length, C.c_double)
        m.seg_cwr = _ptr(self.seg_cwr, C.c_double)
        m.num_lake = self.num_lake
        m.lake_bathy_off = _ptr(self.lake_bathy_off if self.num_lake else None, C.c_int32)
        m.lake_bathy_y = _ptr(self.lake_bathy_y if self.num_lake else None, C.c_double)
        m.lake_bathy_a = _ptr(self.lake_bathy_a if self.num_lake else None, C.c_double)
        return m

    def params_struct(self):
        p = abi.ShudParamsSoA()
        for k in abi.PARAM_NAMES:
            setattr(p, k, _ptr(self.par[k], C.c_double))
        return p

    def step_struct(self, step=None, bc_tables=None):
        """ShudStepInputs for `step` (defaults to self.step); missing arrays are passed as NULL."""
        step = self.step if step is None else step
        bct = self.bc_tables if bc_tables is None else bc_tables
        s = abi.ShudStepInputs()
        keep = []
        for k in abi.STEP_ARRAYS:
            a = step.get(k)
            if a is not None:
                a = _d(a)
                keep.append(a)
            setattr(s, k, _ptr(a, C.c_double))
        for k in ["ele_ybc", "ele_qbc", "riv_ybc", "riv_qbc"]:
            a = bct.get(k)
            if a is not None:
                a = _d(a)
                keep.append(a)
                setattr(s, k, _ptr(a, C.c_double))
                setattr(s, "n_" + k, len(a) - 1)
            else:
                setattr(s, k, _ptr(None, C.c_double))
                setattr(s, "n_" + k, 0)
        a = step.get("prcp")
        if a is not None:
            a = _d(a)
            keep.append(a)
        s.prcp = _ptr(a, C.c_double)
        s._keep = keep
        return s

    # ---- convenience ----
    def save(self, path):
        d = {"_sizes": np.array([self.num_ele, self.num_riv, self.num_seg, self.close_boundary])}
        for k, v in self.ele.items():
            d["ele_" + k] = v
        for k, v in self.riv.items():
            d["R_" + k] = v
        for k, v in self.par.items():
            d["par_" + k] = v
        for k, v in self.step.items():
            d["step_" + k] = v
        for k, v in self.bc_tables.items():
            d["bct_" + k] = v
        for k in ["nabr", "ibc", "iss", "riv_down", "riv_bc", "seg_ele", "seg_riv", "seg_length", "seg_cwr"]:
            d[k] = getattr(self, k)
        if self.ilake is not None:
            d["ilake"] = self.ilake
        if self.num_lake:
            d["lake_bathy_off"], d["lake_bathy_y"], d["lake_bathy_a"] = (self.lake_bathy_off, self.lake_bathy_y,
                                                                        self.lake_bathy_a)
        np.savez_compressed(path, **d)

    @staticmethod
    def load(path):
        z = np.load(path, allow_pickle=False)
        NE, NR, NS, cb = [int(v) for v in z["_sizes"]]
        m = ShudModel(NE, NR, NS, cb)
        for k in z.files:
            if k.startswith("ele_"):
                m.ele[k[4:]] = z[k]
            elif k.startswith("R_"):
                m.riv[k[2:]] = z[k]
            elif k.startswith("par_"):
                m.par[k[4:]] = z[k]
            elif k.startswith("step_"):
                m.step[k[5:]] = z[k]
            elif k.startswith("bct_"):
                m.bc_tables[k[4:]] = z[k]
        for k in ["nabr", "ibc", "iss", "riv_down", "riv_bc", "seg_ele", "seg_riv", "seg_length", "seg_cwr"]:
            setattr(m, k, z[k])
        if "ilake" in z.files:
            m.ilake = z["ilake"]
        if "lake_bathy_off" in z.files:
            m.lake_bathy_off, m.lake_bathy_y, m.lake_bathy_a = z["lake_bathy_off"], z["lake_bathy_y"], z["lake_bathy_a"]
            m.num_lake = int(m.lake_bathy_off.size - 1)
        return m.finalize()
