"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/liboracle.so (the CPU restatement in
shud_oracle.c).  Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
Parity status: "parity unpinned" (see shud_oracle.c header and DESIGN.md §Oracle).
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "shud-up_amd"))
from shud_rhs import abi  # noqa: E402  (struct layouts of include/shud_rhs.h)

LIB_PATH = os.path.join(HERE, "liboracle.so")
_LIB = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_create.restype = C.c_void_p
        L.oracle_create.argtypes = [C.POINTER(abi.ShudMeshSoA), C.POINTER(abi.ShudParamsSoA), C.c_int]
        L.oracle_set_step_inputs.argtypes = [C.c_void_p, C.POINTER(abi.ShudStepInputs)]
        L.oracle_f.restype = C.c_int
        L.oracle_f.argtypes = [C.c_void_p, C.c_double, C.c_void_p, C.c_void_p]
        L.oracle_get_diag.argtypes = [C.c_void_p, C.POINTER(abi.ShudFluxOut)]
        L.oracle_destroy.argtypes = [C.c_void_p]
        L.oracle_set_threads.argtypes = [C.c_int]
        L.oracle_get_threads.restype = C.c_int
        for n in ["oracle_exit_index", "oracle_exit_kind"]:
            getattr(L, n).restype = C.c_int
            getattr(L, n).argtypes = [C.c_void_p]
        for n in ["oracle_num_calls", "oracle_num_warn"]:
            getattr(L, n).restype = C.c_longlong
            getattr(L, n).argtypes = [C.c_void_p]
        L.oracle_et_create.restype = C.c_void_p
        L.oracle_et_create.argtypes = [C.POINTER(abi.ShudEtMeshSoA), C.POINTER(abi.ShudEtParams)]
        L.oracle_et_set_state.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_et_step.restype = C.c_int
        L.oracle_et_step.argtypes = [C.c_void_p, C.POINTER(abi.ShudEtForcing)]
        L.oracle_et_exit_index.restype = C.c_int
        L.oracle_et_exit_index.argtypes = [C.c_void_p]
        L.oracle_et_get.argtypes = [C.c_void_p, C.POINTER(abi.ShudEtOut)]
        L.oracle_et_destroy.argtypes = [C.c_void_p]
        _LIB = L
    return _LIB


def set_threads(n):
    lib().oracle_set_threads(int(n))


def get_threads():
    return lib().oracle_get_threads()


class OracleRhs:
    """Same call sequence as shud_rhs.runtime.RhsHandle, evaluated by the CPU restatement."""

    def __init__(self, model, mode=abi.SHUD_MODE_SERIAL):
        self.model = model
        self._mesh = model.mesh_struct()
        self._par = model.params_struct()
        self.h = lib().oracle_create(C.byref(self._mesh), C.byref(self._par), int(mode))
        if not self.h:
            raise ValueError("oracle: unsupported configuration (lakes need serial mode)")
        self.mode = mode

    def __del__(self):
        try:
            if self.h:
                lib().oracle_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def set_step_inputs(self, step=None, bc_tables=None):
        s = self.model.step_struct(step, bc_tables)
        lib().oracle_set_step_inputs(self.h, C.byref(s))

    def eval(self, t, y):
        """Returns (ydot, exit_code, exit_index, exit_kind)."""
        y = np.ascontiguousarray(y, dtype=np.float64)
        dy = np.zeros_like(y)
        code = lib().oracle_f(self.h, float(t), y.ctypes.data, dy.ctypes.data)
        return dy, code, lib().oracle_exit_index(self.h), lib().oracle_exit_kind(self.h)

    def num_warn(self):
        return lib().oracle_num_warn(self.h)

    def diagnostics(self):
        m = self.model
        NE, NR, NS = m.num_ele, m.num_riv, m.num_seg
        out, o = {}, abi.ShudFluxOut()
        for name in abi.FLUXOUT_ORDER:
            n = (3 * NE if name in abi.DIAG_ELE3 else NS if name in abi.DIAG_SEG else NR if name in abi.DIAG_RIV
                 else getattr(m, "num_lake", 0) if name in abi.DIAG_LAKE else NE)
            out[name] = np.zeros(n)
            setattr(o, name, out[name].ctypes.data_as(abi.c_double_p))
        lib().oracle_get_diag(self.h, C.byref(o))
        return out


class OracleEt:
    """CPU restatement of the ET-step prelude (shud_oracle_et.c): same calls as RhsHandle.et_*."""

    def __init__(self, etm):
        self.n = etm.num_ele
        self._m = etm.mesh_struct()
        self._p = etm.params_struct()
        self.h = lib().oracle_et_create(C.byref(self._m), C.byref(self._p))

    def set_state(self, y_is=None, y_snow=None):
        a = None if y_is is None else np.ascontiguousarray(y_is, dtype=np.float64)
        b = None if y_snow is None else np.ascontiguousarray(y_snow, dtype=np.float64)
        lib().oracle_et_set_state(self.h, None if a is None else a.ctypes.data, None if b is None else b.ctypes.data)

    def step(self, forcing):
        """returns (exit code, first element index)"""
        fs = forcing.struct()
        code = lib().oracle_et_step(self.h, C.byref(fs))
        return code, lib().oracle_et_exit_index(self.h)

    def get(self):
        from shud_rhs.et import out_struct
        o, arrs = out_struct(self.n)
        lib().oracle_et_get(self.h, C.byref(o))
        return arrs

    def step_inputs(self):
        """the RHS step inputs this step produced (ShudStepInputs names)"""
        g = self.get()
        return dict(net_prep=g["qEleNetPrep"], pot_evap=g["qPotEvap"], pot_tran=g["qPotTran"], etp=g["qEleETP"],
                    lai=g["t_lai"], fu_surf=g["fu_surf"], fu_sub=g["fu_sub"], e_ic=g["qEleE_IC"])

    def __del__(self):
        try:
            if self.h:
                lib().oracle_et_destroy(self.h)
                self.h = None
        except Exception:  # noqa: BLE001
            pass


class OracleOde:
    """CPU restatement of the CVODE 6.0.0 BDF/Newton/SPGMR integrator (shud_oracle_ode.c).

    rhs: an OracleRhs (the SHUD RHS) or a built-in test problem "robertson" / "decay" / "decayn"."""

    STATS = ["nst", "nfe", "nfe_ls", "nni", "ncfn", "nnf", "netf", "nsetups", "nli", "ncfl", "njtimes", "qlast",
             "qcur"]
    RSTATS = ["hlast", "hcur", "tcur", "hnext"]

    def __init__(self, rhs, t0, y0, rtol, atol, init_step, max_step=0.0, min_step=1e-6, max_num_steps=1000000,
                 maxl=0):
        L = lib()
        if not getattr(L, "_ode_bound", False):
            vp, d, lg = C.c_void_p, C.c_double, C.c_long
            L.oracle_ode_create_shud.restype = vp
            L.oracle_ode_create_shud.argtypes = [vp, lg, d, vp, d, d, d, d, d, lg, C.c_int]
            L.oracle_ode_create_test.restype = vp
            L.oracle_ode_create_test.argtypes = [C.c_int, lg, d, vp, d, d, d, d, d, lg, C.c_int]
            L.oracle_ode_solve.restype = C.c_int
            L.oracle_ode_solve.argtypes = [vp, d, vp, C.POINTER(d), C.c_int]
            L.oracle_ode_get_dky.restype = C.c_int
            L.oracle_ode_get_dky.argtypes = [vp, d, C.c_int, vp]
            L.oracle_ode_set_stop_time.argtypes = [vp, d]
            L.oracle_ode_get_stats.argtypes = [vp, vp, vp]
            L.oracle_ode_destroy.argtypes = [vp]
            L.oracle_ode_set_reduction_order.argtypes = [C.c_int]
            L._ode_bound = True
        self._y0 = np.ascontiguousarray(y0, dtype=np.float64).copy()
        self.n = self._y0.size
        args = (float(t0), self._y0.ctypes.data, float(rtol), float(atol), float(init_step), float(max_step),
                float(min_step), int(max_num_steps), int(maxl))
        if isinstance(rhs, str):
            prob = {"robertson": 1, "decay": 2, "decayn": 3}[rhs]
            self.h = L.oracle_ode_create_test(prob, self.n, *args)
        else:
            self._rhs = rhs                                   # keep the OracleRhs alive
            self.h = L.oracle_ode_create_shud(rhs.h, self.n, *args)
        if not self.h:
            raise ValueError("oracle_ode_create: invalid options")

    @staticmethod
    def set_reduction_order(order):
        """0: serial N_Vector order (CVODE's); 1: the device integrator's fixed blocked order"""
        lib().oracle_ode_set_reduction_order(int(order))

    def set_stop_time(self, tstop):
        lib().oracle_ode_set_stop_time(self.h, float(tstop))

    def solve(self, tout, one_step=False):
        """CVode(mem, tout, y, &t, CV_NORMAL | CV_ONE_STEP) -> (flag, t, y)"""
        y = np.empty(self.n)
        t = C.c_double()
        flag = lib().oracle_ode_solve(self.h, float(tout), y.ctypes.data, C.byref(t), 2 if one_step else 1)
        return flag, t.value, y

    def get_dky(self, t, k):
        d = np.empty(self.n)
        flag = lib().oracle_ode_get_dky(self.h, float(t), int(k), d.ctypes.data)
        return flag, d

    def stats(self):
        c = (C.c_long * 16)()
        r = (C.c_double * 8)()
        lib().oracle_ode_get_stats(self.h, c, r)
        out = {k: c[i] for i, k in enumerate(self.STATS)}
        out.update({k: r[i] for i, k in enumerate(self.RSTATS)})
        return out

    def __del__(self):
        try:
            if self.h:
                lib().oracle_ode_destroy(self.h)
                self.h = None
        except Exception:  # noqa: BLE001
            pass
