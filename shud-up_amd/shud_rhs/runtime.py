"""ctypes front end of libshud_rhs.so — the product path.  Fails loudly if the HIP library is absent.

`RhsHandle` mirrors the reference call sequence: construct once from a ShudModel (Model_Data after
initialize(), MD_initialize.cpp:168-245), `set_step_inputs` once per ET step (updateforcing()/ET(),
MD_ET.cpp:14-342), then `eval(t, y)` per CVODE RHS call (f(), src/Model/f.cpp:2-32).
"""
import ctypes as C
import os

import numpy as np

from . import abi

_LIB = None
LIB_PATH = os.environ.get("SHUD_RHS_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "libshud_rhs.so")   # env: A/B builds only


class ShudRhsError(RuntimeError):
    def __init__(self, code, msg, err=None):
        super().__init__(f"shud_rhs error {code}: {msg}")
        self.code = code
        self.err = err


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"HIP library {LIB_PATH} not built: run `make -C shud-up_amd` "
                              "or __graft_entry__.build() (there is no CPU fallback)")
        _LIB = abi.bind(C.CDLL(LIB_PATH))
    return _LIB


def _check(rc, what):
    if rc != abi.SHUD_OK:
        raise ShudRhsError(rc, f"{what}: {lib().shud_rhs_last_error_string().decode(errors='replace')}")


class RhsHandle:
    def __init__(self, model, mode=abi.SHUD_MODE_SERIAL, device=0, stream=None, check_errors=True,
                 partition=None):
        self.model = model
        self._mesh = model.mesh_struct()
        self._par = model.params_struct()
        opt = abi.ShudRhsOptions(mode, device, stream, 1 if check_errors else 0)
        h = C.c_void_p()
        if partition is None:
            _check(lib().shud_rhs_create(C.byref(self._mesh), C.byref(self._par), C.byref(opt), C.byref(h)),
                   "shud_rhs_create")
            self.n_own, self.n_own_riv = model.num_ele, model.num_riv
            self.n_lake = getattr(model, "num_lake", 0)
        else:
            self._part = partition.struct()
            _check(lib().shud_rhs_create_partitioned(C.byref(self._mesh), C.byref(self._par), C.byref(opt),
                                                     C.byref(self._part), C.byref(h)),
                   "shud_rhs_create_partitioned")
            self.n_own, self.n_own_riv = partition.n_own_ele, partition.n_own_riv
            self.n_lake = getattr(model, "num_lake", 0)   # the local mesh carries the owned lakes
        self.h = h
        self.mode = mode

    @property
    def num_y(self):
        return 3 * self.n_own + self.n_own_riv + self.n_lake

    def close(self):
        if self.h:
            lib().shud_rhs_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_step_inputs(self, step=None, bc_tables=None):
        s = self.model.step_struct(step, bc_tables)
        _check(lib().shud_rhs_set_step_inputs(self.h, C.byref(s)), "shud_rhs_set_step_inputs")

    def eval(self, t, y, ydot=None, raise_on_physics=True):
        """Host-array RHS: returns ydot (numpy).  Raises ShudRhsError on a physics error (the reference
        would have exited; the error details are in .err)."""
        y = np.ascontiguousarray(y, dtype=np.float64)
        if y.size != self.num_y:
            raise ValueError(f"y has {y.size} entries, expected {self.num_y}")
        if ydot is None:
            ydot = np.empty_like(y)
        rc = lib().shud_rhs_eval(self.h, float(t), y.ctypes.data, ydot.ctypes.data, abi.SHUD_WHERE_HOST)
        if rc == abi.SHUD_ERR_PHYSICS and raise_on_physics:
            e = self.get_error()
            raise ShudRhsError(rc, e["message"], e)
        if rc not in (abi.SHUD_OK, abi.SHUD_ERR_PHYSICS):
            _check(rc, "shud_rhs_eval")
        return ydot

    def eval_device(self, t, d_y, d_ydot):
        """Stream-ordered eval on device pointers (ints)."""
        _check(lib().shud_rhs_eval(self.h, float(t), C.c_void_p(d_y), C.c_void_p(d_ydot), abi.SHUD_WHERE_DEVICE),
               "shud_rhs_eval(device)")

    def get_error(self):
        e = abi.ShudErr()
        _check(lib().shud_rhs_get_error(self.h, C.byref(e)), "shud_rhs_get_error")
        return {"flags": e.flags, "exit_code": e.exit_code, "first_index": list(e.first_index),
                "n_aet_warn": e.n_aet_warn, "message": e.message.decode(errors="replace")}

    def clear_error(self):
        _check(lib().shud_rhs_clear_error(self.h), "shud_rhs_clear_error")

    def num_calls(self):
        return lib().shud_rhs_num_calls(self.h)

    def layout(self):
        pk, nc, ns = C.c_int(), C.c_int(), C.c_int()
        _check(lib().shud_rhs_layout(self.h, C.byref(pk), C.byref(nc)), "shud_rhs_layout")
        _check(lib().shud_rhs_layout_streamed(self.h, C.byref(ns)), "shud_rhs_layout_streamed")
        sh = C.c_int()
        if hasattr(lib(), "shud_rhs_layout_shared"):     # (A/B builds of older sources lack it)
            _check(lib().shud_rhs_layout_shared(self.h, C.byref(sh)), "shud_rhs_layout_shared")
        out = {"packed": bool(pk.value), "n_classes": nc.value}
        if ns.value:
            out["streamed_fields"] = ns.value
        if sh.value:
            out["shared_edges"] = sh.value
        return out

    def diagnostics(self):
        m = self.model
        NE, NR, NS = m.num_ele, m.num_riv, m.num_seg
        out = {}
        o = abi.ShudFluxOut()
        for name in abi.FLUXOUT_ORDER:
            n = (3 * NE if name in abi.DIAG_ELE3 else NS if name in abi.DIAG_SEG else NR if name in abi.DIAG_RIV
                 else getattr(m, "num_lake", 0) if name in abi.DIAG_LAKE else NE)
            out[name] = np.zeros(n)
            setattr(o, name, out[name].ctypes.data_as(abi.c_double_p))
        _check(lib().shud_rhs_sync_diagnostics(self.h, C.byref(o)), "shud_rhs_sync_diagnostics")
        return out

    # ---- device memory helpers (bench / tests without torch) ----
    def device_alloc(self, nbytes):
        p = C.c_void_p()
        _check(lib().shud_rhs_device_alloc(self.h, nbytes, C.byref(p)), "device_alloc")
        return p.value

    def device_free(self, p):
        _check(lib().shud_rhs_device_free(self.h, C.c_void_p(p)), "device_free")

    def h2d(self, dptr, arr):
        arr = np.ascontiguousarray(arr)
        _check(lib().shud_rhs_memcpy(self.h, C.c_void_p(dptr), arr.ctypes.data, arr.nbytes, 1), "memcpy H2D")

    def d2h(self, arr, dptr):
        _check(lib().shud_rhs_memcpy(self.h, arr.ctypes.data, C.c_void_p(dptr), arr.nbytes, 2), "memcpy D2H")
        return arr

    def synchronize(self):
        _check(lib().shud_rhs_synchronize(self.h), "synchronize")

    def stream(self):
        return lib().shud_rhs_stream(self.h)

    def time_kernels(self, t, d_y, d_ydot, reps):
        ms_eval = C.c_double()
        ms = (C.c_double * 8)()
        nk = C.c_int(8)
        names = C.create_string_buffer(256)
        _check(lib().shud_rhs_time_kernels(self.h, float(t), C.c_void_p(d_y), C.c_void_p(d_ydot), int(reps),
                                           C.byref(ms_eval), ms, C.byref(nk), names, 256), "time_kernels")
        nm = names.value.decode().split(",")
        return ms_eval.value, {nm[k]: ms[k] for k in range(nk.value)}

    def timing(self, max_evals, stride=1):
        """record per-kernel HIP events in every `stride`-th of the next evals, up to `max_evals` of them
        (shud_rhs_timing)"""
        _check(lib().shud_rhs_timing(self.h, int(max_evals), int(stride)), "timing")

    def timing_read(self):
        """(ms_ele, ms_riv, ms_eval, n): per-eval averages of the evals recorded since timing()"""
        a, b, c, n = C.c_double(), C.c_double(), C.c_double(), C.c_int()
        _check(lib().shud_rhs_timing_read(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(n)), "timing_read")
        return a.value, b.value, c.value, n.value

    # ---- output path (include/shud_out.h) ----
    def summary(self, d_y):
        """Model_Data::summary(udata) on the device: SHUD_ARR_Y_* from the state at d_y"""
        _check(lib().shud_rhs_summary(self.h, C.c_void_p(d_y)), "summary")

    def refresh_diagnostics(self):
        """the last RHS evaluation replayed with diagnostic stores into the device arrays (no host copy)"""
        _check(lib().shud_rhs_refresh_diagnostics(self.h), "refresh_diagnostics")

    def prepare_outputs(self):
        """allocate every device output array (zeros) without evaluating anything (shud_rhs_prepare_outputs)"""
        _check(lib().shud_rhs_prepare_outputs(self.h), "prepare_outputs")

    def device_array(self, which):
        n = C.c_int64()
        p = lib().shud_rhs_device_array(self.h, int(which), C.byref(n))
        return p, n.value

    # ---- external-transport partition hooks ----
    def halo_buffers(self):
        p = [C.c_void_p() for _ in range(4)]
        _check(lib().shud_rhs_halo_buffers(self.h, *[C.byref(x) for x in p]), "halo_buffers")
        return [x.value for x in p]

    # ---- ET-step prelude (include/shud_et.h) ----
    def et_attach(self, etm):
        self._et_mesh = etm.mesh_struct()
        self._et_par = etm.params_struct()
        _check(lib().shud_et_attach(self.h, C.byref(self._et_mesh), C.byref(self._et_par)), "shud_et_attach")

    def et_set_state(self, y_is=None, y_snow=None):
        a = None if y_is is None else np.ascontiguousarray(y_is, dtype=np.float64)
        b = None if y_snow is None else np.ascontiguousarray(y_snow, dtype=np.float64)
        _check(lib().shud_et_set_state(self.h, None if a is None else a.ctypes.data,
                                       None if b is None else b.ctypes.data), "shud_et_set_state")

    def et_step(self, forcing, raise_on_physics=True):
        fs = forcing.struct()
        rc = lib().shud_et_step(self.h, C.byref(fs))
        if rc == abi.SHUD_ERR_PHYSICS and raise_on_physics:
            e = self.get_error()
            raise ShudRhsError(rc, e["message"], e)
        if rc not in (abi.SHUD_OK, abi.SHUD_ERR_PHYSICS):
            _check(rc, "shud_et_step")
        return rc

    def et_get(self):
        from .et import out_struct
        o, arrs = out_struct(self.model.num_ele)
        _check(lib().shud_et_get(self.h, C.byref(o)), "shud_et_get")
        return arrs

    def eval_pack(self, d_y):
        _check(lib().shud_rhs_eval_pack(self.h, C.c_void_p(d_y)), "eval_pack")

    def eval_compute(self, t, d_y, d_ydot):
        _check(lib().shud_rhs_eval_compute(self.h, float(t), C.c_void_p(d_y), C.c_void_p(d_ydot)), "eval_compute")

    def debug_halo(self, spin_us=0.0, d_ele_src=None, d_riv_src=None, publish=True, timeout_ms=0.0):
        """test hook (shud_rhs_debug_halo): late / kernel-written / missing halo on the comm stream"""
        _check(lib().shud_rhs_debug_halo(self.h, float(spin_us), C.c_void_p(d_ele_src), C.c_void_p(d_riv_src),
                                         1 if publish else 0, float(timeout_ms)), "debug_halo")


def nccl_unique_id():
    buf = C.create_string_buffer(128)
    _check(lib().shud_rhs_nccl_unique_id(buf), "nccl_unique_id")
    return buf.raw


class OdeSolver:
    """Device-resident CVODE-semantics integrator (include/shud_ode.h) over an RhsHandle, or over a raw device
    RHS function pointer (tests).  Mirrors SetCVODE (cvode_config.cpp:149-197) + CVode() as SHUD() calls it."""

    def __init__(self, rhs, t0, y0, reltol, abstol, init_step, max_step=0.0, min_step=1e-6,
                 max_num_steps=1000000, maxl=0, max_order=0, fn=None):
        self._opt = abi.ShudOdeOptions(reltol, abstol, init_step, max_step, min_step, max_num_steps, maxl, max_order)
        y0 = np.ascontiguousarray(y0, dtype=np.float64)
        self.n = y0.size
        h = C.c_void_p()
        if fn is None:
            self._rhs = rhs
            if self.n != rhs.num_y:
                raise ValueError(f"y0 has {self.n} entries, expected {rhs.num_y}")
            _check(lib().shud_ode_create(rhs.h, float(t0), y0.ctypes.data, abi.SHUD_WHERE_HOST, C.byref(self._opt),
                                         C.byref(h)), "shud_ode_create")
        else:                                   # fn = (function pointer, user pointer, stream)
            self._fn = fn
            _check(lib().shud_ode_create_fn(self.n, fn[0], fn[1], fn[2], float(t0), y0.ctypes.data,
                                            abi.SHUD_WHERE_HOST, C.byref(self._opt), C.byref(h)), "shud_ode_create_fn")
        self.h = h

    def set_stop_time(self, tstop):
        lib().shud_ode_set_stop_time(self.h, float(tstop))

    def solve(self, tout, one_step=False, y_out=True):
        """CVode(mem, tout, y, &t, CV_NORMAL | CV_ONE_STEP) -> (flag, t, y or None)"""
        y = np.empty(self.n) if y_out else None
        t = C.c_double()
        flag = lib().shud_ode_solve(self.h, float(tout), None if y is None else y.ctypes.data, abi.SHUD_WHERE_HOST,
                                    C.byref(t), abi.ODE_ONE_STEP if one_step else abi.ODE_NORMAL)
        return flag, t.value, y

    def solve_device(self, tout, d_y, one_step=False):
        """CVode() with y(t) written to device memory at d_y (NY doubles): -> (flag, t)"""
        t = C.c_double()
        flag = lib().shud_ode_solve(self.h, float(tout), C.c_void_p(d_y), abi.SHUD_WHERE_DEVICE, C.byref(t),
                                    abi.ODE_ONE_STEP if one_step else abi.ODE_NORMAL)
        return flag, t.value

    def get_dky(self, t, k):
        d = np.empty(self.n)
        flag = lib().shud_ode_get_dky(self.h, float(t), int(k), d.ctypes.data, abi.SHUD_WHERE_HOST)
        return flag, d

    def stats(self):
        s = abi.ShudOdeStats()
        lib().shud_ode_get_stats(self.h, C.byref(s))
        return {k: getattr(s, k) for k, _ in abi.ShudOdeStats._fields_}

    def state_device(self):
        return lib().shud_ode_state_device(self.h)

    def close(self):
        if self.h:
            lib().shud_ode_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class Output:
    """The reference's Print_Ctrl set (Control_Data::ExportResults, Model_Control.cpp:123-127) with its buffers
    in HBM (include/shud_out.h): add() = Print_Ctrl::Init[IJ] + open_file, export(t) = ExportResults(t)."""

    def __init__(self, device=0, stream=None):
        h = C.c_void_p()
        _check(lib().shud_out_create(int(device), None if stream is None else C.c_void_p(stream), C.byref(h)),
               "shud_out_create")
        self.h = h
        self._keep = []

    def add(self, basename, d_src, n_all, interval, iflux, start_time=0, flag_io=None, binary=True, ascii=False,
            radiation_input_mode=0, terrain_radiation=0, solar_lonlat_mode="FORCING_FIRST", lon=0.0, lat=0.0):
        flags = None if flag_io is None else np.ascontiguousarray(flag_io, dtype=np.int32)
        bn, sm = str(basename).encode(), str(solar_lonlat_mode).encode()
        spec = abi.ShudPrintSpec(bn, C.c_void_p(d_src), int(n_all), None if flags is None else flags.ctypes.data,
                                 int(interval), int(iflux), int(start_time), int(bool(binary)), int(bool(ascii)),
                                 int(radiation_input_mode), int(terrain_radiation), sm, float(lon), float(lat))
        _check(lib().shud_out_add(self.h, C.byref(spec)), "shud_out_add")
        self._keep.append((bn, sm, flags))
        return len(self._keep) - 1

    def export(self, t):
        _check(lib().shud_out_export(self.h, float(t)), "shud_out_export")

    def rows(self, k):
        return lib().shud_out_rows(self.h, int(k))

    def flush(self):
        """wait until every exported row is in the files (shud_out_flush)"""
        _check(lib().shud_out_flush(self.h), "shud_out_flush")

    def close(self):
        """shud_out_destroy; raises if the asynchronous writer failed (a lost row or a file write error)"""
        if self.h:
            rc = lib().shud_out_destroy(self.h)
            self.h = None
            _check(rc, "shud_out_destroy")

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
