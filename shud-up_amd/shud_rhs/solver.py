"""SHUD()'s time loop on the device (src/Model/shud.cpp:89-131).

`ShudSolver` drives, per solver step, the device ET prelude (updateforcing/tReadForcing + ET(t, tout),
MD_ET.cpp:14-341, include/shud_et.h) and then the device integrator (CVode(mem, tout, y, &t, CV_NORMAL),
include/shud_ode.h) over an RhsHandle.  State, step inputs and the Nordsieck history stay in HBM; only the
per-interval forcing rows (host bookkeeping in the reference too) and the requested outputs cross PCIe.

Control settings are the reference's Model_Control fields (Model_Control.hpp:176-182, .cpp:137,502):
SolverStep = MaxStep, NumSteps = (END - START)/SolverStep, ET sub-stepping when ETStep < SolverStep.
"""
from dataclasses import dataclass

import numpy as np

from . import abi
from .runtime import OdeSolver, ShudRhsError

ZERO = 1.0e-10                      # Macros.hpp:32


@dataclass
class SolverControl:
    reltol: float = 1.0e-3          # Model_Control.hpp:177 defaults; ccw/heihe/qhh cfg.para use 1e-4
    abstol: float = 1.0e-4
    init_step: float = 1.0e-2
    max_step: float = 30.0
    et_step: float = 60.0
    start: float = 0.0
    min_step: float = 1.0e-6        # SetCVODE (cvode_config.cpp:182)
    max_num_steps: int = 1000000    # SetCVODE (cvode_config.cpp:185)

    @property
    def solver_step(self):          # Model_Control.cpp:502
        return self.max_step

    @property
    def et_substep(self):           # shud.cpp:86-87
        return self.et_step > ZERO and self.et_step + ZERO < self.solver_step


class ShudSolver:
    """handle: RhsHandle with step inputs set (and shud_et_attach'ed when forcing is given).
    forcing(t, tout) -> et.EtForcing for the ET prelude of [t, tout), or None to keep the step inputs."""

    def __init__(self, handle, y0, ctl: SolverControl):
        self.h = handle
        self.ctl = ctl
        self.t = ctl.start
        self.ode = OdeSolver(handle, ctl.start, y0, ctl.reltol, ctl.abstol, ctl.init_step, ctl.max_step,
                             ctl.min_step, ctl.max_num_steps)
        self.y = None

    def run(self, num_steps, forcing=None, on_output=None, output=None):
        """num_steps solver steps (the reference's NumSteps loop); on_output(i, t, y) after each (host copy of y).
        output: runtime.Output whose controls point at the handle's device arrays — after each solver step
        summary(udata) + ExportResults(t) run on the device (shud.cpp:137,153): no host copy of y at all."""
        ctl = self.ctl
        tnext = self.t
        d_y = None
        if output is not None:
            d_y = self._out_y = getattr(self, "_out_y", None) or self.h.device_alloc(8 * self.h.num_y)
        for i in range(num_steps):
            tnext += ctl.solver_step
            while self.t + ZERO < tnext:
                tout = min(self.t + ctl.et_step, tnext) if ctl.et_substep else tnext
                if forcing is not None:
                    f = forcing(self.t, tout)
                    if f is not None:
                        self.h.et_step(f)
                if ctl.et_substep:
                    self.ode.set_stop_time(tout)
                if d_y is not None:
                    flag, t = self.ode.solve_device(tout, d_y)
                    y = None
                else:
                    flag, t, y = self.ode.solve(tout)
                if flag < 0:
                    if flag == abi.ODE_RHSFUNC_FAIL:
                        e = self.h.get_error()
                        if e["exit_code"]:
                            raise ShudRhsError(abi.SHUD_ERR_PHYSICS, e["message"], e)
                    raise RuntimeError(f"CVode failed with flag {flag} at t={t}")
                self.t, self.y = t, y
            if output is not None:
                # Model_Data::summary(udata) on y(tout); the flux arrays are those of CVODE's last f() call,
                # replayed on its input buffer (the integrator never rewrites that buffer before its next RHS
                # call: the Newton residual's y and the DQ work vector are only written right before an RHS)
                self.h.summary(d_y)
                self.h.refresh_diagnostics()
                output.export(self.t)
            if on_output is not None:
                if self.y is None:
                    self.y = self.h.d2h(np.empty(self.h.num_y), d_y)
                on_output(i, self.t, self.y)
        return self.t, self.y

    def stats(self):
        return self.ode.stats()

    def close(self):
        self.ode.close()
        if getattr(self, "_out_y", None):
            self.h.device_free(self._out_y)
            self._out_y = None
