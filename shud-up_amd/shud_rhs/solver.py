"""SHUD()'s time loop on the device (src/Model/shud.cpp:89-131).

`ShudSolver` drives, per solver step, the device ET prelude (updateforcing/tReadForcing + ET(t, tout),
MD_ET.cpp:14-341, include/shud_et.h) and then the device integrator (CVode(mem, tout, y, &t, CV_NORMAL),
include/shud_ode.h) over an RhsHandle.  State, step inputs and the Nordsieck history stay in HBM; only the
per-interval forcing rows (host bookkeeping in the reference too) and the requested outputs cross PCIe.

Control settings are the reference's Model_Control fields (Model_Control.hpp:176-182, .cpp:137,502):
SolverStep = MaxStep, NumSteps = (END - START)/SolverStep, ET sub-stepping when ETStep < SolverStep.
"""
from dataclasses import dataclass

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

    def run(self, num_steps, forcing=None, on_output=None):
        """num_steps solver steps (the reference's NumSteps loop); on_output(i, t, y) after each."""
        ctl = self.ctl
        tnext = self.t
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
                flag, t, y = self.ode.solve(tout)
                if flag < 0:
                    if flag == abi.ODE_RHSFUNC_FAIL:
                        e = self.h.get_error()
                        if e["exit_code"]:
                            raise ShudRhsError(abi.SHUD_ERR_PHYSICS, e["message"], e)
                    raise RuntimeError(f"CVode failed with flag {flag} at t={t}")
                self.t, self.y = t, y
            if on_output is not None:
                on_output(i, self.t, self.y)
        return self.t, self.y

    def stats(self):
        return self.ode.stats()

    def close(self):
        self.ode.close()
