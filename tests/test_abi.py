"""CPU: the C-ABI library loads and exports every function include/*.h declares; ctypes mirrors
match the header.  No compute calls (no GPU here)."""
import ctypes as C
import os
import re
import subprocess

from conftest import ROOT
from shud_rhs import abi

HEADERS = {"shud_rhs.h": ("shud_rhs_", abi.FUNCTIONS), "shud_et.h": ("shud_et_", abi.ET_FUNCTIONS),
           "shud_ode.h": ("shud_ode_", abi.ODE_FUNCTIONS), "shud_out.h": ("shud_(?:out|rhs)_", abi.OUT_FUNCTIONS)}
LIB = os.path.join(ROOT, "shud-up_amd", "libshud_rhs.so")


def header_functions(header=None):
    names = set()
    for h, (prefix, _) in HEADERS.items():
        if header and h != header:
            continue
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"\b(" + prefix + r"\w+)\s*\(", txt))
    return sorted(names)


def test_header_functions_all_bound():
    for h, (_, table) in HEADERS.items():
        names = header_functions(h)
        assert len(names) >= 4
        assert set(names) == set(table), (h, set(names) ^ set(table))


def test_library_exports_every_symbol():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "shud-up_amd")])
    lib = C.CDLL(LIB)
    for n in header_functions():
        assert hasattr(lib, n), n
    abi.bind(lib)
    assert lib.shud_rhs_abi_version() == 2


def _c_sizeof(struct):
    src = f'#include "shud_rhs.h"\n#include "shud_et.h"\n#include "shud_ode.h"\n#include "shud_out.h"\n#include <stdio.h>\nint main(){{printf("%zu\\n", sizeof({struct}));return 0;}}\n'
    exe = f"/tmp/sz_{struct}_{os.getpid()}"
    subprocess.run(["gcc", "-x", "c", "-", "-I", os.path.join(ROOT, "include"), "-o", exe], input=src.encode(),
                   check=True)
    out = subprocess.check_output([exe]).decode().strip()
    os.unlink(exe)
    return int(out)


def test_struct_layouts_match_header():
    for name, cls in [("ShudMeshSoA", abi.ShudMeshSoA), ("ShudParamsSoA", abi.ShudParamsSoA),
                      ("ShudStepInputs", abi.ShudStepInputs), ("ShudRhsOptions", abi.ShudRhsOptions),
                      ("ShudFluxOut", abi.ShudFluxOut), ("ShudErr", abi.ShudErr),
                      ("ShudPartition", abi.ShudPartition), ("ShudEtMeshSoA", abi.ShudEtMeshSoA),
                      ("ShudEtParams", abi.ShudEtParams), ("ShudEtForcing", abi.ShudEtForcing),
                      ("ShudEtOut", abi.ShudEtOut), ("ShudOdeOptions", abi.ShudOdeOptions),
                      ("ShudOdeStats", abi.ShudOdeStats), ("ShudPrintSpec", abi.ShudPrintSpec)]:
        assert C.sizeof(cls) == _c_sizeof(name), name


def test_host_library_exports_partition_symbols():
    """libshud_host.so exports every function include/shud_partition.h and shud_host.h declare; the ctypes
    mirrors of ShudPartStats / ShudPlanInfo match the C layout."""
    from shud_rhs import partition
    lib_path = os.path.join(ROOT, "shud-up_amd", "libshud_host.so")
    if not os.path.exists(lib_path):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "shud-up_amd"), "libshud_host.so"])
    lib = C.CDLL(lib_path)
    for h, prefix in (("shud_partition.h", r"shud_(?:partition|plan)_"), ("shud_host.h", r"shud_project_")):
        txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", h)).read(), flags=re.S)
        names = set(re.findall(r"\b(" + prefix + r"\w+)\s*\(", txt))
        assert len(names) >= 5, h
        for n in names:
            assert hasattr(lib, n), n
    partition._host()                     # binds every partitioner symbol with its signature
    for name, cls in (("ShudPartStats", partition.ShudPartStats), ("ShudPlanInfo", partition.ShudPlanInfo)):
        src = (f'#include "shud_partition.h"\n#include <stdio.h>\n'
               f'int main(){{printf("%zu\\n", sizeof({name}));return 0;}}\n')
        exe = f"/tmp/sz_{name}_{os.getpid()}"
        subprocess.run(["gcc", "-x", "c", "-", "-I", os.path.join(ROOT, "include"), "-o", exe], input=src.encode(),
                       check=True)
        out = int(subprocess.check_output([exe]).decode().strip())
        os.unlink(exe)
        assert out == C.sizeof(cls), (name, out, C.sizeof(cls))
