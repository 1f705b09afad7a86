"""CPU: the C-ABI library loads and exports every function include/shud_rhs.h declares; ctypes mirrors
match the header.  No compute calls (no GPU here)."""
import ctypes as C
import os
import re
import subprocess

from conftest import ROOT
from shud_rhs import abi

HEADER = os.path.join(ROOT, "include", "shud_rhs.h")
LIB = os.path.join(ROOT, "shud-up_amd", "libshud_rhs.so")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(shud_rhs_\w+)\s*\(", txt)))


def test_header_functions_all_bound():
    names = header_functions()
    assert len(names) >= 20
    assert set(names) == set(abi.FUNCTIONS), set(names) ^ set(abi.FUNCTIONS)


def test_library_exports_every_symbol():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "shud-up_amd")])
    lib = C.CDLL(LIB)
    for n in header_functions():
        assert hasattr(lib, n), n
    abi.bind(lib)
    assert lib.shud_rhs_abi_version() == 1


def _c_sizeof(struct):
    src = f'#include "shud_rhs.h"\n#include <stdio.h>\nint main(){{printf("%zu\\n", sizeof({struct}));return 0;}}\n'
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
                      ("ShudPartition", abi.ShudPartition)]:
        assert C.sizeof(cls) == _c_sizeof(name), name
