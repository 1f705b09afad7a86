"""List scratch spill/reload sites (source file:line) of one kernel in a HIP source: python tools/spills.py src.hip kernel_substring [hipcc flags]"""
import re, subprocess, sys, os
src, kname = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                "-gline-tables-only", f"-I{root}/include", f"-I{root}/shud-up_amd/csrc", "--cuda-device-only", "-S",
                src, "-o", "/tmp/_spills.s"] + sys.argv[3:], check=True, capture_output=True)
s = open("/tmp/_spills.s").read()
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", s, re.M)]
name = next(n for n in names if kname in subprocess.run(["c++filt", n], capture_output=True, text=True).stdout)
a = s.index(name + ":"); b = s.index(".Lfunc_end", a)
files = {m.group(1): (m.group(3) or m.group(2)).split("/")[-1]
         for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s)}
cur = None
for l in s[a:b].splitlines():
    t = l.strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
    if m: cur = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"; continue
    if "scratch_" in t: print(cur, t[:70])
