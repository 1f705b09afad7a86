"""Print per-kernel VGPR / spill / occupancy for a HIP source (hipcc -Rpass-analysis=kernel-resource-usage)."""
import re, subprocess, sys, os
src = sys.argv[1]
extra = sys.argv[2:]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       f"-I{root}/include", f"-I{root}/shud-up_amd/csrc", "-c", src, "-o", "/tmp/_kres.o",
       "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m: continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip(); rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1); rows[cur][k.strip()] = v.strip()
for k, r in rows.items():
    name = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
    name = re.sub(r"shud::|DevMesh|DevPacked|YView|DevDiag|double\*|, ", lambda x: "" if x.group(0) != ", " else ",", name)
    print(f"{r.get('VGPRs','?'):>4} vgpr  spill {r.get('VGPRs Spill','?'):>3}/{r.get('SGPRs Spill','?'):<3} "
          f"occ {r.get('Occupancy [waves/SIMD]','?')}  {name[:110]}")
