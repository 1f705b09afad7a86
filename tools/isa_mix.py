#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S (gfx950) listing.

usage: isa_mix.py listing.s mangled-name-substring [--dump]
Counts VALU (by opcode family), SALU, VMEM, LDS, SMEM and branches between the kernel's label and its .Lfunc_end.
"""
import collections
import re
import sys


def body(path, key):
    out, on = [], False
    for line in open(path):
        if not on and line.startswith("_Z") and key in line.split(":")[0]:
            on = True
            continue
        if on:
            if line.startswith(".Lfunc_end"):
                break
            out.append(line.rstrip("\n"))
    return out


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = body(path, key)
    cnt = collections.Counter()
    fam = collections.Counter()
    for l in lines:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        if op.startswith("v_"):
            cnt["VALU"] += 1
            fam[op] += 1
        elif op.startswith("s_"):
            if op.startswith("s_load") or op.startswith("s_buffer"):
                cnt["SMEM"] += 1
            elif op.startswith("s_cbranch") or op.startswith("s_branch"):
                cnt["BRANCH"] += 1
            elif op.startswith("s_waitcnt") or op.startswith("s_nop"):
                cnt["WAIT"] += 1
            else:
                cnt["SALU"] += 1
        elif op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
            cnt["VMEM"] += 1
        elif op.startswith("ds_"):
            cnt["LDS"] += 1
        else:
            cnt["other:" + op] += 1
    print(dict(cnt))
    for k, v in fam.most_common(60):
        print(f"{v:5d} {k}")
    if "--dump" in sys.argv:
        print("\n".join(lines))


if __name__ == "__main__":
    main()
