"""Audit of the register-dequant GEMM's inline-asm LDS reads (gemm_q.hip: qd_read / ReadRows): between an asm
ds_read and the lgkmcnt wait that retires it, no other instruction may touch its destination registers (hipcc
treats an asm result as available at once; a copy or reuse before the wait reads / loses the data).
Usage: python tools/audit_lds_asm.py [build/gemm_q-hip-amdgcn-amd-amdhsa-gfx950.s]"""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "ace-step-1.5-ggml_amd/build/gemm_q-hip-amdgcn-amd-amdhsa-gfx950.s"
s = open(path).read()


def regs_of(text):
    used = set()
    for a, b, c in re.findall(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", text):
        if c:
            used.add(int(c))
        else:
            used.update(range(int(a), int(b) + 1))
    return used


bad = 0
names = re.findall(r"^(_ZN5acemi11gemm_detail14gemm_qr_kernel[A-Za-z0-9_]*):", s, re.M)
for name in names:
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    body = [l.split(";")[0].strip() for l in s[i:j].splitlines()]
    body = [l for l in body if l and not l.startswith(".")]
    pend = []  # (dest regs, line index, text)
    for k, l in enumerate(body):
        m = re.search(r"lgkmcnt\((\d+)\)", l) if l.startswith("s_waitcnt") else None
        if m:  # LDS operations retire in order: at most N remain outstanding
            n = int(m.group(1))
            pend = pend[len(pend) - n:] if n > 0 else []
            continue
        if pend:
            ops = l.split(None, 1)
            if len(ops) == 2:
                touched = regs_of(ops[1])
                for d, k0, t0 in pend:
                    if touched & d:
                        bad += 1
                        if bad <= 20:
                            print(name[40:110], "|", t0, "->", l)
                        break
        if l.startswith("ds_read"):
            dest = regs_of(l.split(",")[0])
            pend.append((dest, k, l))
        elif l.startswith(("ds_write", "ds_add", "ds_bpermute", "ds_swizzle", "s_load", "s_buffer_load")):
            pend.append((set(), k, l))  # counts toward lgkmcnt
print(f"{len(names)} kernels, {bad} touches of in-flight asm LDS read destinations")
