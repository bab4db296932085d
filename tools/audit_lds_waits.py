"""Static audit (CPU): in every loop of the kernels of a save-temps .s file, find instructions that READ a VGPR whose
inline-asm ds_read result may still be in flight (issued, not yet retired by an s_waitcnt lgkmcnt) -- the compiler
cannot see that an asm ds_read's output arrives late, so a consumer it schedules above the wait reads stale data.
DS reads retire in order: lgkmcnt(N) retires all but the N youngest.  The loop body is walked twice (wrap-around).
Usage: python tools/audit_lds_waits.py file.s [kernel-substring]"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(s):
    out = set()
    for m in REG.finditer(s):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def audit(name, body):
    pending = []  # list of sets (in issue order) of VGPRs written by outstanding ds_reads
    bad = []
    for rnd in range(2):
        for ln, l in body:
            s = l.strip()
            if not s or s.startswith((";", ".")):
                continue
            op = s.split()[0]
            args = s[len(op):].split(";")[0]
            if op == "s_waitcnt":
                m = re.search(r"lgkmcnt\((\d+)\)", args)
                if m:
                    n = int(m.group(1))
                    pending = pending[len(pending) - n:] if n < len(pending) else pending
                    if n == 0:
                        pending = []
                continue
            if op.startswith("ds_read") or op.startswith("ds_bpermute"):
                parts = [p.strip() for p in args.split(",")]
                dst, srcs = regs(parts[0]), set().union(*[regs(p) for p in parts[1:]]) if len(parts) > 1 else set()
                live = set().union(*pending) if pending else set()
                if srcs & live and rnd == 1:
                    bad.append((ln, s, sorted(srcs & live)))
                pending.append(dst)
                continue
            if op.startswith("s_") or op.startswith("ds_") and not op.startswith("ds_read"):
                # LDS writes / scalar ops: count DS writes as LGKM ops too (they retire in order with reads)
                if op.startswith("ds_"):
                    pending.append(set())
                continue
            parts = [p.strip() for p in args.split(",")]
            if not parts or not parts[0]:
                continue
            srcs = set().union(*[regs(p) for p in parts[1:]]) if len(parts) > 1 else set()
            if op.startswith(("buffer_", "global_", "scratch_")) and "store" in op:
                srcs |= regs(parts[0])
            live = set().union(*pending) if pending else set()
            hit = srcs & live
            if hit and rnd == 1:
                bad.append((ln, s, sorted(hit)))
            # a write to a pending register: the ds_read result will still overwrite it later (also a bug)
            dst = regs(parts[0]) if not op.startswith(("buffer_", "global_")) else set()
            if dst & live and rnd == 1 and not op.startswith("v_mfma"):
                bad.append((ln, s + "   [WAW with in-flight ds_read]", sorted(dst & live)))
    return bad


def main(path, pat=""):
    lines = open(path).read().split("\n")
    cur, start = None, 0
    funcs = []
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            cur, start = m.group(1), i
        if cur and l.startswith(".Lfunc_end"):
            funcs.append((cur, start, i))
            cur = None
    total = 0
    for name, a, b in funcs:
        if pat and pat not in name:
            continue
        text = lines[a:b]
        for i, l in enumerate(text):
            m = re.match(r"^(\.LBB\d+_\d+):", l)
            if not m or not ("Loop Header" in l or (i + 1 < len(text) and "Loop Header" in text[i + 1])):
                continue
            lab = m.group(1)
            for j in range(i + 1, len(text)):
                if re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\b", text[j]):
                    body = [(a + k + 1, text[k]) for k in range(i, j + 1)]
                    for ln, s, r in audit(name, body)[:6]:
                        print(f"{name[:90]} {lab} line {ln}: {s[:90]}  regs {r[:6]}")
                        total += 1
                    break
    print(f"{total} findings")


if __name__ == "__main__":
    main(*sys.argv[1:])
