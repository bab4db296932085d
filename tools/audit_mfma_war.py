"""Static audit of hipcc's gfx950 output (-save-temps .s): an MFMA's A/B source registers overwritten by an instruction
issued shortly after it (write-after-read on an in-flight MFMA's operands).

Found in round 5: in the register-dequant GEMM at two waves per SIMD, a VALU that wrote the A operand
register of the MFMA issued one instruction before it produced wrong 16-column groups on some launches (the v21 x Q4_K
anomaly of rounds 3-4); putting >= 9 wait states between them removed it.  Distances are counted in issue slots (s_nop N = N + 1).  hipcc pads this pair for the C operand only.
Usage: python tools/audit_mfma_war.py FILE.s [--window N] [--kernel SUBSTR] -> per kernel: pairs closer than N."""
import argparse
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def regs(tok):
    """set of (file, index) named by an operand like v[4:7], a12, v5"""
    out = set()
    for m in REG.finditer(tok):
        f = m.group(1)
        if m.group(4) is not None:
            out.add((f, int(m.group(4))))
        else:
            for i in range(int(m.group(2)), int(m.group(3)) + 1):
                out.add((f, i))
    return out


def split_ops(line):
    body = line.split(";")[0].strip()
    if not body or body.endswith(":") or body.startswith("."):
        return None, []
    parts = body.split(None, 1)
    op = parts[0]
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return op, ops


def writes(op, ops):
    """VGPR/AGPR destinations of an instruction (first operand of VALU / vector loads / LDS reads)"""
    if not ops:
        return set()
    if op.startswith(("s_", "global_store", "buffer_store", "ds_write", "flat_store", "scratch_store", "global_load_lds",
                      "buffer_load_dword_lds")) or op.startswith("v_cmp"):
        return set()
    if op.startswith(("v_", "ds_read", "global_load", "buffer_load", "flat_load", "scratch_load", "ds_bpermute",
                      "ds_permute", "ds_swizzle")):
        return regs(ops[0])
    return set()


def audit(path, window, ksub, valu_only=False):
    fn = None
    hist = {}
    recent = []  # (index, srcAB set) of recent MFMAs
    n = 0
    with open(path) as f:
        for line in f:
            s = line.rstrip("\n")
            if re.match(r"^[A-Za-z_.$][\w.$]*:", s) and not s.startswith("."):
                name = s.split(":")[0]
                if not name.startswith(".L"):
                    fn = name
                    recent = []
                continue
            if s.lstrip().startswith(".LBB"):
                continue
            op, ops = split_ops(s)
            if op is None:
                continue
            n += int(ops[0]) + 1 if op == "s_nop" and ops else 1  # distance in issue slots / wait states
            if fn is None or (ksub and ksub not in fn):
                continue
            w = writes(op, ops) if (not valu_only or op.startswith("v_")) else set()
            if w:
                for (idx, src) in recent:
                    d = n - idx
                    if d <= window and (w & src):
                        hist.setdefault(fn, []).append((d, op, ops[0]))
            if op.startswith("v_mfma"):
                recent.append((n, regs(ops[1]) | regs(ops[2]) if len(ops) > 2 else set()))
            recent = [(i, r) for (i, r) in recent if n - i < window]
    return hist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--window", type=int, default=8)
    ap.add_argument("--kernel", default="")
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--valu", action="store_true", help="only VALU writers (an LDS / memory load lands >= ~100 cycles later)")
    a = ap.parse_args()
    bad = 0
    for p in a.files:
        h = audit(p, a.window, a.kernel, a.valu)
        for fn, hits in sorted(h.items()):
            bad += len(hits)
            dmin = min(d for d, _, _ in hits)
            print(f"{p}: {fn[:110]}: {len(hits)} pairs, closest {dmin}")
            if a.v:
                for d, op, dst in hits[:8]:
                    print(f"    d={d} {op} {dst}")
    print(f"total pairs within {a.window}: {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
