"""Static audit of hipcc's gfx950 output (-save-temps .s): an MFMA's A/B (and block-scale) source registers overwritten
by a VALU issued shortly after it on some execution path (write-after-read on an in-flight MFMA's operands).

Found in round 5: in the register-dequant GEMM at two waves per SIMD, a VALU that wrote the A operand
register of the MFMA issued one instruction before it produced wrong 16-column groups on some launches (the v21 x Q4_K
anomaly of rounds 3-4); >= 9 wait states between them removed it.  hipcc pads this pair for the C operand only.

Round 6: the walk follows the control-flow graph.  Each function is split into basic blocks (labels start one, a
branch / s_endpgm ends one); successors are the branch target(s) plus the fall-through block unless the block ends in an
unconditional `s_branch` or `s_endpgm`.  From every MFMA the audit walks all paths forward until the distance exceeds the
window, so loader-wave code that merely FOLLOWS the MFMA-wave code in the file (warp-specialised kernels branch on the
wave id) is no longer paired with it.  Distances are counted in issue slots (`s_nop N` = N + 1 wait states).

Every remaining pair is classified by the kernel's occupancy (`; Occupancy: N` that hipcc prints per kernel, the waves
per SIMD its register count allows):
  * exposed  -- N >= 2: a second wave can share the SIMD, the condition under which the hazard was observed; such a
               pair is a defect (guard it: gemm_common.h mfma_war_guard, or restructure).
  * single   -- N == 1: the kernel can never have a partner wave on its SIMD (registers > 256 per lane), the hazard's
               precondition never holds; reported, not a defect.
Usage: python tools/audit_mfma_war.py FILE.s [...] [--window N] [--kernel SUBSTR] [-v] [--all]
Exit status 1 when an exposed pair exists (--all: any pair)."""
import argparse
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")
LABEL = re.compile(r"^([A-Za-z_.$][\w.$]*):")


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
    if op.startswith("v_mfma"):
        return set()  # the matrix pipe runs in order: a later MFMA writes its result after an earlier one read its sources
    if op.startswith(("s_", "global_store", "buffer_store", "ds_write", "flat_store", "scratch_store", "global_load_lds",
                      "buffer_load_dword_lds")) or op.startswith("v_cmp"):
        return set()
    if op.startswith(("v_", "ds_read", "global_load", "buffer_load", "flat_load", "scratch_load", "ds_bpermute",
                      "ds_permute", "ds_swizzle")):
        return regs(ops[0])
    return set()


def mfma_sources(op, ops):
    """registers an MFMA reads besides its accumulator: A, B and, for the block-scaled forms, the two scale VGPRs"""
    src = set()
    if len(ops) > 2:
        src = regs(ops[1]) | regs(ops[2])
    if op.startswith("v_mfma_scale") and len(ops) > 5:
        src |= regs(ops[4]) | regs(ops[5].split()[0])
    return src


class Func:
    def __init__(self, name):
        self.name = name
        self.blocks = []      # list of [label or None, [(op, ops, cost)], succ labels, falls_through]
        self.occupancy = None


def parse(path):
    """functions of a .s: basic blocks with their instructions and successors, plus hipcc's occupancy line"""
    funcs = {}
    fn = None
    cur = None
    with open(path) as f:
        for lineno, line in enumerate(f, 1):
            s = line.rstrip("\n")
            m = LABEL.match(s)
            if m and not s.startswith("."):
                fn = Func(m.group(1))
                funcs[fn.name] = fn
                cur = [None, [], [], True]
                fn.blocks.append(cur)
                continue
            if m and m.group(1).startswith(".LBB") and fn is not None:
                cur = [m.group(1), [], [], True]
                fn.blocks.append(cur)
                continue
            if s.startswith("; Occupancy:") and fn is not None:
                fn.occupancy = int(s.split(":")[1])
                continue
            if s.strip().startswith("; %bb.") and fn is not None and cur is not None and cur[1]:
                cur = [None, [], [], True]  # hipcc's un-labelled fall-through block start: same flow
                fn.blocks.append(cur)
                continue
            op, ops = split_ops(s)
            if op is None or fn is None or cur is None:
                continue
            cost = int(ops[0], 0) + 1 if op == "s_nop" and ops else 1
            cur[1].append((op, ops, cost, lineno))
            if op == "s_branch":
                cur[2].append(ops[0])
                cur[3] = False
                cur = [None, [], [], True]
                fn.blocks.append(cur)
            elif op.startswith("s_cbranch"):
                cur[2].append(ops[0])
                cur = [None, [], [], True]
                fn.blocks.append(cur)
            elif op in ("s_endpgm", "s_setpc_b64"):
                cur[3] = False
                cur = [None, [], [], True]
                fn.blocks.append(cur)
    return funcs


def audit_func(fn, window, valu_only=True):
    """[(distance, mfma, writer op, writer dst)] for every path-feasible VALU write to an in-flight MFMA's sources"""
    blocks = [b for b in fn.blocks if b[1] or b[0]]
    index = {b[0]: i for i, b in enumerate(blocks) if b[0]}
    succ = []
    for i, b in enumerate(blocks):
        s = [index[t] for t in b[2] if t in index]
        if b[3] and i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)
    hits = []
    for bi, b in enumerate(blocks):
        for ii, (op, ops, _, mline) in enumerate(b[1]):
            if not op.startswith("v_mfma"):
                continue
            src = mfma_sources(op, ops)
            if not src:
                continue
            # walk forward: (block, start index, distance so far); best distance seen per (block, index) prunes revisits
            seen = {}
            stack = [(bi, ii + 1, 0)]
            while stack:
                cb, ci, d = stack.pop()
                if seen.get((cb, ci), window + 1) <= d:
                    continue
                seen[(cb, ci)] = d
                insts = blocks[cb][1]
                stop = False
                while ci < len(insts):
                    wop, wops, cost, wline = insts[ci]
                    d += cost
                    if d > window:
                        stop = True
                        break
                    w = writes(wop, wops) if (not valu_only or wop.startswith("v_")) else set()
                    if w & src:
                        hits.append((d, op, wop, wops[0], mline, wline))
                    ci += 1
                if not stop:
                    for nb in succ[cb]:
                        stack.append((nb, 0, d))
    return hits


def audit(path, window=8, ksub="", valu_only=True):
    """{kernel: (occupancy, hits)} for every function of the file with at least one hit"""
    out = {}
    for name, fn in parse(path).items():
        if ksub and ksub not in name:
            continue
        h = audit_func(fn, window, valu_only)
        if h:
            out[name] = (fn.occupancy, h)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--window", type=int, default=8)
    ap.add_argument("--kernel", default="")
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--loads", action="store_true", help="also count LDS / memory load destinations (they land >= ~100 "
                    "cycles later, so by default only VALU writers are audited)")
    ap.add_argument("--all", action="store_true", help="fail on single-wave kernels' pairs too")
    a = ap.parse_args()
    exposed = single = 0
    for p in a.files:
        for fn, (occ, hits) in sorted(audit(p, a.window, a.kernel, not a.loads).items()):
            cls = "exposed" if (occ or 1) >= 2 else "single"
            if cls == "exposed":
                exposed += len(hits)
            else:
                single += len(hits)
            dmin = min(h[0] for h in hits)
            print(f"{p}: {fn[:110]}: occupancy {occ} [{cls}] {len(hits)} pairs, closest {dmin}")
            if a.v:
                for d, mop, op, dst, ml, wl in hits[:8]:
                    print(f"    d={d} {mop} (line {ml}) -> {op} {dst} (line {wl})")
    print(f"pairs within {a.window}: exposed {exposed}, single-wave {single}")
    return 1 if exposed or (a.all and single) else 0


if __name__ == "__main__":
    sys.exit(main())
