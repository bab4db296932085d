"""Static ISA audit: for every kernel in a save-temps .s file, count per innermost loop body the
MFMAs, v_accvgpr moves/writes/reads and s_nops, to spot accumulator rotation."""
import re
import sys

def main(path, pat=""):
    cur = None
    funcs = {}
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur:
            funcs[cur].append(line)
    for name, lines in funcs.items():
        if pat and pat not in name:
            continue
        # loop = from a label with "Loop Header" to the backward branch to it
        text = lines
        for i, l in enumerate(text):
            m = re.match(r"^(\.LBB\d+_\d+):.*Loop Header", l)
            if not m:
                continue
            lab = m.group(1)
            for j in range(i + 1, len(text)):
                if re.search(r"s_cbranch\w*\s+" + re.escape(lab) + r"\b", text[j]) or re.search(r"s_branch\s+" + re.escape(lab) + r"\b", text[j]):
                    body = text[i:j + 1]
                    c = lambda r: sum(1 for b in body if re.search(r, b))
                    print(f"{name[:110]} {lab}: mfma={c(r'v_mfma')} accmov={c(r'v_accvgpr_mov')} "
                          f"accw={c(r'v_accvgpr_write')} accr={c(r'v_accvgpr_read')} len={len(body)}")
                    break

if __name__ == "__main__":
    main(*sys.argv[1:])
