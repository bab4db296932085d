"""Opcode histogram (and optional class sequence) of one loop of one kernel in a save-temps .s file.
Usage: python tools/isa_hist.py file.s kernel-substring loop-label [seq]"""
import collections
import re
import sys

path, pat, lab = sys.argv[1:4]
lines = open(path).read().split("\n")
st = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(pat) + r"\S*:", l)][0]
body = lines[st:]
a = [i for i, l in enumerate(body) if l.startswith(lab + ":")][0]
e = [i for i, l in enumerate(body) if re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\b", l) and i > a][0]
ops = [l.split()[0] for l in body[a:e + 1] if l.startswith("\t") and l.strip() and not l.strip().startswith((";", "."))]
print(collections.Counter(ops).most_common(60))
if len(sys.argv) > 4:
    m = {"v_mfma": "M", "ds_read": "R", "v_exp": "E", "v_accvgpr": "a", "global_load_lds": "D", "s_waitcnt": "w",
         "s_barrier": "B", "s_nop": "n"}
    out = []
    for o in ops:
        c = next((v for k, v in m.items() if o.startswith(k)), "v" if o.startswith("v_") else "s" if o.startswith("s_") else "?")
        out.append(c)
    print("".join(out))
