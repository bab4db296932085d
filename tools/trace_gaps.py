"""Per-forward GPU busy time vs wall time from a rocprofv3 kernel-trace database (rocpd SQLite): where a
sampling loop's step goes between kernels.  Usage: python tools/trace_gaps.py <results.db> [n_last_forwards]"""
import collections
import sqlite3
import sys

db = sys.argv[1]
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 27
cur = sqlite3.connect(db).cursor()
rows = cur.execute("select name, start, end from kernels order by start").fetchall()
starts = [i for i, r in enumerate(rows) if "pack_input" in r[0]]
fw = []
for a, b in zip(starts, starts[1:] + [len(rows)]):
    ks = rows[a:b]
    busy = sum(e - s for _, s, e in ks)
    wall = (rows[b][1] if b < len(rows) else ks[-1][2]) - ks[0][1]
    fw.append((len(ks), busy, wall, ks))
fw = fw[-n_last:]
n = len(fw)
med = sorted(fw, key=lambda f: f[2])[n // 2]  # median forward (the last one's wall runs into the host)
print(f"{n} forwards: launches/forward {sum(f[0] for f in fw) / n:.0f}, busy {sum(f[1] for f in fw) / n / 1e6:.3f} ms "
      f"mean; median forward: busy {med[1] / 1e6:.3f} ms, wall {med[2] / 1e6:.3f} ms, gap per launch "
      f"{(med[2] - med[1]) / med[0] / 1e3:.2f} us")
tot = collections.Counter()
cnt = collections.Counter()
for f in fw:
    for name, s, e in f[3]:
        short = name.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].split("::")[-1][-40:]
        tot[short] += e - s
        cnt[short] += 1
for k, v in tot.most_common(25):
    print(f"  {k:42s} {v / n / 1e3:9.1f} us/forward  {cnt[k] / n:5.1f} launches  {v / cnt[k] / 1e3:7.2f} us avg")
