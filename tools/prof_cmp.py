"""Per-kernel totals of rocprofv3 --stats runs side by side: prof_cmp.py name=dir [name=dir ...]."""
import csv
import glob
import sys


def load(d):
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)
    out = {}
    for row in csv.DictReader(open(f[0])):
        name = row["Name"].split("(")[0][:60]
        out[name] = out.get(name, 0.0) + float(row["TotalDurationNs"]) / 1e6
    return out


runs = [(a.split("=")[0], load(a.split("=")[1])) for a in sys.argv[1:]]
names = sorted(set().union(*[r.keys() for _, r in runs]), key=lambda n: -runs[0][1].get(n, 0))
print(f"{'kernel (ms total)':60s}" + "".join(f"{n:>12s}" for n, _ in runs))
for k in names:
    print(f"{k:60s}" + "".join(f"{r.get(k, 0):12.2f}" for _, r in runs))
print(f"{'TOTAL':60s}" + "".join(f"{sum(r.values()):12.2f}" for _, r in runs))
