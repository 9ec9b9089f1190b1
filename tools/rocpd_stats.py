"""Kernel statistics (calls, total, mean, share) from a rocprofv3 SQLite database (rocpd), the
format this image's rocprofv3 writes by default:  python tools/rocpd_stats.py gpurun_out/prof/run_results.db"""
import sqlite3
import sys


def stats(path):
    db = sqlite3.connect(path)
    q = ("select s.display_name, count(*), sum(d.end - d.start), min(d.end - d.start), max(d.end - d.start) "
         "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.display_name")
    rows = sorted(db.execute(q).fetchall(), key=lambda r: -r[2])
    total = sum(r[2] for r in rows)
    return [(n, c, t, t / c, t / total, mn, mx) for n, c, t, mn, mx in rows]


if __name__ == "__main__":
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
    for n, c, t, avg, frac, mn, mx in stats(sys.argv[1]):
        print(f'"{n}",{c},{t},{avg:.1f},{100*frac:.4f},{mn},{mx}')
