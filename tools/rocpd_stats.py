"""Kernel statistics (the rocprofv3 --stats table) from a rocprofv3 results database.

usage: python tools/rocpd_stats.py gpurun_out/prof_x/run_results.db > profiles/rN_x_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    q = ('select s.display_name, count(*), sum(d."end" - d.start), avg(d."end" - d.start), '
         'min(d."end" - d.start), max(d."end" - d.start) from rocpd_kernel_dispatch d '
         'join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.display_name order by 3 desc')
    rows = list(c.execute(q))
    tot = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs', 'MaxNs'])
    for name, n, s, avg, mn, mx in rows:
        w.writerow([name, n, s, round(avg, 1), round(100.0 * s / tot, 4), mn, mx])


if __name__ == '__main__':
    main(sys.argv[1])
