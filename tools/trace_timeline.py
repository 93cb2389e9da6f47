"""Print one training step's kernel timeline (start / end / duration us, queue) from a rocprofv3 kernel
trace: the dispatches between the last two k_adam launches. usage: python tools/trace_timeline.py CSV"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_adam' in r['Kernel_Name']]
a, b = idx[-2], idx[-1]
st = rows[a + 1:b + 1]
t0 = int(st[0]['Start_Timestamp'])
for r in st:
    s = (int(r['Start_Timestamp']) - t0) / 1e3
    e = (int(r['End_Timestamp']) - t0) / 1e3
    print('%7.1f %7.1f %6.1f q%s %s' % (s, e, e - s, r.get('Queue_Id', '?'), r['Kernel_Name'].replace('anr::', '')[:70]))
