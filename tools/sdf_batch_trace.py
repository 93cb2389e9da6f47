"""Per-kernel durations of one sdf_pdf batch from a rocprofv3 kernel trace (usage: trace.csv [batch])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
seq = [(r['Kernel_Name'], int(r['End_Timestamp']) - int(r['Start_Timestamp'])) for r in rows]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 5
i = [j for j, (n, _) in enumerate(seq) if 'k_sdf_prep' in n][k]
tot = 0
for n, d in seq[i:]:
    print(f"{n[:70]:70s} {d / 1e3:8.1f}")
    tot += d
    if 'k_sdf_raw' in n:
        break
print('batch total us', tot / 1e3)
