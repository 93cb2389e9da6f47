"""Summarise one training step from a rocprofv3 kernel trace: per-kernel totals between the last two
k_adam dispatches, or the K-th last step (bench.py --mode train profiles 3 steps after the timed ones,
so K = 4 is the last timed step). usage: python tools/train_trace_summary.py <run_kernel_trace.csv> [K]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_adam' in r['Kernel_Name']]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 1
a, b = idx[-1 - K], idx[-K]
step = rows[a + 1:b + 1]
t0, t1 = int(step[0]['Start_Timestamp']), int(step[-1]['End_Timestamp'])
busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in step)
print('step span %.1f us, kernels %d, busy %.1f us' % ((t1 - t0) / 1e3, len(step), busy / 1e3))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in step:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    agg[r['Kernel_Name'].replace('anr::', '')[:60]][0] += 1
    agg[r['Kernel_Name'].replace('anr::', '')[:60]][1] += d
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:14]:
    print('%-60s %3d %8.1f %6.1f' % (n, c, t, t / c))
gaps = []
for p, q in zip(step[:-1], step[1:]):
    g = (int(q['Start_Timestamp']) - int(p['End_Timestamp'])) / 1e3
    gaps.append((g, p['Kernel_Name'].replace('anr::', '')[:40], q['Kernel_Name'].replace('anr::', '')[:40]))
print('idle between kernels %.1f us; largest gaps:' % sum(max(g[0], 0) for g in gaps))
for g in sorted(gaps, reverse=True)[:8]:
    print('  %7.1f us  %s -> %s' % g)

# concurrency sweep: time with no kernel running (idle), and per kernel the time it runs ALONE (the
# serial stretches of the step: every microsecond there is on the critical path)
ev = []
for k, r in enumerate(step):
    ev.append((int(r['Start_Timestamp']), 1, k))
    ev.append((int(r['End_Timestamp']), -1, k))
ev.sort()
running = set()
alone = collections.defaultdict(float)
idle = 0.0
conc = collections.defaultdict(float)
prev = ev[0][0]
for t, d, k in ev:
    dt = (t - prev) / 1e3
    if dt > 0:
        conc[len(running)] += dt
        if not running:
            idle += dt
        elif len(running) == 1:
            alone[step[next(iter(running))]['Kernel_Name'].replace('anr::', '')[:60]] += dt
    prev = t
    if d > 0:
        running.add(k)
    else:
        running.discard(k)
print('time by concurrency (us):', {c: round(v, 1) for c, v in sorted(conc.items())})
print('kernels running alone (critical stretches), us:')
for n, t in sorted(alone.items(), key=lambda x: -x[1])[:16]:
    print('  %-60s %7.1f' % (n, t))
