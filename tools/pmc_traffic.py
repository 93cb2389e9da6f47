"""Summarise rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE, separate passes) into HBM bytes
per launch of one kernel, with the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE
(KiB) reads half the bytes of a wide coalesced read -> x2; WRITE_SIZE (KiB) is exact for 16-B
stores. Updates this kernel's entry of profiles/pmc_latest.json ({kernel: {...}}), which bench.py
reports as roofline.traffic of that kernel.

python tools/pmc_traffic.py <fetch.csv> <write.csv> <kernel-substring> <label>
"""
import csv
import json
import os
import sys


def mean_counter(path, kernel, name):
    vals = [float(r['Counter_Value']) for r in csv.DictReader(open(path))
            if kernel in r['Kernel_Name'] and r['Counter_Name'] == name]
    return sum(vals) / len(vals), len(vals)


def main():
    fetch, write, kernel, label = sys.argv[1:5]
    f, nf = mean_counter(fetch, kernel, 'FETCH_SIZE')
    w, nw = mean_counter(write, kernel, 'WRITE_SIZE')
    out = {'kernel': kernel, 'fetch_kib': f, 'write_kib': w, 'launches': [nf, nw],
           'bytes_per_launch': (2.0 * f + w) * 1024.0,
           'correction': 'FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1', 'source': label}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, 'profiles', 'pmc_latest.json')
    table = json.load(open(path)) if os.path.exists(path) else {}
    if 'kernel' in table:  # the round-2 single-kernel format
        table = {table['kernel']: table}
    table[kernel] = out
    with open(path, 'w') as fh:
        json.dump(table, fh, indent=1)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
