"""Condense one gpu_round.sh output dir into profiles/<tag>/: rocprof kernel
stats, the bench line, and per-launch HBM traffic of the fused kernel from the
PMC passes, corrected as MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE is in
KiB and reads half of a 16-B/lane coalesced stream on gfx950 → ×2)."""
import csv
import json
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, 'profiles', tag)
os.makedirs(dst, exist_ok=True)
KERNEL = 'sg_fast_kernel'


def pmc(counter):
    f = os.path.join(src, 'pmc_' + counter, 'run_counter_collection.csv')
    vals = {}
    for row in csv.DictReader(open(f)):
        if KERNEL in row['Kernel_Name'] and 'true' in row['Kernel_Name'].split(',')[1]:
            vals[row['Dispatch_Id']] = vals.get(row['Dispatch_Id'], 0.0) + float(row['Counter_Value'])
    v = list(vals.values())
    return sum(v) / len(v), len(v)


fetch_kib, nf = pmc('FETCH_SIZE')
write_kib, nw = pmc('WRITE_SIZE')
traffic = {'kernel': KERNEL, 'fetch_bytes_raw': fetch_kib * 1024, 'fetch_bytes': 2 * fetch_kib * 1024,
           'write_bytes': write_kib * 1024,
           'traffic_bytes_per_launch': 2 * fetch_kib * 1024 + write_kib * 1024,
           'dispatches': [nf, nw],
           'correction': 'FETCH_SIZE(KiB)*1024*2 (gfx950 half-count for 16-B/lane streams) + WRITE_SIZE(KiB)*1024'}
stats = os.path.join(src, 'trace', 'run_kernel_stats.csv')
shutil.copy(stats, os.path.join(dst, 'kernel_stats.csv'))
rows = list(csv.DictReader(open(stats)))
fk = [r for r in rows if KERNEL in r['Name']]
if fk:
    traffic['rocprof_avg_ns'] = float(fk[0]['AverageNs'])
    traffic['rocprof_calls'] = int(fk[0]['Calls'])
shutil.copy(os.path.join(src, 'bench.json'), os.path.join(dst, 'bench.json'))
json.dump(traffic, open(os.path.join(dst, 'traffic.json'), 'w'), indent=1)
json.dump(traffic, open(os.path.join(root, 'profiles', 'traffic.json'), 'w'), indent=1)
print(json.dumps(traffic, indent=1))
