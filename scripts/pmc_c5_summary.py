"""Per-kernel summary of scripts/gpu_r4_c5.sh: kernel-trace durations (average and largest
call, i.e. a full chunk) and, from the two PMC passes, SQ_WAIT_ANY / SQ_WAVE_CYCLES,
SQ_ACTIVE_INST_ANY / _VALU per wave-cycle and FETCH_SIZE in GB per call (KiB x 1024, x2:
the gfx950 half-count correction of MI355X_MICROARCH.md for 16-B/lane loads).
usage: python scripts/pmc_c5_summary.py gpurun_out/TAG"""
import collections
import csv
import glob
import sys


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0]


def main(d):
    for f in glob.glob(d + '/trace/**/run_kernel_stats.csv', recursive=True):
        print('kernel trace (pipeline off):', f[len(d) + 1:])
        rows = list(csv.DictReader(open(f)))
        for r in rows[:12]:
            print('  {:42s} calls {:3d}  avg {:8.3f} ms  max {:8.3f} ms'.format(
                short(r['Name'])[:42], int(r['Calls']), float(r['AverageNs']) / 1e6,
                float(r['MaxNs']) / 1e6))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + '/pmc*/**/run_counter_collection.csv', recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(short(r['Kernel_Name']), r['Dispatch_Id'], r['Counter_Name'])] += \
                float(r['Counter_Value'])
        for (k, _, c), v in per.items():
            acc[k][c].append(v)
    print('PMC (per call averages):')
    for k in sorted(acc):
        if not k.startswith('web_') and 'sg_' not in k:
            continue
        a = {c: sum(v) / len(v) for c, v in acc[k].items()}
        w = a.get('SQ_WAVE_CYCLES', 0.0)
        parts = []
        if w:
            parts.append('SQ_WAIT_ANY/SQ_WAVE_CYCLES {:.2f}'.format(a.get('SQ_WAIT_ANY', 0) / w))
            parts.append('ACTIVE_INST_ANY {:.2f}'.format(a.get('SQ_ACTIVE_INST_ANY', 0) / w))
            parts.append('ACTIVE_INST_VALU {:.2f}'.format(a.get('SQ_ACTIVE_INST_VALU', 0) / w))
        if 'FETCH_SIZE' in a:
            parts.append('fetch GB/call {:.2f}'.format(a['FETCH_SIZE'] * 1024 * 2 / 1e9))
        print('  {:32s} {}'.format(k[:32], '  '.join(parts)))


if __name__ == '__main__':
    main(sys.argv[1])
