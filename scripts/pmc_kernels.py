"""Per-kernel PMC summary of scripts/profile_counters.sh passes (any bench workload).
usage: python scripts/pmc_kernels.py gpurun_out/TAG [kernel-name substring ...]

For every kernel whose name contains one of the substrings: dispatches, and the
per-dispatch averages of every counter collected, plus derived ratios (wait and
LDS fractions of wave cycles, LDS bank conflicts per LDS-active cycle)."""
import collections
import csv
import glob
import sys


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0]


def main(d, subs):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(d + '/pass*/run_counter_collection.csv')):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = short(r['Kernel_Name'])
            if subs and not any(s in k for s in subs):
                continue
            per[(k, r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
        for (k, _, c), v in per.items():
            acc[k][c].append(v)
    for k, m in sorted(acc.items()):
        avg = {c: sum(v) / len(v) for c, v in m.items()}
        print(k)
        for c in sorted(avg):
            print('   {:28s} {:14.4g}'.format(c, avg[c]))
        w = avg.get('SQ_WAVE_CYCLES')
        if w:
            for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_LDS',
                      'SQ_ACTIVE_INST_LDS', 'SQ_ACTIVE_INST_VALU'):
                if c in avg:
                    print('   {:28s} {:14.3f}'.format(c + '/wave_cyc', avg[c] / w))
        if avg.get('SQ_LDS_IDX_ACTIVE'):
            print('   {:28s} {:14.3f}'.format('bank_conflict/lds_active',
                                              avg.get('SQ_LDS_BANK_CONFLICT', 0) /
                                              avg['SQ_LDS_IDX_ACTIVE']))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:])
