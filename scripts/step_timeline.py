"""Per-step GPU timeline from a rocprofv3 kernel trace of bench.py.

Splits the trace into steps at each launch of the fused kernel and reports,
per step (median over the timed steps): period (fused start → next fused
start), the duration of every kernel in the step, and the idle gaps between
consecutive kernels.  Used to price the fixed per-step costs that decide
strong scaling.

  python scripts/step_timeline.py gpurun_out/TAG/trace/run_kernel_trace.csv
"""
import csv
import statistics
import sys


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0].split('<')[0]


def main(path, key='sg_fast'):
    rows = [r for r in csv.DictReader(open(path))]
    ks = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), short(r['Kernel_Name']))
                 for r in rows), key=lambda x: x[0])
    starts = [i for i, k in enumerate(ks) if k[2].startswith(key)]
    steps = []
    for a, b in zip(starts, starts[1:]):
        seq = ks[a:b]
        period = ks[b][0] - ks[a][0]
        items = []
        for i, (s, e, n) in enumerate(seq):
            nxt = ks[a + i + 1][0]
            items.append((n, e - s, nxt - e))
        steps.append((period, items))
    # keep the common step shape (the timed steps)
    shape = statistics.mode(tuple(n for n, _, _ in it) for _, it in steps)
    steps = [(p, it) for p, it in steps if tuple(n for n, _, _ in it) == shape]
    print('steps analysed: {}  (shape: {})'.format(len(steps), ' -> '.join(shape)))
    print('median period: {:.1f} us'.format(statistics.median(p for p, _ in steps) / 1e3))
    for i, n in enumerate(shape):
        d = statistics.median(it[i][1] for _, it in steps) / 1e3
        g = statistics.median(it[i][2] for _, it in steps) / 1e3
        print('  {:<28s} {:9.1f} us   gap after {:6.1f} us'.format(n, d, g))


if __name__ == '__main__':
    main(*sys.argv[1:])
