"""Condense one scripts/gpu_round3.sh output dir into profiles/<tag>/:
- kernel_stats.csv: the kernel-trace-only rocprof pass of the driver's bench command
  (bench.py --gpus 1 --steps 20 --warmup 5), with that run's own bench line
  (trace_bench.json) beside it, so the profiler/event ratio is from one run;
- traffic.json: per-launch HBM bytes of the fused kernel from the PMC passes, corrected
  as MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE is in KiB and counts half of a
  16-B/lane coalesced stream on gfx950 -> x2; WRITE_SIZE in KiB);
- mfma_work.json: executed MFMA work per pair (SQ_INSTS_VALU_MFMA_MOPS_* x 512 FLOP,
  instruction counts, MFMA-busy cycles) against the algorithmic FLOPs per pair;
- bench.json: the bench line of the un-profiled run.
Usage: python scripts/make_profile_summary.py gpurun_out/TAG TAG [--no-global]"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, 'profiles', tag)
os.makedirs(dst, exist_ok=True)
KERNEL = 'sg_fast_kernel'


def is_fused_bwd(name):
    return KERNEL in name and 'true' in name.split(',')[1]


def pmc_pass(d):
    """{counter: mean per dispatch} over the fused fwd+bwd dispatches of one pass."""
    f = os.path.join(src, d, 'run_counter_collection.csv')
    per = defaultdict(lambda: defaultdict(float))
    for row in csv.DictReader(open(f)):
        if is_fused_bwd(row['Kernel_Name']):
            per[row['Dispatch_Id']][row['Counter_Name']] += float(row['Counter_Value'])
    ds = list(per.values())
    keys = ds[0].keys()
    return {k: sum(x[k] for x in ds) / len(ds) for k in keys}, len(ds)


passes = sorted(d for d in os.listdir(src) if d.startswith('pmc') and
                os.path.isdir(os.path.join(src, d)))
counters, ndisp = {}, {}
for d in passes:
    c, n = pmc_pass(d)
    for k, v in c.items():
        counters.setdefault(k, v)
        ndisp[k] = n

bench = json.load(open(os.path.join(src, 'bench.json')))
tb = json.load(open(os.path.join(src, 'trace_bench.json')))
n_pairs = bench['config']['global_batch'] // max(1, bench['n_gpus'])
flops_pair = float(bench['roofline']['note'].split('algorithmic ')[1].split(' FLOP')[0])

stats = os.path.join(src, 'trace', 'run_kernel_stats.csv')
shutil.copy(stats, os.path.join(dst, 'kernel_stats.csv'))
rows = list(csv.DictReader(open(stats)))
fk = [r for r in rows if is_fused_bwd(r['Name'])]
ev_ms = float(tb['roofline']['note'].split('event time ')[1].split(' ms')[0])
traffic = {'kernel': KERNEL + '<10, true, ...> (fused fwd+bwd)'}
if 'FETCH_SIZE' in counters:
    fetch_kib, write_kib = counters['FETCH_SIZE'], counters.get('WRITE_SIZE', 0.0)
    traffic.update({'fetch_bytes_raw': fetch_kib * 1024, 'fetch_bytes': 2 * fetch_kib * 1024,
                    'write_bytes': write_kib * 1024,
                    'traffic_bytes_per_launch': 2 * fetch_kib * 1024 + write_kib * 1024,
                    'algorithmic_bytes_per_launch': n_pairs * bench['roofline_hbm']['bytes_per_pair'],
                    'dispatches': [ndisp.get('FETCH_SIZE'), ndisp.get('WRITE_SIZE')],
                    'correction': 'FETCH_SIZE(KiB)*1024*2 (gfx950 half-count for 16-B/lane '
                                  'streams) + WRITE_SIZE(KiB)*1024'})
if fk:
    traffic['rocprof_avg_ns'] = float(fk[0]['AverageNs'])
    traffic['rocprof_calls'] = int(fk[0]['Calls'])
    traffic['same_run_sg_fwd_bwd_event_ms'] = ev_ms
    traffic['same_run_ms_per_step'] = tb['ms_per_step']
    traffic['rocprof_over_event'] = float(fk[0]['AverageNs']) * 1e-6 / ev_ms
traffic['tree'] = tag
# the fused kernel's sources the counters belong to: bench.py reports these bytes only
# while the tree's sources hash the same (a kernel change makes them stale)
sys.path.insert(0, root)
from bench import fused_kernel_source_hash  # noqa: E402
traffic['sources_sha1'] = fused_kernel_source_hash()
json.dump(traffic, open(os.path.join(dst, 'traffic.json'), 'w'), indent=1)

mf = {}
if 'SQ_INSTS_VALU_MFMA_MOPS_F32' in counters:
    f32 = counters['SQ_INSTS_VALU_MFMA_MOPS_F32'] * 512 / n_pairs
    bf16 = counters.get('SQ_INSTS_VALU_MFMA_MOPS_BF16', 0.0) * 512 / n_pairs
    mf = {'pairs_per_launch': n_pairs,
          'algorithmic_flop_per_pair': flops_pair,
          'executed_f32_mfma_flop_per_pair': f32,
          'executed_bf16_mfma_flop_per_pair': bf16,
          'f32_mfma_over_algorithmic': f32 / flops_pair,
          'bf16_mfma_over_algorithmic': bf16 / flops_pair,
          'f32_mfma_insts_per_pair': counters.get('SQ_INSTS_VALU_MFMA_F32', 0) / n_pairs,
          'bf16_mfma_insts_per_pair': counters.get('SQ_INSTS_VALU_MFMA_BF16', 0) / n_pairs,
          'valu_insts_per_pair_incl_mfma': counters.get('SQ_INSTS_VALU', 0) / n_pairs,
          'mfma_busy_cycles_per_pair': counters.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / n_pairs,
          'note': 'MOPS counters count FLOP/512; f32 MFMA = v_mfma_f32_16x16x4_f32 (2048 FLOP, '
                  '32 cycles); bf16 = split-bf16 products (3 bf16 MFMAs per f32-accurate '
                  'product)'}
    for k in ('SQ_ACTIVE_INST_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_LDS', 'SQ_WAVE_CYCLES',
              'SQ_WAIT_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_INSTS_BRANCH'):
        if k in counters:
            mf[k.lower() + '_per_pair'] = counters[k] / n_pairs
    json.dump(mf, open(os.path.join(dst, 'mfma_work.json'), 'w'), indent=1)

shutil.copy(os.path.join(src, 'bench.json'), os.path.join(dst, 'bench.json'))
shutil.copy(os.path.join(src, 'trace_bench.json'), os.path.join(dst, 'trace_bench.json'))
for f in ('summary.txt', 'smoke.log'):
    if os.path.isfile(os.path.join(src, f)):
        shutil.copy(os.path.join(src, f), os.path.join(dst, f))
if os.path.isfile(os.path.join(src, 'pytest_gpu.log')):
    with open(os.path.join(src, 'pytest_gpu.log')) as f:
        tail = f.read().splitlines()[-3:]
    open(os.path.join(dst, 'pytest_gpu_tail.txt'), 'w').write('\n'.join(tail) + '\n')
if '--no-global' not in sys.argv:
    json.dump(traffic, open(os.path.join(root, 'profiles', 'traffic.json'), 'w'), indent=1)
print(json.dumps(traffic, indent=1))
print(json.dumps(mf, indent=1))
