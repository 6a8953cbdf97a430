"""Summarise rocprofv3 --pmc CSVs for one kernel: per-dispatch means and
per-pair / utilisation ratios.  Usage: pmc_summary.py DIR [kernel-substring] [pairs]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else 'sg_fast_kernel'
pairs = float(sys.argv[3]) if len(sys.argv) > 3 else 490000.0
agg = collections.defaultdict(lambda: collections.defaultdict(float))
meta = None
for f in sorted(glob.glob(d + '/pass*/run_counter_collection.csv')):
    for row in csv.DictReader(open(f)):
        if ksub not in row['Kernel_Name']:
            continue
        agg[row['Counter_Name']][(f, row['Dispatch_Id'])] += float(row['Counter_Value'])
        meta = (row['VGPR_Count'], row['SGPR_Count'], row['LDS_Block_Size'], row['Grid_Size'],
                row['Workgroup_Size'])
mean = {c: sum(v.values()) / len(v) for c, v in agg.items()}
print('VGPR/SGPR/LDS/grid/wg:', meta)
for c in sorted(mean):
    print('{:28s} {:14.4e}  per pair {:10.2f}'.format(c, mean[c], mean[c] / pairs))
if 'GRBM_GUI_ACTIVE' in mean:
    cyc = mean['GRBM_GUI_ACTIVE'] / 8.0
    print('kernel cycles ~ {:.3e}'.format(cyc))
    if 'SQ_LDS_IDX_ACTIVE' in mean:
        print('LDS busy per CU: {:.1%}'.format(mean['SQ_LDS_IDX_ACTIVE'] / 256 / cyc))
    if 'SQ_VALU_MFMA_BUSY_CYCLES' in mean:
        print('MFMA busy per SIMD: {:.1%}'.format(mean['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc))
if 'SQ_WAVE_CYCLES' in mean:
    w = mean['SQ_WAVE_CYCLES']
    for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY'):
        if c in mean:
            print('{:20s} {:.1%} of wave cycles'.format(c, mean[c] / w))
