"""Summarise rocprofv3 PMC passes of a fused bwd kernel (sg_fast_kernel<.., true, ..>).
usage: python scripts/pmc_report.py gpurun_out/TAG [n_pairs] [kernel name, default sg_fast_kernel]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
P = float(sys.argv[2]) if len(sys.argv) > 2 else 490000.0
KN = sys.argv[3] if len(sys.argv) > 3 else 'sg_fast_kernel'
acc = collections.defaultdict(list)
for f in glob.glob(d + '/pass*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if KN + '<' in k and 'true' in k.split('<')[1].split(',')[0 if KN == 'sg_fast32_kernel' else 1]:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
m = {k: sum(v) / len(v) for k, v in acc.items()}
g = m.get('GRBM_GUI_ACTIVE', 0) / 8.0   # per-XCD cycles of the dispatch
simd = 1024.0
out = {}
if g:
    out['kernel_cycles'] = g
    if 'SQ_VALU_MFMA_BUSY_CYCLES' in m:
        out['mfma_util'] = m['SQ_VALU_MFMA_BUSY_CYCLES'] / (g * simd)
    if 'SQ_ACTIVE_INST_VALU' in m:
        out['valu_active(quad*4)/simd_cycles'] = m['SQ_ACTIVE_INST_VALU'] * 4 / (g * simd)
    if 'SQ_VALU_MFMA_COEXEC_CYCLES' in m:
        out['coexec/simd_cycles'] = m['SQ_VALU_MFMA_COEXEC_CYCLES'] / (g * simd)
    if 'SQ_LDS_IDX_ACTIVE' in m:
        out['lds_active/cu_cycles'] = m['SQ_LDS_IDX_ACTIVE'] / (g * 256)
        out['lds_bank_conflict/cu_cycles'] = m.get('SQ_LDS_BANK_CONFLICT', 0) / (g * 256)
for k in ('SQ_INSTS_VALU', 'SQ_INSTS_MFMA', 'SQ_INSTS_LDS', 'SQ_INSTS_BRANCH', 'SQ_INSTS_SALU',
          'SQ_INSTS_SMEM', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_VMEM_WR'):
    if k in m:
        out[k + '/pair'] = m[k] / P
if 'SQ_WAVE_CYCLES' in m:
    w = m['SQ_WAVE_CYCLES']
    for k in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_LDS'):
        out[k + '/wave_cycles'] = m.get(k, 0) / w
for k, v in out.items():
    print('{:36s} {:.4g}'.format(k, v))
