"""Per-wave timeline of one sg_fast_kernel launch (diagnostic, GPU only).

Build the timing variant here, then run on the box:
    python graphembedding_amd/build.py --out graphembedding_amd/lib/libsiamese_timing.so \
        -DSG_FAST_TIMING=1
    SG_LIB=graphembedding_amd/lib/libsiamese_timing.so python scripts/fast_timing.py 1 8
        [--stack=average|attention] [--records=bf16]

For each emulated world size W the script runs rank 0's shard of the bench workload
(AIDS700nef all-pairs), then reads the per-wave s_memrealtime stamps (100 MHz): start,
after the prologue, after the pair loop, at the end. It prints where the launch's
time goes: the dispatch ramp, the prologue, the spread of pair-loop finish times (the
tail), and the flush.
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def stats(x):
    x = np.asarray(x, dtype=np.float64)
    return 'min {:7.2f} med {:7.2f} p90 {:7.2f} max {:7.2f}'.format(
        x.min(), np.median(x), np.percentile(x, 90), x.max())


def main():
    import torch
    from graphembedding_amd import _lib
    from graphembedding_amd.allpairs import AllPairsShard, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE

    L = _lib.lib()
    if not hasattr(L, 'sg_fast_timing_fetch'):
        raise SystemExit('SG_LIB must point at a -DSG_FAST_TIMING=1 build')
    L.sg_fast_timing_fetch.argtypes = [ctypes.c_void_p, ctypes.c_int]
    device = torch.device('cuda', 0)
    # --stack average|attention (the tuning.py stack), --records bf16 (config C3)
    opt = {a.split('=')[0]: a.split('=')[1] for a in sys.argv[1:] if '=' in a}
    fl = dict(dropout=0.1, record_dtype=opt.get('--records', 'f32'))
    stack = opt.get('--stack', 'default')
    if stack in ('average', 'attention'):
        fl.update(num_layers=4,
                  layer_2='Average' if stack == 'average' else 'Attention:input_dim=16',
                  layer_3='NTN:input_dim=16,feature_map_dim=10,inneract=relu,dropout=True,'
                          'bias=True')
    flags = Flags(**fl)
    gs = load_graph_set('syn_aids700nef', n_max=10)
    labels = gs.label_matrix(flags.yeta)
    balance = '--batch-order' not in sys.argv
    worlds = [int(a) for a in sys.argv[1:] if not a.startswith('--')] or [1, 8]
    print('stack:', stack, 'records:', fl['record_dtype'])
    print('order:', 'class' if balance else 'batch')
    for W in worlds:
        model = SiameseGCNTNMSE(gs.d_in, flags, device=device, n_max=gs.n_max)
        shard = AllPairsShard(gs, labels, 0, W, device=device, dtype=fl['record_dtype'])
        batch = shard.batch(model, balance=balance)
        model.workspace(batch.n_pairs)
        for _ in range(5):
            model.fwd_bwd(batch, add_label_term=True)
        torch.cuda.synchronize()
        buf = np.zeros(4096 * 5, dtype=np.uint64)
        n = L.sg_fast_timing_fetch(buf.ctypes.data, buf.size)
        assert n == buf.size
        T = buf.reshape(-1, 5).astype(np.int64)
        T = T[T[:, 0] > 0]
        # only the last launch: stamps of earlier launches were overwritten wave by wave
        t0 = T[:, 0].min()
        us = (T[:, :4] - t0) / 100.0       # 100 MHz -> µs
        pairs = T[:, 4] & 0xFFFFFFFF
        wcls = (T[:, 4] >> 32) - 1   # class of a class-exclusive wave, -1 = mixed schedule
        nwv = len(T)
        print('W={} pairs={} waves={} pairs/wave {}'.format(W, shard.n, nwv, stats(pairs)))
        print('  start      ', stats(us[:, 0]))
        print('  prologue   ', stats(us[:, 1] - us[:, 0]))
        print('  loop       ', stats(us[:, 2] - us[:, 1]))
        print('  loop end   ', stats(us[:, 2]))
        print('  flush      ', stats(us[:, 3] - us[:, 2]))
        print('  end        ', stats(us[:, 3]))
        per_pair = (us[:, 2] - us[:, 1]) / np.maximum(pairs, 1)
        print('  µs/pair/wave', stats(per_pair))
        if (wcls >= 0).any():   # class-exclusive schedule: cost per class -> SG_CLS_W
            base = None
            for c in range(4):
                sel = wcls == c
                if not sel.any():
                    continue
                med = float(np.median(per_pair[sel]))
                base = base or med
                print('  class {} ({}{}) waves {:5d} µs/pair {}  rel {:.3f}  loop end {}'.format(
                    c, 3 if c & 1 else 2, 3 if c & 2 else 2, int(sel.sum()),
                    stats(per_pair[sel]), med / base, stats(us[sel, 2])))
        # blocks go round-robin over the 8 XCDs: block b -> XCD b % 8
        nwpb = 8
        blk = np.arange(nwv) // nwpb
        xcd = blk % 8
        print('  loop end by XCD:', ' '.join('{:.1f}'.format(np.median(us[xcd == x, 2]))
                                              for x in range(8)))
        print('  µs/pair by XCD: ', ' '.join('{:.3f}'.format(np.median(per_pair[xcd == x]))
                                              for x in range(8)))
        # the two waves sharing a SIMD: w and w+4 of a block
        w = np.arange(nwv) % nwpb
        old = us[w < 4, 2] - us[w < 4, 1]
        young = us[w >= 4, 2] - us[w >= 4, 1]
        m = min(len(old), len(young))
        print('  young-old loop time', stats(young[:m] - old[:m]))
        # the waves that end last, with their SIMD partner (w ^ 4 of the same block)
        print('  last loop ends: wave (block, w, xcd) class pairs loop µs/pair | partner class '
              'pairs loop-end')
        for i in np.argsort(-us[:, 2])[:12]:
            pi = (i // nwpb) * nwpb + ((i % nwpb) ^ 4)
            pe = '{:2d} {:4d} {:8.2f}'.format(int(wcls[pi]), int(pairs[pi]), us[pi, 2]) \
                if pi < nwv else '-'
            print('    {:5d} ({:4d}, {}, {}) {:2d} {:4d} {:8.2f} {:5.2f} | {}'.format(
                int(i), int(i // nwpb), int(i % nwpb), int(xcd[i]), int(wcls[i]), int(pairs[i]),
                us[i, 2], per_pair[i], pe))
        sys.stdout.flush()


if __name__ == '__main__':
    main()
