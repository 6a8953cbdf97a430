"""Throughput probe for config C4 (AIDS10knef-shaped graphs, N <= 30, n_max 30).

Packs the first P pairs of the all-pairs stream and times fwd+bwd (+ reduce) on one
GPU, for f32 and bf16 records and both processing orders.
    python scripts/c4_probe.py [P]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from graphembedding_amd.allpairs import AllPairsShard, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd import _lib
    from graphembedding_amd.model_mse import SiameseGCNTNMSE

    P = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    t0 = time.time()
    gs = load_graph_set('syn_aids10knef', n_max=32)   # capacity-32 records (sg_fast32)
    print('graph set: {} graphs, d_in {}, {:.1f} s'.format(len(gs.graphs), gs.d_in,
                                                         time.time() - t0), flush=True)
    dev = torch.device('cuda', 0)
    for dtype in ('f32', 'bf16'):
        flags = Flags(dropout=0.1, record_dtype=dtype,
                      layer_3='Padding:max_in_dims=30,padding_value=0',
                      layer_4='NTN:input_dim=30,feature_map_dim=10,inneract=relu,dropout=True,'
                              'bias=True')
        labels = gs.label_matrix(flags.yeta)
        model = SiameseGCNTNMSE(gs.d_in, flags, device=dev, n_max=30)
        assert model.n_max == gs.n_max, (model.n_max, gs.n_max)
        shard = AllPairsShard(gs, labels, 0, 1, device=dev, n_pairs=P, dtype=dtype)
        for balance in (False, True):
            batch = shard.batch(model, balance=balance)
            model.workspace(batch.n_pairs)
            model.fwd_bwd(batch)
            torch.cuda.synchronize()
            n_it = 3
            t = time.perf_counter()
            for _ in range(n_it):
                model.fwd_bwd(batch)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / n_it
            print('{} records ({} B/pair), order={}: path={} {:.3f} ms/step  {:.2f} M pairs/s'.format(
                dtype, shard.record_bytes, 'class' if balance else 'batch',
                _lib.PATH_NAMES[model.kernel_path], dt * 1e3, P / dt / 1e6),
                flush=True)
        del shard, batch
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
