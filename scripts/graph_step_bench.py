"""Eager vs hipGraph-replayed all-pairs steps on one GPU (diagnostic).

One emulated rank's share of a W-GPU AIDS700nef step (pair shard, label term, slab
reduce, Adam; no collective), timed three ways:
  eager    bench.py's loop: sg_fwd_bwd_ex → sg_adam_tf launched from Python per step,
  graph1   one captured step (sg_fwd_bwd_dseed → Adam → seed + 1), replayed per step,
  graphK   K captured steps per graph.
Prints one JSON line per W.

  python scripts/graph_step_bench.py [--worlds 1,8] [--steps 200] [--per-graph 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--worlds', default='1,8')
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--per-graph', type=int, default=10)
    a = ap.parse_args()
    import torch
    from graphembedding_amd import _lib
    from graphembedding_amd.allpairs import AllPairsShard, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE

    gs = load_graph_set('syn_aids700nef', n_max=10)
    flags = Flags(dropout=0.1)
    labels = gs.label_matrix(flags.yeta)
    dev = torch.device('cuda', 0)
    for W in [int(x) for x in a.worlds.split(',')]:
        model = SiameseGCNTNMSE(gs.d_in, flags, device=dev, n_max=gs.n_max)
        shard = AllPairsShard(gs, labels, 0, W, device=dev)
        batch = shard.batch(model, balance=True)
        ws = model.workspace(batch.n_pairs)
        out = {'world': W, 'pairs': batch.n_pairs}

        def eager():
            model.fwd_bwd(batch)
            model.apply_adam()
            model.step_count += 1

        for _ in range(20):
            eager()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            eager()
        torch.cuda.synchronize()
        out['eager_us'] = (time.perf_counter() - t0) * 1e6 / a.steps

        seed_dev = torch.tensor([model._seed(None)], dtype=torch.int64, device=dev)

        def body():
            _lib.fwd_bwd_dseed(model.sg, batch.records, batch.n_pairs, batch.pair_offset,
                               batch.batch_total, model.params, seed_dev, batch.y_stats, 1, None,
                               model.grad, model.loss_buf, ws, order=batch.order)
            model.apply_adam()
            _lib.seed_advance(seed_dev, 1)

        for k in (1, a.per_graph):
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                body()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(k):
                    body()
            reps = max(1, a.steps // k)
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                g.replay()
            torch.cuda.synchronize()
            out['graph{}_us'.format(k)] = (time.perf_counter() - t0) * 1e6 / (reps * k)
        out['loss'] = float(model.loss_buf[0].item())
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
