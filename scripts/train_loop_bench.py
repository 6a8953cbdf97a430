"""The reference's own training loop, timed three ways on one GPU (diagnostic).

train.py:8-44 runs FLAGS.iters steps of get_feed_dict + sess.run([opt_op, loss]) with
B = 5 pairs per step (config.py:70): a launch-bound loop.  Steps/s of
  host     model.get_feed_dict (host samplers + packing, H2D) → train_step (synced),
  device   DeviceFeed.next_batch (device samplers + packing) → train_step, no syncs,
  graph    hipGraph replay of captured DeviceFeed → fwd_bwd → Adam → seed steps.
Prints one JSON line.

  python scripts/train_loop_bench.py [--dataset syn_aids700nef] [--steps 2000] [--stack average]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dataset', default='syn_aids700nef')
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--graph-steps', type=int, default=50, help='steps per captured graph')
    ap.add_argument('--stack', choices=('default', 'average'), default='default')
    a = ap.parse_args()
    import torch
    from _fixtures import AVERAGE_STACK
    from graphembedding_amd.config import Flags
    from graphembedding_amd.data import synthetic_ged_matrix
    from graphembedding_amd.data_siamese import SiameseModelData
    from graphembedding_amd.device_sampler import DeviceFeed
    from graphembedding_amd.dist_calculator import DistCalculator
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    f = Flags(dataset=a.dataset, **(dict(AVERAGE_STACK) if a.stack == 'average' else {}))

    def make():
        data = SiameseModelData(f)
        gs = list(data.orig_train_graphs) + [data.test_data.gs[i].nxgraph for i in range(data.m)]
        dc = DistCalculator.from_matrix(f.dataset, gs, synthetic_ged_matrix(gs))
        model = SiameseGCNTNMSE(data.input_dim(), f, device='cuda')
        return data, dc, model

    out = {'workload': 'reference train loop, {}, B = {} pairs per step, {} stack'.format(
        a.dataset, f.batch_size, a.stack)}
    # host feed (the reference's get_feed_dict) + synced train_step
    data, dc, model = make()
    n_host = max(50, a.steps // 10)
    for _ in range(5):
        model.train_step(model.get_feed_dict(data, dc, 'train'))
    t0 = time.perf_counter()
    for _ in range(n_host):
        model.train_step(model.get_feed_dict(data, dc, 'train'))
    out['host_steps_per_s'] = n_host / (time.perf_counter() - t0)
    # device feed, eager launches, no per-step sync
    data, dc, model = make()
    feed = DeviceFeed(model, data, dc, 'train')
    for _ in range(5):
        model.train_step(feed.next_batch(), sync=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        model.train_step(feed.next_batch(), sync=False)
    torch.cuda.synchronize()
    out['device_steps_per_s'] = a.steps / (time.perf_counter() - t0)
    # hipGraph replay
    data, dc, model = make()
    feed = DeviceFeed(model, data, dc, 'train')
    g = model.capture_train_steps(feed, n_steps=a.graph_steps)
    g.replay(1)
    torch.cuda.synchronize()
    reps = max(1, a.steps // a.graph_steps)
    t0 = time.perf_counter()
    g.replay(reps)
    torch.cuda.synchronize()
    out['graph_steps_per_s'] = reps * a.graph_steps / (time.perf_counter() - t0)
    out['graph_us_per_step'] = 1e6 / out['graph_steps_per_s']
    out['loss'] = float(model.loss_buf[0].item() + model.reg_buf[0].item())
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
