"""Per-step cost of the gradient all-reduce path on one GPU (diagnostic).

One emulated rank's share of a W-GPU AIDS700nef step (bench.py --emulate-world W), timed
with no collective, with torch.distributed's RCCL backend (shard.make_allreduce_hook:
side stream + events), and with RCCL called on the compute stream
(rccl.RcclComm + shard.make_rccl_hook).  Both collectives run at world size 1 (one GPU
per box), so this prices the stream hand-offs around the collective, not xGMI latency.
Prints one JSON line per W.

  python scripts/collective_overhead.py [--worlds 8,1] [--steps 300]
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
    ap.add_argument('--worlds', default='8,1')
    ap.add_argument('--steps', type=int, default=300)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from graphembedding_amd.allpairs import AllPairsShard, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    from graphembedding_amd.rccl import RcclComm
    from graphembedding_amd.shard import make_allreduce_hook, make_rccl_hook

    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    store = dist.HashStore()
    dist.init_process_group('nccl', store=store, rank=0, world_size=1, device_id=dev)
    comm = RcclComm(0, 1, store=store)
    gs = load_graph_set('syn_aids700nef', n_max=10)
    flags = Flags(dropout=0.1)
    labels = gs.label_matrix(flags.yeta)
    hooks = {'none': None, 'torch_pg': make_allreduce_hook(), 'rccl_direct': make_rccl_hook(comm)}
    for W in [int(x) for x in a.worlds.split(',')]:
        model = SiameseGCNTNMSE(gs.d_in, flags, device=dev, n_max=gs.n_max)
        shard = AllPairsShard(gs, labels, 0, W, device=dev)
        batch = shard.batch(model, balance=True)
        model.workspace(batch.n_pairs)
        out = {'world': W, 'pairs': batch.n_pairs}
        for rep in range(2):
            for name, hook in hooks.items():
                def step():
                    model.fwd_bwd(batch)
                    if hook is not None:
                        hook(model)
                    model.apply_adam()
                    model.step_count += 1
                for _ in range(20):
                    step()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    step()
                torch.cuda.synchronize()
                out['{}_us_{}'.format(name, rep)] = (time.perf_counter() - t0) * 1e6 / a.steps
        print(json.dumps(out), flush=True)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
