"""bench.py — Siamese fwd+bwd graph-pairs/s on AIDS700nef-shaped all-pairs.

(--dataset syn_aids10knef: config C4, AIDS10knef-shaped all-pairs, 100.4 M pairs per
step, Padding/NTN 30 on the capacity-32 fused kernel; records resident when a rank's
shard fits HBM, else packed chunk by chunk inside the step.
 --dataset syn_web: config C5, 1,100 Web-sized synthetic graphs (N ~ U{64..512}),
1.21 M all-pairs per step, Padding/NTN 512 on the graph-store path: CSR store + pair
ids, NTN as MFMA GEMMs over the pairs.)

One step = one pass of the hot path over the whole 700² = 490,000-pair
all-pairs batch: fused forward + broadcast-MSE loss + backward over this rank's
pair shard, deterministic gradient reduction, RCCL all-reduce of the flat
gradient (N > 1), TF-form Adam.  Inputs (packed pair records) are resident in
HBM before timing starts.  Prints ONE JSON line (rank 0).

  python bench.py [--gpus N --steps K --warmup W]   (N > 1: starts N ranks itself)
  torchrun --nproc-per-node N bench.py --gpus N ...  (--gpus must equal WORLD_SIZE)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3       # gfx950 fp32 peak (vector = f32 MFMA), MI355X_MICROARCH.md


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=None, help='default 50 (C5: 3)')
    p.add_argument('--warmup', type=int, default=None, help='default 10 (C5: 1)')
    p.add_argument('--web-chunk', type=int, default=524288,
                   help='C5: pairs per internal chunk of sg_web_fwd_bwd (524,288: ≈86 GB of '
                        'workspace over the two pipeline slots; 262,144 measured 0.5%% slower)')
    p.add_argument('--dataset', default='syn_aids700nef')
    p.add_argument('--dropout', type=float, default=0.1)
    p.add_argument('--records', choices=('f32', 'bf16'), default='f32',
                   help='storage of Â in the pair records (bf16 = config C3); math is fp32')
    p.add_argument('--cpu-sample', type=int, default=0,
                   help='pairs for the CPU baseline (0 = auto, -1 = skip)')
    p.add_argument('--order', choices=('class', 'batch'), default='class',
                   help='record processing order: class-balanced (sg_pair_order) or batch order')
    p.add_argument('--chunk', type=int, default=4_000_000,
                   help='C4: pairs per packed chunk when a shard does not fit HBM')
    p.add_argument('--source', choices=('auto', 'records', 'store'), default='auto',
                   help='C4: the kernel gathers pairs from the graph store in launches of '
                        '--store-chunk pairs (auto), or records are packed, resident when the '
                        'shard fits --resident-gb, else per --chunk (records); store: also the '
                        'resident C2/C3 shard (diagnostic, no records at all)')
    p.add_argument('--store-chunk', type=int, default=25_000_000,
                   help='C4 streamed from the store: pairs per launch')
    p.add_argument('--resident-gb', type=float, default=150.0,
                   help='C4: keep a shard\'s records resident up to this many GB')
    p.add_argument('--stack', choices=('default', 'average', 'attention'), default='default',
                   help="layer stack: the default config.py:44-66 stack, tuning.py:66-93's "
                        "GCN-GCN-Average-NTN(16), or the same with Attention pooling "
                        "(layers.py:143-160)")
    p.add_argument('--collective', choices=('rccl', 'torch'), default='rccl',
                   help='N > 1: the gradient all-reduce as ncclAllReduce on the compute stream '
                        '(rccl) or through torch.distributed (side stream + events)')
    p.add_argument('--settle-ms', type=float, default=60.0,
                   help='untimed forward-only launches on the resident batch for at least this '
                        'long before the warmup steps (GPU clock settle; 0: none)')
    p.add_argument('--events', choices=('timed', 'after'), default='after',
                   help='where the HIP events around the step\'s kernels (the roofline\'s '
                        'kernel time) are recorded: on as many extra steps right after the '
                        'timed region (default), or on every timed step (the two timing '
                        'events of a step add ≈8 µs of dispatch gaps to it, profiles/r05_n)')
    p.add_argument('--no-fused-adam', action='store_true',
                   help='N = 1: run the gradient reduction and Adam as two launches '
                        '(sg_fwd_bwd + sg_adam_tf) instead of sg_train_step')
    p.add_argument('--json-out', default='')
    p.add_argument('--emulate-world', type=int, default=0,
                   help='diagnostic: time rank 0\'s share of a W-GPU step on one GPU (no collective)')
    p.add_argument('--emulate-collective', action='store_true',
                   help='with --emulate-world: step as a real rank does (fused kernel, gradient '
                        'reduction, ncclAllReduce of the flat gradient on a world-size-1 RCCL '
                        'communicator on the compute stream, Adam launch), so the collective\'s '
                        'launch cost is in the timed step (its data path is a 1-rank no-op)')
    return p.parse_args()


def fused_kernel_source_hash() -> str:
    """sha1 over the headline fused kernel's sources (csrc/sg_fast.hip and the headers it
    includes): profiles/traffic.json records it, and the bench line reports that file's
    PMC traffic only while the tree still hashes the same."""
    import hashlib
    h = hashlib.sha1()
    csrc = os.path.join(ROOT, 'graphembedding_amd', 'csrc')
    for f in ('sg_fast.hip', 'sg_mfma.h', 'sg_plan.h', 'sg_common.h'):
        with open(os.path.join(csrc, f), 'rb') as fh:
            h.update(fh.read())
    with open(os.path.join(ROOT, 'include', 'siamese_hip.h'), 'rb') as fh:
        h.update(fh.read())
    return h.hexdigest()


def cpu_baseline(gs, labels, flags, n_sample, D=None):
    """Time the oracle's C restatement (oracle/siamese_cpu.c, OpenMP) on a
    bounded sample of the same all-pairs stream, on this host's cores (all of
    them, and 1 thread as SURVEY §8(d) asks).  The C port's NTN dim is its record
    capacity, so C4 (D = 30) is timed on capacity-30 records."""
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    from oracle import cpu_ref
    if D is not None and D != gs.n_max:
        from types import SimpleNamespace
        from graphembedding_amd.packer import GraphStore
        gs = SimpleNamespace(graphs=gs.graphs, d_in=gs.d_in, n_max=D,
                             store=GraphStore(gs.mgs, D, gs.d_in))
    out = cpu_ref.time_allpairs_sample(gs, labels, flags, n_sample)
    one = cpu_ref.time_allpairs_sample(gs, labels, flags, 0, target_s=4.0, threads=1)
    out['value_1thread'] = one['value']
    out['sample_1thread'] = one['sample']
    return out


def time_preparation(model, gs, shard, batch, stream, args):
    """What the timed step leaves out (packing is reported separately):
    the device time of packing this rank's records (sg_pack_pairs over the shard's pair
    ids, the same call AllPairsShard makes once) and of the class order (sg_pair_order,
    once per packed batch).  Both run before the timed steps and are reused by every
    step; re-run here 3 times into scratch buffers and averaged (HIP events)."""
    import numpy as np
    import torch
    from graphembedding_amd.packer import pack_device_into
    G = len(gs.graphs)
    p = torch.arange(shard.start, shard.end, dtype=torch.int64, device=model.device)
    pi = torch.stack([p // G, p % G], dim=1).to(torch.int32).contiguous()
    recs = torch.empty_like(shard.records)
    status = torch.zeros(1, dtype=torch.int32, device=model.device)
    out = {}
    for what in ('pack', 'order'):
        if what == 'order' and batch.order is None:
            continue
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            if what == 'pack':
                pack_device_into(gs.store, pi, shard.labels, recs, status, dtype=args.records)
            else:
                model.balance(model.batch_from_records(recs, shard.n, shard.labels,
                                                       pair_offset=shard.start,
                                                       batch_total=shard.total,
                                                       y_stats=shard.y_stats))
            e1.record(stream)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[what + '_ms'] = float(np.mean(ts))
    del recs, pi, p
    torch.cuda.synchronize()
    return out


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` without a torchrun environment: start the N ranks as
    children under torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous)
    before this process touches the GPU, and return their exit status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node={}'.format(args.gpus), '--master-addr=127.0.0.1',
           '--master-port={}'.format(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    env_world = os.environ.get('WORLD_SIZE')
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if env_world is not None and int(env_world) != args.gpus and \
            os.environ.get('SG_BENCH_REHEARSAL') != '1':
        sys.exit('bench.py: --gpus {} but WORLD_SIZE={} (launch one rank per GPU)'.format(
            args.gpus, env_world))
    if args.gpus < 1:
        sys.exit('bench.py: --gpus must be >= 1')
    web = args.dataset == 'syn_web'
    if args.steps is None:
        args.steps = 3 if web else 50
    if args.warmup is None:
        args.warmup = 1 if web else 10
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # SG_BENCH_REHEARSAL=1 (diagnostic): every rank on cuda:0 over gloo, to rehearse the
    # multi-rank path (shards, all-reduce hook, barriers, max-over-ranks timing) on a
    # one-GPU box; its numbers are not a scaling measurement
    rehearsal = os.environ.get('SG_BENCH_REHEARSAL') == '1'
    if rehearsal:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if rehearsal:
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    device = torch.device('cuda', local)

    from graphembedding_amd import _lib
    from graphembedding_amd.allpairs import AllPairsShard, AllPairsStream, load_graph_set
    from graphembedding_amd.config import Flags
    from graphembedding_amd.model_mse import SiameseGCNTNMSE
    from graphembedding_amd.shard import make_allreduce_hook, make_rccl_hook

    c4 = args.dataset == 'syn_aids10knef'
    D = 512 if web else (30 if c4 else 10)
    fl = dict(dropout=args.dropout, record_dtype=args.records)
    if c4:   # AIDS10k: N <= 30 needs Padding / NTN input_dim 30
        fl.update(layer_3='Padding:max_in_dims=30,padding_value=0',
                  layer_4='NTN:input_dim=30,feature_map_dim=10,inneract=relu,dropout=True,'
                          'bias=True')
    if args.stack in ('average', 'attention'):   # the tuning.py stack (Average + NTN(16))
        fl.update(num_layers=4,
                  layer_2='Average' if args.stack == 'average' else 'Attention:input_dim=16',
                  layer_3='NTN:input_dim=16,feature_map_dim=10,inneract=relu,dropout=True,'
                          'bias=True')
    if web:   # Web: N <= 512 needs Padding / NTN input_dim 512
        fl.update(layer_3='Padding:max_in_dims=512,padding_value=0',
                  layer_4='NTN:input_dim=512,feature_map_dim=10,inneract=relu,dropout=True,'
                          'bias=True')
    flags = Flags(**fl)
    gs = load_graph_set(args.dataset, n_max=512 if web else (32 if c4 else 10),
                        with_store=not web)
    labels = gs.label_matrix(flags.yeta)
    model = SiameseGCNTNMSE(gs.d_in, flags, device=device, n_max=gs.n_max)
    assert model.n_max == gs.n_max
    ew = args.emulate_world if (args.emulate_world > 1 and world == 1) else 0
    srank, sworld = (0, ew) if ew else (rank, world)
    balance = args.order == 'class'
    streamed = False
    if web:
        from graphembedding_amd.web import WebAllPairs
        shard = WebAllPairs(gs, labels, srank, sworld, device=device, chunk=args.web_chunk)
        batch = shard.batch(model)
    elif c4:
        from graphembedding_amd.shard import shard_range
        a, b = shard_range(len(gs.graphs) ** 2, srank, sworld)
        from graphembedding_amd.packer import record_words
        streamed = (b - a) * 4 * record_words(gs.n_max, args.records) > args.resident_gb * 1e9
        # the capacity-32 kernel gathers pairs from the cache-resident dense store faster than
        # it reads 8.5 KB records from HBM (an emulated W = 8 rank's resident shard: 148.9
        # against 134.3 M pairs/s, profiles/r04_c4s/), so its shards are store-sourced
        # whatever their size (--source records packs and keeps records)
        if args.source == 'auto' and model.kernel_path == 2 and args.records == 'f32':
            streamed = True
    if streamed:
        store_src = args.source == 'auto' and model.kernel_path == 2 and args.records == 'f32'
        shard = AllPairsStream(gs, labels, srank, sworld, device=device,
                               chunk=args.store_chunk if store_src else args.chunk,
                               dtype=args.records, balance=balance,
                               source='records' if args.source == 'records' else 'auto')
        batch = None
    if not web and not streamed:
        shard = AllPairsShard(gs, labels, srank, sworld, device=device, dtype=args.records)
        batch = shard.batch(model, balance=balance)
        if args.source == 'store':   # same pairs, gathered by the kernel from the store
            batch = model.batch_from_store(gs.store, shard.n, batch.labels,
                                           grid_base=shard.start, pair_offset=shard.start,
                                           batch_total=shard.total, y_stats=batch.y_stats)
            batch = model.balance(batch) if balance else batch
    hook, collective = None, None
    if ew and args.emulate_collective:
        from graphembedding_amd.rccl import RcclComm
        from graphembedding_amd.shard import make_rccl_hook
        comm = RcclComm(0, 1, store=dist.HashStore())
        hook, collective = make_rccl_hook(comm), 'rccl'
    if world > 1:
        # RCCL on the compute stream, in order with the fused kernels (no side stream, no
        # cross-stream events: 8 us less per step than torch.distributed's RCCL call,
        # scripts/collective_overhead.py); torch.distributed for the gloo rehearsal
        collective = 'torch' if rehearsal else args.collective
        if collective == 'rccl':
            # every rank opens the communicator or none does (open_rccl agrees through the
            # process group before and after ncclCommInitRank), so the ranks fall back to
            # torch.distributed together and never wait on a communicator a peer abandoned
            from graphembedding_amd.rccl import open_rccl
            comm, why = open_rccl(rank, world)
            if comm is None:
                print('bench.py: direct RCCL unavailable ({}); torch.distributed all-reduce'.format(
                    why), file=sys.stderr, flush=True)
                collective = 'torch'
            else:
                if comm.device() != local:   # open_rccl's init thread must select our GPU
                    raise RuntimeError('RCCL communicator on GPU {} for local rank {}'.format(
                        comm.device(), local))
                hook = make_rccl_hook(comm)
        if collective == 'torch':
            hook = make_allreduce_hook()
    if not web:
        model.workspace(shard.chunk if streamed else batch.n_pairs)
    stream = torch.cuda.current_stream()
    prep = time_preparation(model, gs, shard, batch, stream, args) \
        if (not web and not streamed and args.source != 'store') else None
    if streamed and shard.keep_orders and shard.uses_store(model):
        # the store-sourced chunks' batches and class orders, built once before the timed
        # steps and reused by every step (AllPairsStream.prepare), as the resident shard's
        # packed, ordered batch is: their device time is reported as order_ms, outside value
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        shard.prepare(model)
        e1.record(stream)
        e1.synchronize()
        prep = {'order_ms': e0.elapsed_time(e1)}

    ev = []
    fuse_adam = not args.no_fused_adam and model.kernel_path == 1 and batch is not None and \
        batch.csr is None and batch.src is None

    def step(timed):
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        if streamed:
            shard.fwd_bwd(model, add_label_term=(rank == 0))
        elif hook is None and fuse_adam:
            # one process: the gradient reduction applies Adam in the same launch
            # (sg_train_step); N > 1 all-reduces the gradient between the two
            model.fwd_bwd_adam(batch, add_label_term=(rank == 0))
        else:
            model.fwd_bwd(batch, add_label_term=(rank == 0))
        if timed:
            e1.record(stream)
            ev.append((e0, e1))
        if streamed or hook is not None or not fuse_adam:
            if hook is not None:
                hook(model)
            model.apply_adam()
        model.step_count += 1

    # GPU clock settle (untimed, before the warmup steps): after the host-side setup the
    # first ≈15 fused launches on a fresh box run up to 9% slower and speed up launch by
    # launch (profiles/r05_h: 945 -> 866 µs over 20 launches of the same step), longer than
    # the driver's 5 warmup steps.  Forward-only launches of the resident batch (another
    # kernel instantiation: the profiled training kernel's average stays the training
    # launches') keep the GPU busy until the clock has settled; nothing of the timed step is
    # computed here or reused by it.
    settle_ms = 0.0
    if args.settle_ms > 0 and batch is not None and not web:
        torch.cuda.synchronize()
        t_s = time.perf_counter()
        while (time.perf_counter() - t_s) * 1e3 < args.settle_ms:
            for _ in range(4):
                model.pred_sim_without_act(batch)
            torch.cuda.synchronize()
        settle_ms = (time.perf_counter() - t_s) * 1e3
    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(args.events == 'timed')
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    params_agree = None
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # after timing: every rank must hold the same parameters (a wrong all-reduce
        # would let them drift apart); max and min of a checksum over ranks
        c = model.params.double().mul(torch.arange(1, model.params.numel() + 1, device=device,
                                                   dtype=torch.float64)).sum()
        ck = torch.stack([c, -c])
        dist.all_reduce(ck, op=dist.ReduceOp.MAX)
        params_agree = bool(float(ck[0].item()) == -float(ck[1].item()))
        if not params_agree:
            print('bench.py: parameters differ across ranks after the timed steps',
                  file=sys.stderr, flush=True)
    # the loss of the last timed step (before the event steps below move the parameters)
    loss = float(model.loss_buf[0].item() + model.reg_buf[0].item())
    event_steps = 0
    if args.events == 'after':
        # the roofline's kernel time: HIP events around as many extra training steps right
        # after the timed region (they keep training: params, Adam state and step_count
        # advance by event_steps more; params_agree and loss above are the timed run's)
        for _ in range(args.steps):
            step(True)
        torch.cuda.synchronize()
        event_steps = args.steps

    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    total_pairs = shard.total
    # the eval path (train.py:47-74 test matrix; pred_sim_without_act): forward only over
    # the same resident batch, one launch per pass (reported beside the training metric)
    fwd_rate = None
    if world == 1 and batch is not None and not ew:
        torch.cuda.synchronize()
        f0 = time.perf_counter()
        for _ in range(5):
            model.pred_sim_without_act(batch)
        torch.cuda.synchronize()
        fwd_rate = 5 * batch.n_pairs / (time.perf_counter() - f0)
    value = total_pairs * args.steps / elapsed
    if ew:
        value = shard.n * args.steps / elapsed   # diagnostic: one emulated rank's own rate

    if rank == 0:
        flops_pair = gs.flops_per_pair_web() if web else gs.flops_per_pair(
            D=D, pool={'default': 'padding'}.get(args.stack, args.stack))
        bytes_pair = gs.csr_bytes_per_pair() if web else shard.record_bytes
        kern_pairs_s = shard.n / (kern_ms * 1e-3)
        achieved_tf = kern_pairs_s * flops_pair / 1e12
        achieved_gbs = kern_pairs_s * bytes_pair / 1e9
        traffic, traffic_src = None, None
        tj = os.path.join(ROOT, 'profiles', 'traffic.json')
        if model.kernel_path == 1 and args.records == 'f32' and os.path.isfile(tj) and \
                args.stack == 'default' and args.source != 'store':
            with open(tj) as f:
                t = json.load(f)
            # HBM bytes per launch: PMC counters cannot be read from inside this process,
            # so they come from the committed rocprofv3 --pmc passes of this same command
            # on this tree (scripts/gpu_round3.sh + scripts/make_profile_summary.py), and
            # only while the fused kernel's sources are the ones those passes measured
            if t.get('sources_sha1') == fused_kernel_source_hash():
                traffic = t.get('traffic_bytes_per_launch') * shard.n / 490000.0
                traffic_src = ('profiles/{}/traffic.json (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE '
                               'passes of bench.py --gpus 1 on these kernel sources; FETCH_SIZE x2 '
                               'gfx950 correction)'.format(t.get('tree', '?')))
            else:
                traffic_src = ('none: profiles/traffic.json ({}) was measured on other sg_fast '
                               'sources'.format(t.get('tree', '?')))
        cpu = None
        if world == 1 and args.cpu_sample >= 0:
            try:
                if web:
                    sys.path.insert(0, os.path.join(ROOT, 'tests'))
                    from oracle import cpu_ref
                    gsd = gs
                    cpu = cpu_ref.time_web_sample(gsd, labels, flags, n_sample=64,
                                                  target_s=12.0)
                else:
                    cpu = cpu_baseline(gs, labels, flags, args.cpu_sample, D=D)
            except Exception as e:  # reported, never fatal for the GPU number
                cpu = {'value': None, 'unit': 'graph-pairs/s', 'cores': 0, 'kind': 'port',
                       'sample': 'failed: {}'.format(e)}
        name = 'Web' if web else ('AIDS10knef' if c4 else 'AIDS700')
        if web:
            workload = ('Web-sized all-pairs ({} synthetic graphs, N ~ U{{64..512}}, {:,} ordered '
                        'pairs), Padding/NTN 512'.format(len(gs.graphs), total_pairs))
            ws_gb = _lib.web_workspace_bytes(model.sg, shard.chunk) / 1e9
            inputs = ('CSR graph store + size-ordered pair ids resident in HBM, {} pairs per '
                      'internal chunk; workspace {:.1f} GB (two pipeline slots of NTN inputs, '
                      'keep bits and D2 rows at node capacity {})'.format(
                          shard.chunk, ws_gb, gs.n_max))
            records = 'CSR store (no pair records), {:.0f} B/pair of graph input'.format(bytes_pair)
        else:
            workload = ('AIDS10knef all-pairs (10,018 graphs, N <= 30, {:,} ordered '
                        'pairs), Padding/NTN 30' if c4 else
                        'AIDS700nef all-pairs (700 graphs, {:,} ordered pairs)').format(total_pairs)
            if streamed and shard.uses_store(model):
                inputs = ('graph store resident in HBM; the kernel gathers each pair\'s graphs '
                          '(no records), {} pairs per launch'.format(shard.chunk))
            elif streamed:
                inputs = 'packed in chunks of {} pairs inside the step'.format(shard.chunk)
            else:
                inputs = ('graph store resident in HBM; the kernel gathers each pair\'s graphs '
                          '(no records)' if args.source == 'store' else 'records resident in HBM')
            records = '{} Â, {} B/pair'.format(args.records, bytes_pair)
        out = {
            # BASELINE.json's metric string for the headline config (C2); the other
            # configs name their dataset the same way
            'metric': ('graph-pairs/sec (Siamese fwd+bwd), AIDS700 all-pairs @ 1/2/4/8 MI355X'
                       if name == 'AIDS700' else
                       'graph-pairs/sec (Siamese fwd+bwd), {} all-pairs'.format(name)),
            'value': value,
            'unit': 'graph-pairs/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': elapsed * 1e3 / args.steps,
            'higher_is_better': True,
            'scaling': 'strong',
            'vs_baseline': None,
            'dtype': 'f32',
            'data': 'synthetic ({}-shaped graphs + GED labels, BASELINE.md §3)'.format(
                'Web' if web else ('AIDS10knef' if c4 else 'AIDS700nef')),
            'config': {'workload': workload +
                                   {'default': ', default 5-layer Siamese GCN-NTN',
                                    'average': ', tuning.py GCN-GCN-Average-NTN(16) stack',
                                    'attention': ', GCN-GCN-Attention(16)-NTN(16) stack '
                                                 '(layers.py:143-160)'}[args.stack] +
                                   ', dropout {}'.format(args.dropout),
                       'global_batch': total_pairs, 'n_max': gs.n_max, 'd_in': gs.d_in,
                       'kernel_path': _lib.PATH_NAMES[model.kernel_path],
                       'records': records,
                       'order': 'size buckets' if web else args.order,
                       # device time of the once-per-batch preparation the timed steps reuse
                       # (records packed from the graph store; class order), outside `value`
                       'pack_ms': prep.get('pack_ms') if prep else None,
                       'order_ms': prep.get('order_ms') if prep else None,
                       # untimed forward-only launches before the warmup steps (clock settle)
                       'settle_ms': round(settle_ms, 1),
                       'inputs': inputs,
                       'parallelism': 'dp{}'.format(world),
                       'adam': ('in the gradient reduction\'s launch (sg_train_step)'
                                if (fuse_adam and hook is None) else 'sg_adam_tf launch'),
                       'collective': ('{} all-reduce of the flat gradient + loss ({} B)'.format(
                           'ncclAllReduce on the compute stream' if collective == 'rccl' else
                           'torch.distributed', 4 * (model.grad.numel() + 1))
                           if collective else None)},
            'roofline': {'bound': 'mfma', 'achieved': achieved_tf, 'peak': FP32_PEAK_TFLOPS,
                         'unit': 'TFLOP/s', 'frac': achieved_tf / FP32_PEAK_TFLOPS,
                         'traffic': traffic, 'traffic_source': traffic_src,
                         'note': 'fp32 compute roof (gfx950 vector fp32 == f32 MFMA peak); '
                                 'algorithmic {:.0f} FLOP/pair x {} pairs per launch / {} '
                                 'event time {:.3f} ms ({})'.format(
                                     flops_pair, shard.n,
                                     'sg_web_fwd_bwd (all its kernels)' if web else
                                     ('sg_train_step (fused kernel, then the gradient reduction '
                                      'with Adam)' if (fuse_adam and hook is None) else
                                      'sg_fwd_bwd'),
                                     kern_ms, 'events on every timed step'
                                     if args.events == 'timed' else
                                     'events on {} steps right after the timed region'.format(
                                         args.steps))},
            'roofline_hbm': {'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                             'frac': achieved_gbs / HBM_PEAK_GBS,
                             'bytes_per_pair': bytes_pair},
            'cpu_baseline': cpu,
            'forward_pairs_per_s': fwd_rate,
            'loss': loss,
            'event_steps_after_timed': event_steps,
            'params_agree_across_ranks': params_agree,
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, 'w') as f:
                f.write(line + '\n')
    if collective == 'rccl':
        comm.destroy()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
