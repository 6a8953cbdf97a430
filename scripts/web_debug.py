"""Diagnostic (GPU): compare the graph-store path's intermediate buffers (NTN
inputs X1/X2 and T = W·x2) with the oracle's for one small C5-shaped case."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests')]


def main(dropout=0.1):
    import torch
    assert torch.cuda.is_available()
    from _fixtures import small_problem
    from oracle import siamese_oracle as O
    prob = small_problem(n_graphs=10, n_pairs=24, seed=31, n_lo=20, n_hi=60, n_max=64,
                         flags_overrides=dict(dropout=dropout))
    model, batch = prob.make_gpu_web_model(device='cuda')
    seed = 4321
    s = model.pred_sim_without_act(batch, seed=seed).cpu().numpy()
    ws = model._web_ws.cpu().numpy()
    P, Dp, K, D = batch.n_pairs, 128, 10, 64
    Cp = (batch.chunk + 127) // 128 * 128
    X1 = ws[:Cp * Dp].reshape(Cp, Dp)[:P]
    X2 = ws[Cp * Dp:2 * Cp * Dp].reshape(Cp, Dp)[:P]
    toff = 4 * Cp * Dp
    T = ws[toff:toff + Cp * K * Dp].reshape(Cp, K, Dp)[:P]
    spec = prob.oracle_spec()
    Pm = O.unflatten(spec, prob.params.astype(np.float64))
    g1, g2 = prob.oracle_graphs()
    for i in range(3):
        sref, c = O.pair_forward(spec, Pm, g1[i], g2[i], i, seed)
        n1, n2 = g1[i].n, g2[i].n
        print('pair', i, 'n', n1, n2, 's gpu {:.6f} ref {:.6f}'.format(s[i], sref))
        print('  x1 err', np.abs(X1[i, :D] - c['x1']).max(), 'x1 tail', np.abs(X1[i, D:]).max())
        print('  x2 err', np.abs(X2[i, :D] - c['x2']).max())
        u = c['u']   # [a][k] = Σ_b W[a][b][k] x2[b]
        print('  T err (a<n1)', np.abs(T[i, :, :n1].T - u[:n1]).max(), 'u max', np.abs(u).max())
        W = Pm[(4, 'weights_W')]
        err = np.abs(T[i, :, :n1].T - u[:n1]).max(axis=1)
        print('  T err by a/16', [float(np.round(err[a:a + 16].max(), 4)) for a in range(0, n1, 16)])
        for bt in (16, 32, 48, 64):
            x2t = c['x2'].copy(); x2t[bt:] = 0
            ut = np.einsum('abk,b->ak', W, x2t)
            print('  vs x2[:%d]' % bt, np.abs(T[i, :, :n1].T - ut[:n1]).max())


if __name__ == '__main__':
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 0.1)
