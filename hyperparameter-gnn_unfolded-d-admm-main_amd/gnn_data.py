"""Drop-in ``gnn_data``: the synthetic LASSO dataset the drivers train on.

Reference gnn_data.py:6-27. x* = 2 N(0,1) * Bernoulli(0.25) [N,n,1]; b_p = A_p x* [N,P,m,1]. The
reference first draws a noisy b with sigma = 10^(-snr/40) and then overwrites every agent's slice
with the noise-free product (:9-14); the noise draw is kept so the RNG stream stays aligned.
"""
from __future__ import annotations

import torch
from torch.utils.data import DataLoader, Dataset


def set_Data(A, data_len, args):
    device = A.device
    sigma = torch.pow(10, torch.tensor(-args.snr / 40, device=device))
    _, P, m, n = A.shape
    # one expression in the reference: randn is drawn before rand (gnn_data.py:8)
    x = 2 * torch.randn(data_len, n, 1, device=device)
    x = x * (torch.rand(data_len, n, 1, device=device) <= 0.25)
    noisy = torch.randn(data_len, P, m, 1, device=device) * sigma   # overwritten: noise-free b
    del noisy
    b = torch.einsum('pmn,snc->spmc', A[0], x).contiguous()
    return DataLoader(GNN_Data(b, x), batch_size=args.batch_size, shuffle=True, drop_last=True)


class GNN_Data(Dataset):
    """(b [P,m,1], x* [n,1]) pairs."""

    def __init__(self, b, y):
        self.b = b
        self.y = y

    def __len__(self):
        return self.b.shape[0]

    def __getitem__(self, item):
        return self.b[item], self.y[item]
