"""north_star's tolerance against the reference-form CPU forward.

BASELINE.json north_star: "final-iterate MSE <= 1e-5 vs CPU reference". Importing or running the
reference itself is denied here, so the closest CPU reference is
``oracle.ref_torch.forward``: the reference's own op sequence replayed with torch eager ops in
fp32 on the CPU — the Gram matrix AtA and per-agent GEMVs (unfolded_DLASSO.py:16, :69-71),
compute_Atx (:120-124), the gradient / clamp / update expressions (:73-99) and the Python edge
loop of compute_delta (:127-140). These tests run the drop-in module (DLASSO_unfolded.forward on
the GPU, HIP kernels) on the same A, b, graph, inits and hyper-parameters and assert the
final-iterate MSE against that replay, at the headline shape (a 32-sample slice) and at
BASELINE configs[0] (P=5, n=200, m=50, B=32, K=15). Stated tolerance: 1e-5 (north_star).
"""
import argparse
import os

import numpy as np
import pytest
import torch

import oracle as O
from oracle import ref_torch

pytestmark = pytest.mark.gpu

TOL = 1e-5
TRAINED = np.load(os.path.join(os.path.dirname(__file__), "golden",
                               "fixture_25_iter_general_learning_seq_hyp_param.npy"))


def _module_vs_ref(dev, P, m, n, B, K, param, seed):
    import unfolded_DLASSO
    A, b, _ = O.make_problem(P, m, n, B, seed=seed)
    G = O.er_graph(P, 0.5, seed=7)
    rng = np.random.default_rng(99)
    y0, U0, d0 = (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)
    args = argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99,
                              rho_max=0.99, eta_max=0.99, max_penalty_threshold=0.8,
                              penalty_reduction_factor=0.95)
    model = unfolded_DLASSO.DLASSO_unfolded(torch.from_numpy(A)[None].to(dev), args).to(dev).eval()
    with torch.no_grad():
        model.seq_hyp.param.copy_(torch.from_numpy(param))
        Y, hyp = model(torch.from_numpy(b).to(dev)[..., None], [G] * B,
                       inits=tuple(torch.from_numpy(v).to(dev) for v in (y0, U0, d0)))
        table = model.hyp_table(K).cpu().numpy()
    assert model.guard_warnings() == []
    Y = Y[..., 0].cpu().numpy()
    Yr = ref_torch.forward(A, b, [G] * B, table, y0, U0, d0)
    Y64, _, _ = O.forward_f64(A, b, [G] * B, table, y0, U0, d0)
    mse = lambda a, c: float(((a[-1] - c[-1]) ** 2).mean())   # noqa: E731
    return mse(Y, Yr), mse(Yr, Y64), mse(Y, Y64)


def test_headline_slice_vs_reference_form(cuda):
    """H = (P 5, n 256, m 64, K 25), 32 problems, the trained seq_hyp fixture."""
    m_ref, m_ref64, m_64 = _module_vs_ref(cuda, 5, 64, 256, 32, 25, TRAINED, 1234)
    assert m_ref <= TOL, (m_ref, m_ref64, m_64)


@pytest.mark.parametrize("kind", ["reference_default_init", "trained"])
def test_configs0_vs_reference_form(cuda, kind):
    """BASELINE configs[0] = (P 5, n 200, m 50, B 32, K 15): the reference's default
    hyper-parameter init (param = 0) and the trained fixture's first 15 rows."""
    param = np.zeros((15, 5, 4), np.float32) if kind == "reference_default_init" else TRAINED[:15]
    m_ref, m_ref64, m_64 = _module_vs_ref(cuda, 5, 50, 200, 32, 15, param, 1200)
    assert m_ref <= TOL, (m_ref, m_ref64, m_64)
