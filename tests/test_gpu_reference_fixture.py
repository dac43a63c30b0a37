"""The reference's own published configuration through the drop-in module on the GPU.

Operands are the reference's shipped data fixtures (tests/golden/make_fixtures.py, read without
unpickling): results/25_iter_general_learning/A.pt, fp32 [1, 5, 100, 500] — the reference's
default m = 100 rows per agent and n = 500 (configurations.py:6-9) — and the trained
seq_hyp.param [25, 5, 4] of the same run (model.pt). Inputs follow gnn_data.set_Data
(x* = 2 N(0,1) Bernoulli(0.25), b_p = A_p x*, gnn_data.py:6-15) and the reference driver's
single ER graph replicated over the batch (unfolded_train_new.py:56, 67).

Bar (the same as every GPU parity test):
  * forward: Y bit-exact (np.array_equal) vs oracle.forward_f32, the order-matched fp32
    restatement of unfolded_DLASSO.py:34-140; final-iterate MSE <= 1e-5 vs oracle.forward_f64
    (the reference's Gram-form algorithm in fp64; BASELINE north_star tolerance);
  * training step (model.train(), compute_loss, loss_final.backward() as unfolded_train_new.py:
    74-80): seq_hyp.param.grad within 1e-4 x max |grad| of the oracle adjoint
    (oracle.backward_np64, pinned to torch autograd through the reference's op sequence) chained
    through the hyper-parameter table.
Parity with the reference's own outputs is unpinned: the reference ships no (b, graph, Y) tuples.
"""
import argparse
import os

import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
A_REF = np.load(os.path.join(GOLD, "fixture_25_iter_general_learning_A.npy"))          # [1,5,100,500]
PARAM_REF = np.load(os.path.join(GOLD, "fixture_25_iter_general_learning_seq_hyp_param.npy"))
MAXP = [0.1, 0.99, 0.99, 0.99]


def _args(K=25):
    # configurations.py defaults the module reads (DADMM_mode 'diff', the maxima, the penalty)
    return argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99,
                              rho_max=0.99, eta_max=0.99, max_penalty_threshold=0.8,
                              penalty_reduction_factor=0.95)


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _data(B, seed):
    """set_Data (gnn_data.py:6-15) on the fixture operator: x*, b_p = A_p x* (noise-free)."""
    rng = np.random.default_rng(seed)
    n = A_REF.shape[-1]
    x = (2.0 * rng.standard_normal((B, n)) * (rng.random((B, n)) <= 0.25)).astype(np.float32)
    b = np.einsum("pmn,bn->bpm", A_REF[0].astype(np.float64), x).astype(np.float32)
    inits = (1e-2 * rng.standard_normal((3, B, 5, n))).astype(np.float32)
    return x, b, inits


def _model(dev, K=25):
    import unfolded_DLASSO
    model = unfolded_DLASSO.DLASSO_unfolded(_t(A_REF, dev), _args(K)).to(dev)
    with torch.no_grad():
        model.seq_hyp.param.copy_(torch.from_numpy(PARAM_REF[:K]))
    return model


def test_fixture_shapes():
    assert A_REF.shape == (1, 5, 100, 500) and A_REF.dtype == np.float32
    assert PARAM_REF.shape == (25, 5, 4)


@pytest.mark.parametrize("path", ["auto", "stepwise"])
def test_reference_operator_forward_bit_exact(cuda, path):
    """DLASSO_unfolded.forward at the reference's m = 100, n = 500 with its trained table (eval
    mode, B = 32, K = 25). "auto" runs the tiled path (two m-groups per agent), "stepwise" the
    guarded per-iteration kernels."""
    from dadmm_hip import PreparedOperator, forward_raw, ingest
    B, K, P = 32, 25, 5
    x, b, (y0, U0, d0) = _data(B, seed=3)
    graphs = [O.er_graph(P, 0.5, seed=7)] * B
    model = _model(cuda, K).eval()
    with torch.no_grad():
        if path == "auto":
            Y, hyp = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in (y0, U0, d0)))
            Y = Y[..., 0]
            st = int(model.last_status.item())
        else:
            op = PreparedOperator(_t(A_REF, cuda))
            Y, _, st = forward_raw(op, _t(b, cuda), ingest(graphs, P, B, cuda),
                                   model.hyp_table(K).detach(), _t(y0, cuda), _t(U0, cuda), _t(d0, cuda),
                                   path="stepwise")
            st = int(st.item())
    table = model.hyp_table(K).detach().cpu().numpy()
    # the module's table (torch cumsum/sigmoid on the device) is what the kernel consumes and what
    # the oracle is given; the numpy restatement of seq_hyperparam agrees to rounding
    np.testing.assert_allclose(table, O.hyp_table(PARAM_REF, MAXP), rtol=1e-6)
    Yo, _, sto = O.forward_f32(A_REF[0], b, graphs, table, y0, U0, d0)
    assert st == sto == 0
    Y = Y.cpu().numpy()
    assert np.array_equal(Y, Yo), f"max |diff| {np.abs(Y - Yo).max():.3e}"
    Y64, _, _ = O.forward_f64(A_REF[0], b, graphs, table, y0, U0, d0)
    mse = float(((Y[-1].astype(np.float64) - Y64[-1]) ** 2).mean())
    assert mse <= 1e-5, mse


def test_reference_defaults_training_step(cuda):
    """One training step of unfolded_train_new.py:74-80 at the reference's defaults
    (m = 100, n = 500, P = 5, K = 25 trained table, batch 32): forward in train mode, compute_loss,
    loss_final.backward() through the general adjoint (dadmm_adjoint)."""
    import gnn_dlasso_utils
    import unfolded_DLASSO
    B, K, P = 32, 25, 5
    x, b, (y0, U0, d0) = _data(B, seed=5)
    graphs = [O.er_graph(P, 0.5, seed=7)] * B
    model = _model(cuda, K).train()
    Y, _ = model(_t(b, cuda)[..., None], graphs, inits=tuple(_t(v, cuda) for v in (y0, U0, d0)))
    label = _t(x, cuda)[..., None]
    loss_mean, loss_final = gnn_dlasso_utils.compute_loss(Y, label)
    loss_final.backward()
    got = model.seq_hyp.param.grad.cpu().numpy().astype(np.float64)
    assert np.isfinite(got).all() and np.abs(got).max() > 0

    table = model.seq_hyp.table(K).detach().cpu().numpy()
    Yo, _, sto, Go, Uro = O.forward_f32_rec(A_REF[0], b, graphs, table, y0, U0, d0)
    assert sto == 0
    assert np.array_equal(Y[..., 0].detach().cpu().numpy(), Yo)
    n = A_REF.shape[-1]
    gY = np.zeros((K, B, P, n))
    gY[-1] = 2.0 * (Yo[-1].astype(np.float64) - x[:, None, :]) / (B * n * P)
    dtab = O.backward_np64(A_REF[0], graphs, table, y0, d0, Yo, Go, Uro, gY)
    seq = unfolded_DLASSO.seq_hyperparam([K, P, 4], torch.tensor(MAXP, dtype=torch.float64), _args(K))
    seq.param = torch.nn.Parameter(torch.tensor(PARAM_REF, dtype=torch.float64))
    seq.train()
    want, = torch.autograd.grad(seq.table(K), seq.param, grad_outputs=torch.from_numpy(dtab))
    want = want.numpy()
    err = np.abs(got - want)
    assert (err <= 1e-4 * np.abs(want).max() + 1e-4 * np.abs(want)).all(), \
        f"max err {err.max():.3e} of max |grad| {np.abs(want).max():.3e}"
