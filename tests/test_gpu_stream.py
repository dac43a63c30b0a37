"""GPU parity of the single-launch streamed forward (csrc/dadmm_stream.hip): the shapes the fused
kernel cannot hold on chip with m <= 64 and P <= 16 (BASELINE configs[2]: P = 16, n = 512,
m = 64) run all K iterations in one launch, R_k held in registers, U_k streamed in place.

Bar: bit-exact (np.array_equal on every iterate and on U_K) against oracle.forward_f32, and
bit-identical to the per-iteration launches of the tiled path (DADMM_TILED_STREAM=0), which the
same tests run as the second form. Reference: unfolded_DLASSO.py:53-107, :127-140 and the GNN
variant's clamps (gnn_dlasso_models_progressive.py:205-232)."""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu

MAXP = [0.1, 0.99, 0.99, 0.99]


def _inits(B, P, n, seed=99):
    rng = np.random.default_rng(seed)
    return (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _run(dev, A, b, graphs, hyp, y0, U0, d0, variant=0, want_U=True):
    from dadmm_hip import PreparedOperator, forward_raw, ingest
    B = y0.shape[0]
    op = PreparedOperator(_t(A, dev))
    g = ingest(graphs, A.shape[0], B, dev)
    Y, U, st = forward_raw(op, _t(b, dev), g, _t(hyp, dev), _t(y0, dev), _t(U0, dev),
                           _t(d0, dev), variant=variant, want_U=want_U, path="tiled")
    torch.cuda.synchronize()
    return Y.cpu().numpy(), (U.cpu().numpy() if U is not None else None), int(st.item())


# (P, m, n, B, K, graph prob, per-sample graphs, variant, hyp rows)
SHAPES = [
    (16, 64, 512, 37, 6, 0.3, True, 0, 16),   # configs[2] agents / size, ragged batch
    (16, 64, 500, 20, 4, 0.3, True, 1, 16),   # n not a multiple of 32 (padded block), GNN clamps
    (12, 48, 256, 33, 5, 0.5, False, 0, 1),   # shared graph, 'same' mode, m < 64
    (8, 64, 128, 16, 3, 0.6, True, 0, 8),     # one agent per wave, the shortest ring (4 blocks)
    (1, 16, 192, 5, 4, 0.5, False, 0, 1),     # a single agent: no consensus
    (9, 40, 320, 18, 1, 0.4, True, 0, 9),     # K = 1: no GEMM1 beyond R_0
    (16, 64, 512, 16, 2, 1.0, False, 1, 16),  # complete graph: the longest visit rows (2 (P - 1))
]


@pytest.mark.parametrize("form", ["stream", "launches"])
@pytest.mark.parametrize("P,m,n,B,K,prob,per_sample,variant,H", SHAPES)
def test_tiled_forms_bit_exact(cuda, monkeypatch, form, P, m, n, B, K, prob, per_sample, variant, H):
    monkeypatch.setenv("DADMM_TILED_STREAM", "1" if form == "stream" else "0")
    A, b, _ = O.make_problem(P, m, n, B, seed=31 * P + n)
    graphs = ([O.connected_er_graph(P, prob, seed=500 + s) for s in range(B)] if per_sample
              else [O.er_graph(P, prob, seed=7)] * B)
    y0, U0, d0 = _inits(B, P, n, seed=B + K)
    rng = np.random.default_rng(P + K)
    hyp = O.hyp_table((0.5 * rng.standard_normal((K, H, 4))).astype(np.float32), MAXP)
    Y, U, st = _run(cuda, A, b, graphs, hyp, y0, U0, d0, variant=variant)
    Yo, Uo, sto = O.forward_f32(A, b, graphs, hyp, y0, U0, d0, variant=variant)
    assert st == sto == 0
    assert np.array_equal(Y, Yo), f"max |diff| {np.abs(Y - Yo).max()}"
    assert np.array_equal(U, Uo), f"U_K max |diff| {np.abs(U - Uo).max()}"


def test_stream_without_U_out(cuda, monkeypatch):
    """want_U = False: the launch skips the final dual-update phase; Y is unchanged."""
    monkeypatch.setenv("DADMM_TILED_STREAM", "1")
    P, m, n, B, K = 16, 64, 512, 24, 5
    A, b, _ = O.make_problem(P, m, n, B, seed=3)
    graphs = [O.connected_er_graph(P, 0.3, seed=s) for s in range(B)]
    y0, U0, d0 = _inits(B, P, n, seed=4)
    rng = np.random.default_rng(5)
    hyp = O.hyp_table((0.5 * rng.standard_normal((K, P, 4))).astype(np.float32), MAXP)
    Y, U, st = _run(cuda, A, b, graphs, hyp, y0, U0, d0, want_U=False)
    Yo, _, _ = O.forward_f32(A, b, graphs, hyp, y0, U0, d0)
    assert U is None and st == 0
    assert np.array_equal(Y, Yo)


def test_stream_flags_nonfinite_inputs(cuda, monkeypatch):
    """The streamed launch flags every case where one of the reference's batch-global guards
    fires (unfolded_DLASSO.py:55-61, 84-86, 102-104); path='tiled' has no recompute behind it."""
    monkeypatch.setenv("DADMM_TILED_STREAM", "1")
    P, m, n, B, K = 10, 32, 128, 19, 3
    A, b, _ = O.make_problem(P, m, n, B, seed=1)
    G = O.er_graph(P, 0.5, seed=1)
    y0, U0, d0 = _inits(B, P, n)
    hyp = O.hyp_table(np.zeros((K, P, 4), np.float32), MAXP)
    run = lambda *a: _run(cuda, A, *a)[2]   # noqa: E731
    b2 = b.copy(); b2[3, 1, 2] = np.nan
    assert run(b2, [G] * B, hyp, y0, U0, d0) & 4
    y2 = y0.copy(); y2[18, 9, 127] = np.inf
    assert run(b, [G] * B, hyp, y2, U0, d0) & 1
    U2 = U0.copy(); U2[7, 2, 63] = -np.inf
    assert run(b, [G] * B, hyp, y0, U2, d0) & 2
    h2 = hyp.copy(); h2[1, 9, 0] = np.nan
    assert run(b, [G] * B, h2, y0, U0, d0) & 8
    assert run(b, [G] * B, hyp, y0, U0, d0) == 0


@pytest.mark.parametrize("P,m,n,B,K,prob,per_sample,variant,H", [
    (16, 64, 512, 37, 6, 0.3, True, 0, 16),
    (9, 40, 320, 18, 5, 0.4, True, 1, 1),
    (8, 64, 128, 16, 3, 0.6, False, 0, 8),
])
def test_stream_recording_bit_exact(cuda, P, m, n, B, K, prob, per_sample, variant, H):
    """Training forward (record=True) on the streamed launch (dadmm_forward_tiled_record): Y, U_K
    and the adjoint's trajectory Grec / Urec bit-exact against oracle.forward_f32_rec, and the
    general adjoint on it agrees with the one on the stepwise recording."""
    from dadmm_hip import PreparedOperator, forward_raw, ingest
    from dadmm_hip.ops import backward_raw
    A, b, _ = O.make_problem(P, m, n, B, seed=7 * P + n)
    graphs = ([O.connected_er_graph(P, prob, seed=900 + s) for s in range(B)] if per_sample
              else [O.er_graph(P, prob, seed=9)] * B)
    y0, U0, d0 = _inits(B, P, n, seed=K)
    rng = np.random.default_rng(P * K)
    hyp = O.hyp_table((0.5 * rng.standard_normal((K, H, 4))).astype(np.float32), MAXP)
    op = PreparedOperator(_t(A, cuda))
    g = ingest(graphs, P, B, cuda)
    outs = {}
    for path in ("auto", "stepwise"):
        Y, U, st, traj = forward_raw(op, _t(b, cuda), g, _t(hyp, cuda), _t(y0, cuda), _t(U0, cuda),
                                     _t(d0, cuda), variant=variant, want_U=True, path=path,
                                     record=True)
        torch.cuda.synchronize()
        outs[path] = (Y, U, int(st.item()), traj)
    Yo, Uo, sto, Go, Uro = O.forward_f32_rec(A, b, graphs, hyp, y0, U0, d0, variant=variant)
    for path, (Y, U, st, traj) in outs.items():
        assert st == sto == 0, path
        assert np.array_equal(Y.cpu().numpy(), Yo), path
        assert np.array_equal(U.cpu().numpy(), Uo), path
        assert np.array_equal(traj.Grec[..., :n].cpu().numpy(), Go), path
        assert np.array_equal(traj.Urec[..., :n].cpu().numpy(), Uro), path
    gY = np.random.default_rng(3).standard_normal((K, B, P, n)).astype(np.float32)
    dh = [backward_raw(op, g, outs[p][3], _t(gY, cuda)).cpu().numpy() for p in ("auto", "stepwise")]
    assert np.array_equal(dh[0], dh[1])


@pytest.mark.parametrize("case", ["b_nan", "hyp_nan", "y0_inf"])
def test_stream_recording_guard_fired_matches_stepwise(cuda, case):
    """a training forward (record=True, path='auto': the streamed recording launch)
    whose inputs fire one of the reference's batch-global guards is redone by the gated stepwise
    recomputation, which re-records Grec / Urec. Y, U_K, the status, Grec, Urec and the adjoint
    on that trajectory must be bit-identical to the stepwise recording (path='stepwise'), and Y /
    U_K / the trajectory to oracle.forward_f32_rec (unfolded_DLASSO.py:55-61, 84-86, 102-104)."""
    from dadmm_hip import PreparedOperator, forward_raw, ingest
    from dadmm_hip.ops import backward_raw
    P, m, n, B, K = 16, 64, 512, 21, 4
    A, b, _ = O.make_problem(P, m, n, B, seed=44)
    graphs = [O.connected_er_graph(P, 0.3, seed=1300 + s) for s in range(B)]
    y0, U0, d0 = _inits(B, P, n, seed=45)
    rng = np.random.default_rng(46)
    hyp = O.hyp_table((0.5 * rng.standard_normal((K, P, 4))).astype(np.float32), MAXP)
    if case == "b_nan":
        b = b.copy(); b[5, 3, 7] = np.nan
    elif case == "hyp_nan":
        hyp = hyp.copy(); hyp[2, 11, 0] = np.nan
    else:
        y0 = y0.copy(); y0[20, 15, 511] = np.inf
    op = PreparedOperator(_t(A, cuda))
    g = ingest(graphs, P, B, cuda)
    outs = {}
    for path in ("auto", "stepwise"):
        Y, U, st, traj = forward_raw(op, _t(b, cuda), g, _t(hyp, cuda), _t(y0, cuda), _t(U0, cuda),
                                     _t(d0, cuda), want_U=True, path=path, record=True)
        torch.cuda.synchronize()
        outs[path] = (Y.cpu().numpy(), U.cpu().numpy(), int(st.item()),
                      traj.Grec[..., :n].cpu().numpy(), traj.Urec[..., :n].cpu().numpy(), traj)
    Yo, Uo, sto, Go, Uro = O.forward_f32_rec(A, b, graphs, hyp, y0, U0, d0)
    assert sto != 0
    for path, (Y, U, st, Gr, Ur, _) in outs.items():
        assert st == sto, (path, st, sto)
        assert np.array_equal(Y, Yo, equal_nan=True), path
        assert np.array_equal(U, Uo, equal_nan=True), path
        assert np.array_equal(Gr, Go, equal_nan=True), path
        assert np.array_equal(Ur, Uro, equal_nan=True), path
    gY = np.random.default_rng(47).standard_normal((K, B, P, n)).astype(np.float32)
    dh = [backward_raw(op, g, outs[p][5], _t(gY, cuda)).cpu().numpy() for p in ("auto", "stepwise")]
    assert np.array_equal(dh[0], dh[1], equal_nan=True)
