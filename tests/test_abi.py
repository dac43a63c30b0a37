"""CPU: the C-ABI library loads, exports every symbol include/dadmm.h declares, and validates its
arguments before touching the GPU (no kernel is launched by these tests)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dadmm.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dadmm_[a-z_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def L():
    from dadmm_hip import _lib
    return _lib.load()


def test_header_and_binding_agree():
    from dadmm_hip import _lib
    assert _declared() == sorted(_lib.EXPORTED_SYMBOLS)


def test_every_declared_symbol_is_exported(L):
    for name in _declared():
        assert hasattr(L, name), name


def test_abi_version(L):
    from dadmm_hip import _lib
    assert L.dadmm_abi_version() == _lib.ABI_VERSION


def _dims(**kw):
    from dadmm_hip import _lib
    d = dict(B=8, P=5, m=64, n=256, K=25, variant=0, hyp_rows=5, graph_shared=1)
    d.update(kw)
    return _lib.Dims(**d)


def test_operator_bytes(L):
    d = _dims()
    assert L.dadmm_operator_bytes(ctypes.byref(d)) == 2 * 4 * 5 * 64 * 256
    d = _dims(n=200)
    assert L.dadmm_operator_bytes(ctypes.byref(d)) == 2 * 4 * 5 * 64 * 256   # n padded to 256
    d = _dims(P=0)
    assert L.dadmm_operator_bytes(ctypes.byref(d)) == 0


FAKE = [ctypes.c_void_p(0x10000 * (i + 1)) for i in range(12)]   # 16-B aligned, never touched
FAKE.insert(3, None)                                                 # nbr_order: ascending


def _fwd(L, d):
    return L.dadmm_forward(ctypes.byref(d), *FAKE, None)


@pytest.mark.parametrize("kw,code", [
    (dict(P=0), -1), (dict(P=256), -1), (dict(P=65, n=64, hyp_rows=1), -2), (dict(m=0), -1), (dict(n=-3), -1), (dict(K=-1), -1),
    (dict(variant=2), -1), (dict(hyp_rows=3), -1), (dict(graph_shared=2), -1),
    (dict(m=65), -2), (dict(n=258), -2), (dict(P=7, n=64, hyp_rows=1), -2),
    (dict(P=6, n=256, hyp_rows=6), -2),
    (dict(n=512), -2), (dict(B=1 << 20, n=256), -2),
])
def test_forward_rejects_before_launch(L, kw, code):
    d = _dims(**kw)
    assert _fwd(L, d) == code
    assert L.dadmm_last_error().decode()


def test_forward_order_needs_per_sample_graphs(L):
    args = list(FAKE)
    args[3] = ctypes.c_void_p(0x90000)
    assert L.dadmm_forward(ctypes.byref(_dims(graph_shared=1)), *args, None) == -1
    assert L.dadmm_forward(ctypes.byref(_dims(graph_shared=0, P=9, hyp_rows=1)), *args, None) == -1


def test_forward_empty_work_is_ok(L):
    assert _fwd(L, _dims(B=0)) == 0
    assert _fwd(L, _dims(K=0)) == 0
    assert L.dadmm_last_error().decode() == ""


def test_forward_null_and_misaligned_pointers(L):
    d = _dims()
    args = list(FAKE)
    args[1] = None        # b
    assert L.dadmm_forward(ctypes.byref(d), *args, None) == -1
    args = list(FAKE)
    args[10] = ctypes.c_void_p(0x10004)  # Y misaligned
    assert L.dadmm_forward(ctypes.byref(d), *args, None) == -1
    assert "aligned" in L.dadmm_last_error().decode()


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from dadmm_hip import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(ImportError):
        _lib.load()


# ---- training path: recording forward and the adjoint (argument validation only) -----------------
REC = FAKE[:10] + [ctypes.c_void_p(0xA0000), ctypes.c_void_p(0xB0000)] + FAKE[10:]  # Y, Grec, Urec


def test_forward_record_rejects_before_launch(L):
    d = _dims()
    args = list(REC)
    args[11] = None        # Grec
    assert L.dadmm_forward_record(ctypes.byref(d), *args, None) == -1
    assert "Grec" in L.dadmm_last_error().decode()
    args = list(REC)
    args[12] = ctypes.c_void_p(0xB0008)   # Urec misaligned
    assert L.dadmm_forward_record(ctypes.byref(d), *args, None) == -1
    assert L.dadmm_forward_record(ctypes.byref(_dims(P=7, n=64, hyp_rows=1)), *REC, None) == -2
    assert L.dadmm_forward_record(ctypes.byref(_dims(B=0)), *REC, None) == 0


BWD = [ctypes.c_void_p(0x10000 * (i + 1)) for i in range(14)]
BWD[2] = None   # nbr_order: ascending


def test_backward_scratch_bytes(L):
    d = _dims(B=40)
    assert L.dadmm_backward_scratch_bytes(ctypes.byref(d)) == 4 * 3 * 25 * 5 * 4   # ceil(40/16) wgs
    assert L.dadmm_backward_scratch_bytes(ctypes.byref(_dims(P=0))) == 0


@pytest.mark.parametrize("kw,code", [
    (dict(P=0), -1), (dict(hyp_rows=3), -1), (dict(m=65), -2), (dict(n=258), -2),
    (dict(P=7, n=64, hyp_rows=1), -2), (dict(P=6, n=256, hyp_rows=6), -2), (dict(n=512), -2),
])
def test_backward_rejects_before_launch(L, kw, code):
    assert L.dadmm_backward(ctypes.byref(_dims(**kw)), *BWD, None) == code
    assert L.dadmm_last_error().decode()


def test_backward_null_and_misaligned(L):
    d = _dims()
    args = list(BWD)
    args[11] = None   # gY
    assert L.dadmm_backward(ctypes.byref(d), *args, None) == -1
    args = list(BWD)
    args[12] = None   # dhyp
    assert L.dadmm_backward(ctypes.byref(d), *args, None) == -1
    args = list(BWD)
    args[9] = ctypes.c_void_p(0x10004)   # Grec misaligned
    assert L.dadmm_backward(ctypes.byref(d), *args, None) == -1
    assert L.dadmm_backward(ctypes.byref(_dims(K=0)), *BWD, None) == 0


def test_stepwise_record_pointers_both_or_neither(L):
    d = _dims(graph_shared=1)
    args = [ctypes.c_void_p(0x10000 * (i + 1)) for i in range(11)]   # op .. U_out
    scratch = ctypes.c_void_p(0x100000)
    assert L.dadmm_forward_stepwise(ctypes.byref(d), *args, ctypes.c_void_p(0xA0000), None,
                                    ctypes.c_void_p(0xC0000), 0, scratch, None) == -1
    assert "both" in L.dadmm_last_error().decode()


def _fk(i):
    return ctypes.c_void_p(0x10000 * (i + 1))


@pytest.mark.parametrize("kw,code", [
    (dict(K=6, K1=6), -2),      # K not a multiple of 4
    (dict(K1=6, K=8), -2),      # split point not a multiple of 4
    (dict(ld1=3), -2),          # row stride
    (dict(ldy=2), -2),          # ldy < N
    (dict(K=0), -1),
    (dict(N=0), -1),
    (dict(K1=12, K=8), -1),     # K1 > K
])
def test_hyper_linear_rejects_before_launch(L, kw, code):
    a = dict(rows=32, K=8, N=4, ld1=8, K1=8, ld2=0, ldy=4)
    a.update(kw)
    x2 = _fk(1) if a["K1"] < a["K"] else None
    rc = L.dadmm_hyper_linear(a["rows"], a["K"], a["N"], _fk(0), a["ld1"], a["K1"], x2, a["ld2"],
                              _fk(2), _fk(3), _fk(4), a["ldy"], None)
    assert rc == code, L.dadmm_last_error()


def test_hyper_null_and_misaligned(L):
    assert L.dadmm_hyper_linear(8, 8, 4, None, 8, 8, None, 0, _fk(2), None, _fk(4), 4, None) == -1
    assert L.dadmm_hyper_linear(8, 8, 4, ctypes.c_void_p(0x10004), 8, 8, None, 0, _fk(2), None,
                                _fk(4), 4, None) == -1
    # split input without its second pointer
    assert L.dadmm_hyper_linear(8, 8, 4, _fk(0), 4, 4, None, 4, _fk(2), None, _fk(4), 4, None) == -1
    # GCN: P outside 1..160 (the row tile holds whole samples), missing BatchNorm statistics
    args = lambda P, bn: (4, P, 8, 4, _fk(0), 8, 8, None, 0, _fk(1), _fk(2), _fk(3), 1, bn,
                          _fk(5), _fk(6), _fk(7), 1e-5, 0.01, _fk(8), 4, None)
    assert L.dadmm_hyper_gcn(*args(161, _fk(4))) == -1
    assert L.dadmm_hyper_gcn(*args(5, None)) == -1
    assert L.dadmm_hyper_head(8, 8, 0, _fk(0), 8, _fk(1), _fk(2), 0.1, 0.99, 0.99, 0.99, _fk(3),
                              None) == -1
    assert L.dadmm_hyper_rownorm(8, 2052, _fk(0), _fk(1), _fk(2), 1e-5, 0, 0.0, _fk(3), None) == -2
    assert L.dadmm_hyper_rownorm(8, 6, _fk(0), _fk(1), _fk(2), 1e-5, 0, 0.0, _fk(3), None) == -2
    assert L.dadmm_hyper_rownorm(8, 8, _fk(0), None, _fk(2), 1e-5, 0, 0.0, _fk(3), None) == -1


def test_hyper_empty_batch_is_ok(L):
    assert L.dadmm_hyper_linear(0, 8, 4, _fk(0), 8, 8, None, 0, _fk(2), None, _fk(4), 4, None) == 0
    assert L.dadmm_hyper_rownorm(0, 8, _fk(0), _fk(1), _fk(2), 1e-5, 1, 0.01, _fk(3), None) == 0


def test_hyper_linear_ln_validation(L):
    assert L.dadmm_hyper_linear_ln_scratch_bytes(1024, 2000, 400) >= 4 * 1024 * 400
    assert L.dadmm_hyper_linear_ln_scratch_bytes(0, 8, 4) == 0
    args = lambda N, scratch: (32, 8, N, _fk(0), 8, _fk(1), _fk(2), _fk(3), _fk(4), 1e-5, 1, 0.01,
                               _fk(5), scratch, None)
    assert L.dadmm_hyper_linear_ln(*args(6, _fk(6))) == -2          # LayerNorm width % 4
    assert L.dadmm_hyper_linear_ln(*args(4, None)) == -1            # no scratch
    # a split input whose split point is not a multiple of 16
    assert L.dadmm_hyper_linear(8, 16, 4, _fk(0), 8, 8, _fk(1), 8, _fk(2), None, _fk(4), 4, None) == -2


def test_hyper_train_wgrad_rejects_bad_strides(L):
    """dadmm_hyper_train_wgrad validates its iteration strides before launching (a
    short or negative stride would make the batched kernels read outside the caller's buffers)."""
    from dadmm_hip import _lib
    net = _lib.HyperNet()
    net.P, net.n, net.ld, net.H = 5, 16, 16, 5
    for i in range(5):
        net.width[i] = 8
        net.conv_w[i] = net.conv_b[i] = net.bn_w[i] = net.bn_b[i] = 0x10000
    for jj in range(3):
        net.dec_width[jj] = 8
        net.dec_w[jj] = net.dec_b[jj] = net.ln_w[jj] = net.ln_b[jj] = 0x10000
    net.norm_w = net.norm_b = net.fc_w = net.fc_b = 0x10000
    B, iters = 4, 3
    dfl = L.dadmm_hyper_train_dsave_floats(ctypes.byref(net), B)
    assert dfl > 0
    sv, g = _lib.HyperSaved(), _lib.HyperGrads()
    atay = B * net.P * net.ld

    def call(a_s, s_s, d_s):
        return L.dadmm_hyper_train_wgrad(ctypes.byref(net), B, iters, _fk(0), a_s, _fk(1),
                                         ctypes.byref(sv), s_s, _fk(2), d_s, ctypes.byref(g), None, None)
    assert call(-1, 100, dfl) == -1                  # negative
    assert call(atay, -5, dfl) == -1
    assert call(atay, 100, -16) == -1
    assert call(atay - 1, 100, dfl) == -1            # shorter than one AtAy block
    assert call(atay, 0, dfl) == -1                  # every iteration on the same saved block
    assert call(atay, 100, dfl - 4) == -1            # shorter than one dsave block


def test_bn_running_update_validation(L):
    """dadmm_hyper_bn_running_update checks its layer table before launching; empty work is ok."""
    W = (ctypes.c_int32 * 2)(32, 48)
    vp = ctypes.c_void_p * 2
    ptrs = lambda o: vp(*[0x10000 + 256 * (o + i) for i in range(2)])   # noqa: E731
    assert L.dadmm_hyper_bn_running_scratch_bytes(2, W, 1, 32) == 8 * 2 * 80 * 1        # one split
    assert L.dadmm_hyper_bn_running_scratch_bytes(2, W, 25, 256) == 8 * 2 * 80 * 100    # 64 rows each
    assert L.dadmm_hyper_bn_running_scratch_bytes(2, W, 25, 4096) == 8 * 2 * 80 * 256   # capped
    assert L.dadmm_hyper_bn_running_scratch_bytes(9, W, 1, 1) == 0

    def call(layers=2, widths=W, block=32 * 256 + 48 * 256, iters=25, B=256, P=5, scratch=_fk(9), rm=None):
        return L.dadmm_hyper_bn_running_update(layers, widths, rm or ptrs(0), ptrs(2), None, ptrs(4), ptrs(6),
                                               block, iters, B, P, _fk(8), 0.5, scratch, None)
    assert call(layers=0) == -1
    assert call(P=1) == -1                                   # unbiased variance needs P >= 2
    assert call(scratch=None) == -1
    assert call(block=48 * 256 - 1) == -1                    # an iteration block shorter than [B][width]
    assert call(rm=vp(0x10000, 0)) == -1                     # a NULL running_mean
    assert call(widths=(ctypes.c_int32 * 2)(32, 0)) == -1
    assert call(B=0) == 0 and call(iters=0) == 0
