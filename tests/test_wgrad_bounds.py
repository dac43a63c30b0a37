"""Host-side bounds check of wgrad2_kernel's load addresses (csrc/dadmm_hyper_grad.hip): a numpy
restatement of the kernel's tile / split / wave / row-cursor index arithmetic (both the fast form,
K1 % 32 == 0 with a wave-uniform row cursor, and the generic form) over every load each wave issues,
including the ring's prologue and the clamped tail loads, asserting that each lands inside its
operand. Shapes: the GPU tests' and the training step's, plain and deferred (nb blocks of rows).
(Round 4: a group of X columns past K in the fast form once took the second segment's pointer and
read 4 bytes before it — a fault the GPU run showed as a hang; this test catches that form.)"""
import numpy as np
import pytest

W2_T, WAVES, RING = 64, 4, 8
# the kernel's wave-uniform cursor form (scalar row bases) was measured slower (3.43 vs 3.21 ms at
# 512000 x 400 x 400, profiles/r04/variants_r04z_wgrad2.txt) and removed; the kernel runs the
# per-lane cursor form (UNIFORM_FORM False); the uniform form's index arithmetic is kept for the
# regression check at the end
UNIFORM_FORM = False


def _splits(R, N, K):
    """wgrad_splits: powers of two; (DADMM_W2_SHORT) a short walk on a small grid split to >= 16
    row pairs per wave within 768 workgroups; (DADMM_W2_FILL) a grid past 768 refilled to 768,
    >= 32 row pairs per wave."""
    tiles = ((N + W2_T - 1) // W2_T) * ((K + W2_T - 1) // W2_T)
    steps, s, short = (R + 1) // 2, 1, False
    while tiles * s * 2 <= 1024 and s < 64:
        if steps // (WAVES * s * 2) < 64:
            short = True
            break
        s *= 2
    if short and tiles * s <= 128:   # DADMM_W2_SHORT: >= 16 row pairs per wave, one round
        f = min(768 // tiles, steps // (WAVES * 16))
        if f > s:
            return f
    if tiles * s > 768:
        return max(1, min(768 // tiles, steps // (WAVES * 32)))
    return s


def _bad_loads(R, N, K, K1, ldz, ld1, ld2, nb=1, zs=0, s1=0, s2=0):
    splits = _splits(R * nb, N, K)
    ext_z = (nb - 1) * zs + (R - 1) * ldz + N
    ext_1 = (nb - 1) * s1 + (R - 1) * ld1 + min(K1, K)
    ext_2 = (nb - 1) * s2 + (R - 1) * ld2 + (K - K1) if K1 < K else 0
    gn, gk = (N + W2_T - 1) // W2_T, (K + W2_T - 1) // W2_T
    spb = R // 2
    steps = spb * nb
    per = (steps + splits - 1) // splits
    lane = np.arange(64)
    i, kh = lane & 31, lane >> 5
    bad = 0
    for tl in range(gn * gk * splits):
        kt, nt, split = tl % gk, (tl // gk) % gn, tl // (gk * gn)
        n0, k0 = nt * W2_T, kt * W2_T
        sb = split * per
        se = min(sb + per, steps)
        uni = UNIFORM_FORM and (K1 >= K or K1 % 32 == 0) and spb >= WAVES
        for w in range(WAVES):
            first = sb + w
            if first < se:
                nsteps = (se - first + WAVES - 1) // WAVES
                lst = np.minimum(first + WAVES * np.arange(nsteps + RING), first + WAVES * (nsteps - 1))
                bb = lst // spb
                row = 2 * (lst - bb * spb)[:, None] + kh[None, :]
                bb = bb[:, None]
                for b in range(2):
                    nc = np.minimum(n0 + 32 * b + i, N - 1)
                    k = np.minimum(k0 + 32 * b + i, K - 1)
                    ez = bb * zs + row * ldz + nc[None, :]
                    bad += int(((ez < 0) | (ez >= ext_z)).sum())
                    if uni:   # the group's segment from its first (clamped) column
                        seg1 = min(k0 + 32 * b, K - 1) < K1
                        ex = bb * (s1 if seg1 else s2) + row * (ld1 if seg1 else ld2) + (k if seg1 else k - K1)
                        e = ext_1 if seg1 else ext_2
                        bad += int(((ex < 0) | (ex >= e)).sum())
                    else:     # per-lane segment
                        m1 = k < K1
                        ex1 = (bb * s1 + row * ld1 + k[None, :])[:, m1]
                        ex2 = (bb * s2 + row * ld2 + (k - K1)[None, :])[:, ~m1]
                        bad += int(((ex1 < 0) | (ex1 >= ext_1)).sum() + ((ex2 < 0) | (ex2 >= ext_2)).sum())
        if R & 1 and split == 0:   # odd rows: each block's last row
            for bb in range(nb):
                for b in range(2):
                    nc = np.minimum(n0 + 32 * b + i, N - 1)
                    k = np.minimum(k0 + 32 * b + i, K - 1)
                    ez = bb * zs + (R - 1) * ldz + nc
                    ex = np.where(k < K1, bb * s1 + (R - 1) * ld1 + k, bb * s2 + (R - 1) * ld2 + k - K1)
                    e = np.where(k < K1, ext_1, ext_2)
                    bad += int(((ez < 0) | (ez >= ext_z)).sum() + ((ex < 0) | (ex >= e)).sum())
    return bad


@pytest.mark.parametrize("R,N,K,K1,ld1,ld2", [(1280, 400, 400, 400, 408, 0), (1280, 100, 512, 256, 264, 260),
                                              (256, 400, 2000, 2000, 2008, 0), (256, 20, 100, 100, 108, 0),
                                              (37, 13, 70, 70, 78, 0), (45, 12, 96, 48, 52, 52),
                                              (60, 8, 64, 32, 36, 36), (300, 32, 160, 160, 160, 0)])
def test_wgrad2_loads_in_bounds(R, N, K, K1, ld1, ld2):
    assert _bad_loads(R, N, K, K1, N, ld1, ld2) == 0


@pytest.mark.parametrize("R,N,K,K1", [(256, 32, 160, 160), (51, 32, 160, 160), (255, 8, 64, 32), (1280, 8, 64, 32),
                                      (1280, 32, 32, 32), (4096, 20, 100, 100), (2560, 400, 400, 400),
                                      (2560, 100, 512, 256)])
def test_wgrad2_deferred_loads_in_bounds(R, N, K, K1):
    """Deferred form: nb = 4 blocks; X as two segments (Atb shared: stride 0) when K1 < K."""
    ld = K1 if K1 < K else K
    assert _bad_loads(R, N, K, K1, N, ld, ld, nb=4, zs=R * N + 96, s1=R * ld + 32, s2=0) == 0


def test_bounds_check_catches_segment_past_k():
    """The pre-fix form (segment from the unclamped group start) is flagged on the decoder shape."""
    import inspect
    code = inspect.getsource(_bad_loads).replace("min(k0 + 32 * b, K - 1) < K1", "(k0 + 32 * b) < K1")
    ns = {"np": np, "W2_T": W2_T, "WAVES": WAVES, "RING": RING, "_splits": _splits, "UNIFORM_FORM": True}
    exec(code, ns)
    assert ns["_bad_loads"](256, 32, 160, 160, 32, 160, 160, nb=4, zs=256 * 32 + 96, s1=256 * 160, s2=256 * 160) > 0


def _fast_cursor_ok(R, nb, splits, W=WAVES, ring=RING):
    """The fast form's cursor (csrc/dadmm_hyper_grad.hip, DADMM_W2_FAST): per-step deltas chosen
    by masks, the first (nsteps - 9) / 8 rings without the range test. Its load sequence must equal
    the reference cursor's: step min(first + 4 j, last step of the wave) for load j."""
    spb = R // 2
    steps = spb * nb
    per = (steps + splits - 1) // splits
    big = 1 << 40
    for split in range(splits):
        sb, se = split * per, min(split * per + per, steps)
        for w in range(W):
            first = sb + w
            if first >= se or spb < W:
                continue
            st = {"lst": first, "lloc": first % spb, "pos": (first // spb) * big + 2 * (first % spb)}
            seq = []

            def load(check):
                seq.append(st["pos"])
                wr = st["lloc"] + W >= spb
                if (st["lst"] + W < se) if check else True:
                    st["pos"] += 2 * W + ((big - 2 * spb) if wr else 0)
                    st["lst"] += W
                    st["lloc"] += W - (spb if wr else 0)
            nsteps = (se - first + W - 1) // W
            nfull = nsteps // ring
            nunc = min((nsteps - 9) // ring if nsteps >= 9 else 0, nfull)
            for _ in range(ring):
                load(True)
            for g in range(nfull):
                for _ in range(ring):
                    load(g >= nunc)
            for j, v in enumerate(seq):
                s_ = min(first + W * j, first + W * (nsteps - 1))
                if v != (s_ // spb) * big + 2 * (s_ % spb):
                    return False
    return True


@pytest.mark.parametrize("R,nb,splits", [(20480, 25, 16), (4096, 25, 64), (1280, 25, 16), (510, 4, 1),
                                         (1280, 1, 2), (20480, 25, 8), (300, 3, 4), (16, 3, 1), (74, 2, 3),
                                         (1280, 25, 15), (1280, 25, 27), (256, 25, 3), (256, 25, 25),
                                         (20480, 25, 15), (1280, 25, 96), (256, 25, 50), (256, 25, 27)])
def test_wgrad2_fast_cursor_sequence(R, nb, splits):
    assert _fast_cursor_ok(R, nb, splits)
