#!/usr/bin/env python3
"""Benchmark of the MI355X unfolded D-ADMM forward (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1..3] name the single-GPU shapes; the metric is quoted on
B=4096, P=5, n=256, K=25, m=64): one "step" = one DLASSO_unfolded.forward over a batch of 4096
synthetic problems resident in HBM: the reference's random inits (randn x 3), the hyper-parameter
table and the fused K-iteration HIP kernel. Unit of work = one ADMM iteration of one problem
(all P agents); value = B * K * steps * n_gpus / max-over-ranks wall time (weak scaling: every
rank runs its own 4096-problem batch; no collective inside the step).

Extra fields: "roofline" (dominant kernel: fused_forward_kernel, timed with HIP events on its
stream; FP32 MFMA roofline with SURVEY.md §8(d)'s algorithmic flop/unit P(4mn + 14n) + 2Pn deg,
plus the HBM view with its algorithmic bytes/unit 4P(4n+m) and the PMC-measured bytes;
"traffic" = PMC-measured HBM bytes per launch from profiles/traffic.json), "cpu_baseline" (ports of the reference forward — vectorised torch-CPU, the C
restatement and the loop-faithful eager replay — on all host threads and on 1 thread, bounded
samples; the fastest all-thread leg is the headline), "parity" (bit-exactness vs the order-matched fp32 oracle and
final-iterate MSE vs the fp64 restatement, on a slice of the batch; outside the timed region).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, dense
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E spec peak


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--min-warmup-s", type=float, default=0.5,
                    help="keep warming up (the same step, untimed) until this much wall time has passed: "
                         "the GPU's clocks ramp over the first ~50 forwards (0.567 vs 0.537 ms, "
                         "profiles/r05/clock_ramp_r05z.txt)")
    ap.add_argument("--batch", type=int, default=4096, help="problems per GPU")
    ap.add_argument("--P", type=int, default=5)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--K", type=int, default=25)
    ap.add_argument("--graph-prob", type=float, default=0.5)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=30.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the secondary measurements (training step, GNN model, P=16 path)")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (written from a rocprofv3 --pmc pass)")
    return ap.parse_args()


def make_args(K):
    return argparse.Namespace(GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99,
                              rho_max=0.99, eta_max=0.99, max_penalty_threshold=0.8,
                              penalty_reduction_factor=0.95)


def spawn_ranks(n, cmd=None, timeout=None):
    """Run ``n`` ranks of this benchmark as child processes (one per GPU, LOCAL_RANK = rank) with
    torchrun's environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free
    MASTER_PORT). The parent never touches the GPU. When a rank fails, the others are terminated.
    Returns the exit status to report: 0 when every rank succeeded."""
    import signal
    import socket
    import subprocess
    if cmd is None:
        cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    t0 = time.time()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = abs(bad[0]) or 1
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.time() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    return rc


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without torchrun: launch the N ranks here
        sys.exit(spawn_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        print(f"error: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    dist = None
    # ranks beyond the visible devices share them (a one-GPU rehearsal of the N-rank path; RCCL
    # refuses two ranks on one device, so such a run sets DADMM_DIST_BACKEND=gloo)
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    backend = os.environ.get("DADMM_DIST_BACKEND") or "nccl"
    if world > 1:
        import torch.distributed as dist
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    torch.cuda.set_device(dev)
    # collectives of this script on the backend's device (gloo reduces host tensors)
    cdev = dev if backend == "nccl" else torch.device("cpu")

    import oracle as O   # input generator (reference distribution) and checker only
    import unfolded_DLASSO
    from dadmm_hip import _lib

    P, n, m, K, B = a.P, a.n, a.m, a.K, a.batch
    # A is shared by every rank (one sensing operator per agent); each rank draws its own shard
    A, _, _ = O.make_problem(P, m, n, 1, seed=1234)
    gen = torch.Generator().manual_seed(4321 + rank)
    x = 2 * torch.randn(B, n, generator=gen) * (torch.rand(B, n, generator=gen) <= 0.25)
    b = torch.einsum("pmn,bn->bpm", torch.from_numpy(A), x)
    x = x.float()
    At = torch.from_numpy(A)[None].to(dev)
    bt = b[..., None].to(dev)
    G = O.er_graph(P, a.graph_prob, seed=7)
    graph_list = [G] * B
    model = unfolded_DLASSO.DLASSO_unfolded(At, make_args(K)).to(dev)
    param = np.load(os.path.join(ROOT, "tests", "golden",
                                 "fixture_25_iter_general_learning_seq_hyp_param.npy"))
    if param.shape == (K, P, 4):
        with torch.no_grad():
            model.seq_hyp.param.copy_(torch.from_numpy(param))
    model.eval()

    # --- kernel-level timing hook: HIP events around every fused launch, on its stream ------
    from dadmm_hip import ops
    ev_pairs = []
    orig_forward = _lib.load().dadmm_forward

    class _Timed:
        def __call__(self, *args):
            s = torch.cuda.current_stream(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            rc = orig_forward(*args)
            e1.record(s)
            ev_pairs.append((e0, e1))
            return rc

    timed = _Timed()

    statuses = []

    def step():
        with torch.no_grad():
            Y, _ = model(bt, graph_list)
        statuses.append(model.last_status)     # device word, no host sync here
        return Y

    # W warmup steps, then more of the same until min_warmup_s of wall time has passed (steady
    # clocks before the timed region; every rank warms up alike, the count is reported)
    tw = time.perf_counter()
    warm_steps = 0
    while warm_steps < a.warmup or (time.perf_counter() - tw < a.min_warmup_s and warm_steps < 100000):
        step()
        warm_steps += 1
        if warm_steps % 20 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    warm_s = time.perf_counter() - tw

    # patch the library entry point only for the timed region's event bookkeeping
    L = _lib.load()
    L.dadmm_forward = timed
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    L.dadmm_forward = orig_forward
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev_pairs]))
    # every timed forward must have run the work it claims: a fired guard (status != 0) means
    # the batch went through the reference's reset / recompute path instead
    head_status = _or_all(statuses)

    if dist is not None:
        t = torch.tensor([elapsed, float(head_status != 0)], device=cdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
        if t[1].item() != 0 and head_status == 0:
            head_status = -1          # another rank's forwards fired a guard
        # the reference's one collective: the epoch loss (a scalar all-reduce over RCCL)
        with torch.no_grad():
            Y, _ = model(bt, graph_list)
            lf = ((Y[-1, ..., 0] - x.to(dev)[:, None, :]) ** 2).mean()
        red = torch.stack([lf, torch.ones((), device=dev)]).to(cdev)
        dist.all_reduce(red)

    units_per_step = B * K
    value = units_per_step * a.steps * world / elapsed
    ms_per_step = 1e3 * elapsed / a.steps

    if rank == 0:
        # Roofline of the dominant kernel (fused_forward_kernel), SURVEY.md §8(d): HBM-bound
        # with ALGORITHMIC bytes/unit = 4 P (4n + m) (read y_k, U_k, b_p; write y_{k+1}, U_{k+1}
        # per sample-iteration, the operator amortised), units/launch = B K.
        bytes_unit = 4 * P * (4 * n + m)
        alg_bytes = bytes_unit * units_per_step
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        # MFMA view of the same launch (algorithmic flops/unit)
        deg_avg = float(sum(d for _, d in G.degree())) / P
        flop_unit = P * (4 * m * n + 14 * n) + 2 * P * n * deg_avg
        tflops = flop_unit * units_per_step / (kern_ms * 1e-3) / 1e12
        # bytes the fused launch cannot avoid: inputs once, every iterate once (state on-chip)
        min_bytes = 4 * (K * B * P * n + 3 * B * P * n + B * P * m) + 2 * 4 * P * 64 * n
        traffic = None
        if os.path.exists(a.traffic_file):
            try:
                tr = json.load(open(a.traffic_file))
                key = f"B{B}_P{P}_n{n}_m{m}_K{K}"
                traffic = tr.get(key, {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None

        parity = check_parity(O, model, A, b, G, dev, P, n, m, K)
        # the CPU baseline and the single-GPU secondary measurements belong to the N = 1 run
        cpu = None
        if not (a.no_cpu_baseline or world > 1):
            cpu = cpu_baseline(O, A, b, G, model, P, n, m, K, a.cpu_baseline_seconds)
            # BASELINE configs[0], the reference's own CPU-runnable case ("run
            # at c1 and at H"): P=5, n=200, m_p=50, batch=32, K=15
            cpu["configs0"] = cpu_baseline_configs0(O, a.cpu_baseline_seconds / 3)
        status = {"headline_forward": head_status}
        extras = None if (a.no_extras or world > 1) else secondary(O, dev, A, b, x, G, model, P, n,
                                                                   m, K, B, status)
        out = {
            "metric": "ADMM-iters/sec (node), batch=4096 P=5 n=256 K=25; final-iter MSE vs ref",
            "value": value,
            "unit": "ADMM-iters/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_steps_run": warm_steps,
            "warmup_s": round(warm_s, 3),
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference distribution: A_p = U clamp(S,0.1,10) V^T, "
                    "x* = 2 N(0,1) Bernoulli(0.25), b_p = A_p x*; trained seq_hyp fixture)",
            "config": {"workload": f"DLASSO_unfolded.forward B={B}/GPU P={P} n={n} m={m} K={K} "
                                   f"ER(p={a.graph_prob}) shared graph",
                       "global_batch": B * world, "P": P, "n": n, "m": m, "K": K,
                       "parallelism": f"batch-sharded dp{world}"},
            "agent_iters_per_s": value * P,
            "kernel_ms": kern_ms,
            # the binding resource of the fused kernel is the FP32 matrix pipe (state stays on
            # chip; only Y streams to HBM), so the roofline is MFMA; the HBM view is kept beside it
            "roofline": {"bound": "mfma", "achieved": tflops, "peak": PEAK_FP32_TFLOPS,
                         "unit": "TFLOP/s", "frac": tflops / PEAK_FP32_TFLOPS, "traffic": traffic,
                         "kernel": "fused_forward_kernel", "kernel_ms": kern_ms,
                         "flop_per_unit": flop_unit, "units_per_launch": units_per_step,
                         "hbm_view": {"bytes_per_unit": bytes_unit, "achieved_alg_GBs": achieved,
                                      "frac_alg": achieved / PEAK_HBM_GBS,
                                      "counter_GBs": (traffic / (kern_ms * 1e-3) / 1e9
                                                      if traffic else None),
                                      "min_hbm_bytes_per_launch": min_bytes,
                                      "peak_GBs": PEAK_HBM_GBS}},
            "cpu_baseline": cpu,
            "parity": parity,
            "extras": extras,
            # guard status word of every timed workload (0: the measured work is the work claimed)
            "status": status,
        }
        print(json.dumps(out))
        bad = {k: v for k, v in status.items() if v != 0}
        if bad:
            print(f"error: guard status set on timed workloads {bad}: numbers not valid",
                  file=sys.stderr)
            if dist is not None:
                dist.destroy_process_group()
            sys.exit(3)
    if dist is not None:
        dist.destroy_process_group()


def _or_all(statuses) -> int:
    """Bitwise OR of device status words (one host sync)."""
    if not statuses:
        return 0
    v = torch.cat([t.reshape(-1).to(torch.int64) for t in statuses])
    out = 0
    for w in v.cpu().tolist():
        out |= int(w)
    return out


def _event_ms(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def secondary(O, dev, A, b, x, G, model, P, n, m, K, B, status):
    """Secondary measurements on the same box, outside the timed region (not the headline):
    the training step at the headline shape (recording forward + adjoint kernel, and the module's
    forward + compute_loss + loss.backward()), the GNN-hypernetwork model's forward and training
    step (DLASSO_GNNHyp3_Progressive, h = 100) at B = 1024 / 256 and at the headline batch
    B = 4096, configs[4]'s per-GPU shard of the GNN model, and BASELINE configs[2]'s P=16, n=512
    shape (streamed forward, recording forward, general adjoint). ``status`` collects every timed
    workload's guard status word (bench exits non-zero if any is set)."""
    out = {}

    def st(name, word):
        status[name] = _or_all([word]) if torch.is_tensor(word) else int(word)

    try:
        # BASELINE configs[1]: the same module and operator at B = 1024 (P=5, n=256, m=64, K=25,
        # the trained table): whole module forwards per step like the headline, and the fused
        # launch alone by HIP events on its stream
        from dadmm_hip import _lib as _L1
        B1 = 1024
        b1 = b[:B1, ..., None].to(dev)
        G1 = [G] * B1
        L1 = _L1.load()
        # the launch this batch takes (the column-split forward at B = 1024 on 256 CUs)
        from dadmm_hip.ops import split_cols as _split_cols
        split1 = _split_cols(model.operator(), B1, K)
        entry1 = "dadmm_forward_split" if split1 else "dadmm_forward"
        orig1 = getattr(L1, entry1)
        ev1 = []

        def timed1(*args):
            s_ = torch.cuda.current_stream(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s_)
            rc = orig1(*args)
            e1.record(s_)
            ev1.append((e0, e1))
            return rc

        def f1():
            with torch.no_grad():
                model(b1, G1)
        # the headline's warm-up floor (steady clocks: the secondary legs run after seconds of
        # CPU-only work), then 200 forwards (~40 ms) timed
        tw1 = time.perf_counter()
        while time.perf_counter() - tw1 < 0.5:
            for _ in range(20):
                f1()
            torch.cuda.synchronize()
        ms1 = _event_ms(f1, 200, warm=5)
        st("configs1_forward", model.last_status)
        setattr(L1, entry1, timed1)
        try:
            for _ in range(20):
                f1()
            torch.cuda.synchronize()
        finally:
            setattr(L1, entry1, orig1)
        k1 = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev1]))
        deg1 = float(sum(d for _, d in G.degree())) / P
        fl1 = P * (4 * m * n + 14 * n) + 2 * P * n * deg1
        out["configs1_forward"] = {
            "B": B1, "P": P, "n": n, "m": m, "K": K, "ms": ms1, "kernel_ms": k1,
            "kernel": "split_forward_kernel (dadmm_forward_split, 64-column slices)" if split1
                      else "fused_forward_kernel",
            "units_per_s": B1 * K / (ms1 * 1e-3),
            "kernel_mfma_frac": fl1 * B1 * K / (k1 * 1e-3) / 1e12 / PEAK_FP32_TFLOPS,
            "kernel_hbm_alg_frac": 4 * P * (4 * n + m) * B1 * K / (k1 * 1e-3) / 1e9 / PEAK_HBM_GBS,
            "note": "BASELINE configs[1]: DLASSO_unfolded.forward per step (draws, the forward "
                    "launch, gated stepwise), same A / graph / trained table as the headline; "
                    "kernel_ms: HIP events around the forward launch on its stream"}
        del b1, G1
    except Exception as e:
        out["configs1_error"] = repr(e)[:300]
    try:
        import gnn_dlasso_utils
        from dadmm_hip.ops import backward_raw, forward_raw
        bt = b[..., None].to(dev)
        label = x.to(dev)[..., None]
        op = model.operator()
        from dadmm_hip.graph import ingest
        g = ingest([G] * B, P, B, dev)
        table = model.hyp_table(K).detach()
        bb = b.to(dev)
        out["train_forward_record_ms"] = _event_ms(
            lambda: forward_raw(op, bb, g, table, record=True), 10)
        _, _, s_rec, tr = forward_raw(op, bb, g, table, record=True)
        st("train_forward_record", s_rec)
        gY = torch.randn(K, B, P, n, device=dev)
        out["adjoint_ms"] = _event_ms(lambda: backward_raw(op, g, tr, gY), 10)
        model.train()

        def step():
            Y, _ = model(bt, [G] * B)
            _, lf = gnn_dlasso_utils.compute_loss(Y, label)
            model.zero_grad()
            lf.backward()
        out["module_train_step_ms"] = _event_ms(step, 5)
        st("module_train_step", model.last_status)
        out["train_units_per_s"] = B * K / (out["module_train_step_ms"] * 1e-3)
        model.eval()
    except Exception as e:  # secondary numbers never break the headline line
        out["train_error"] = repr(e)[:300]
    try:
        import argparse as _ap

        import gnn_dlasso_models_progressive as GM
        import gnn_dlasso_utils
        args = _ap.Namespace(GHN_iter_num=K, GHyp_hidden=100, DADMM_mode="diff", alpha_max=0.1,
                             tau_max=0.99, rho_max=0.99, eta_max=0.99)
        gnn = GM.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A)[None].to(dev), args).to(dev).eval()
        from dadmm_hip.graph import ingest as _ing
        graphs = [O.connected_er_graph(P, 0.5, seed=100 + s) for s in range(B)]
        t0 = time.perf_counter()
        gball = _ing(graphs, P, B, dev)     # ingested once; both models accept the GraphBatch
        torch.cuda.synchronize()
        ingest_ms = 1e3 * (time.perf_counter() - t0)
        for Bg in (1024, B):
            bg = b[:Bg, ..., None].to(dev)
            gbg = gball if Bg == B else _ing(graphs[:Bg], P, Bg, dev)

            def gfwd():
                with torch.no_grad():
                    gnn(bg, gbg)
            ms = _event_ms(gfwd, 3, warm=1)
            st(f"gnn_forward_B{Bg}", gnn.last_status)
            rec = {"B": Bg, "P": P, "n": n, "m": m, "K": K, "hidden": 100, "ms": ms,
                   "units_per_s": Bg * K / (ms * 1e-3), "hypernetwork": "fused HIP (dadmm_hyper_*)",
                   "note": "graphs pre-ingested (GraphBatch); host ingestion timed separately"}
            if Bg == 1024:
                gnn.hyper_backend = "torch"
                rec["ms_torch_hypernetwork"] = _event_ms(gfwd, 2, warm=1)
                gnn.hyper_backend = "auto"
                out["gnn_forward"] = rec
            else:
                rec["graph_ingest_ms"] = ingest_ms
                out["gnn_forward_headline_batch"] = rec
            del bg
        # training step of the GNN model (model.train(): dropout, batch statistics, autograd):
        # forward + compute_loss + backward, HIP training hypernetwork (vs the torch composition
        # at B = 256)
        for Bt in (256, B):
            bgt = b[:Bt, ..., None].to(dev)
            lab = x[:Bt].to(dev)[..., None]
            gbt = gball if Bt == B else _ing(graphs[:Bt], P, Bt, dev)
            gnn.train()

            def gstep():
                Y, _ = gnn(bgt, gbt)
                _, lf = gnn_dlasso_utils.compute_loss(Y, lab)
                gnn.zero_grad()
                lf.backward()
            ms_tr = _event_ms(gstep, 3, warm=1)
            st(f"gnn_train_step_B{Bt}", gnn.last_status)
            rec = {"B": Bt, "K": K, "ms": ms_tr, "units_per_s": Bt * K / (ms_tr * 1e-3),
                   "hypernetwork": "HIP training kernels (GnnTrainFn)"}
            if Bt == 256:
                gnn.hyper_backend = "torch"
                rec["ms_torch_hypernetwork"] = _event_ms(gstep, 2, warm=1)
                gnn.hyper_backend = "auto"
                out["gnn_train_step"] = rec
            else:
                out["gnn_train_step_headline_batch"] = rec
            gnn.eval()
        del gnn, gball
    except Exception as e:
        out["gnn_error"] = repr(e)[:300]
    try:
        # BASELINE configs[4]'s per-GPU shard of the GNN model: P=50, n=1024, m=32, K=50,
        # B=8192/8 per GPU, graph_prob 0.5, h=100 (eval forward, fused hypernetwork)
        import argparse as _ap

        import gnn_dlasso_models_progressive as GM
        P5, n5, m5, B5, K5 = 50, 1024, 32, 1024, 50
        A5, b5, _ = O.make_problem(P5, m5, n5, B5, seed=55)
        args5 = _ap.Namespace(GHN_iter_num=K5, GHyp_hidden=100, DADMM_mode="diff", alpha_max=0.1,
                              tau_max=0.99, rho_max=0.99, eta_max=0.99)
        g5 = GM.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A5)[None].to(dev), args5).to(dev).eval()
        graphs5 = [O.connected_er_graph(P5, 0.5, seed=500 + s) for s in range(B5)]
        b5t = torch.from_numpy(b5)[..., None].to(dev)
        from dadmm_hip.graph import generate_er as _gen5
        from dadmm_hip.graph import ingest as _ing5
        t0 = time.perf_counter()
        gb5 = _ing5(graphs5, P5, B5, dev)
        torch.cuda.synchronize()
        ingest5_ms = 1e3 * (time.perf_counter() - t0)
        # the same graph model generated on the device (gnn_dlasso_progressive.py:181-191)
        _gen5(B5, P5, 0.5, 1, dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(5):
            _gen5(B5, P5, 0.5, 2 + i, dev)
        torch.cuda.synchronize()
        gen5_ms = 1e3 * (time.perf_counter() - t0) / 5

        def g5fwd():
            with torch.no_grad():
                g5(b5t, gb5)          # graphs ingested once (the tensor fast path)
        ms5 = _event_ms(g5fwd, 1, warm=1)
        st("c5_gnn_forward", g5.last_status)
        out["c5_gnn_forward"] = {"B": B5, "P": P5, "n": n5, "m": m5, "K": K5, "hidden": 100,
                                 "graph_prob": 0.5, "ms": ms5,
                                 "units_per_s": B5 * K5 / (ms5 * 1e-3),
                                 "graph_ingest_ms": ingest5_ms,
                                 "graph_generate_device_ms": gen5_ms,
                                 "note": "per-GPU shard of configs[4] (8192 / 8); forward with "
                                         "pre-ingested graphs; host networkx ingestion and "
                                         "on-device generation (dadmm_graph_generate, incl. "
                                         "one host sync) timed separately"}
        del g5, b5t
    except Exception as e:
        out["c5_error"] = repr(e)[:300]
    try:
        # BASELINE configs[3] and configs[4] at their GLOBAL batches on this one GPU (the 8-GPU
        # runs shard them 8 ways): configs[3] = the headline shape at B = 32768 (fused forward,
        # Y = 4.2 GB); configs[4] = the GNN model at P=50, n=1024, m=32, K=50, B=8192 (Y = 84 GB),
        # graphs generated on the device (dadmm_graph_generate)
        import argparse as _ap

        import gnn_dlasso_models_progressive as GM
        import unfolded_DLASSO
        from dadmm_hip.graph import generate_er as _gen
        B4 = 32768
        A4, b4, _ = O.make_problem(P, m, n, B4, seed=4444)
        m4 = unfolded_DLASSO.DLASSO_unfolded(torch.from_numpy(A4)[None].to(dev), make_args(K)).to(dev).eval()
        b4t = torch.from_numpy(b4)[..., None].to(dev)
        G4 = [G] * B4

        def f4():
            with torch.no_grad():
                m4(b4t, G4)
        ms4 = _event_ms(f4, 5, warm=2)
        st("c4_global_forward", m4.last_status)
        out["c4_global_forward"] = {"B": B4, "P": P, "n": n, "m": m, "K": K, "ms": ms4,
                                    "units_per_s": B4 * K / (ms4 * 1e-3),
                                    "note": "BASELINE configs[3]'s whole 8-GPU batch on one GPU"}
        del m4, b4t, G4
        P5, n5, m5, B5, K5 = 50, 1024, 32, 8192, 50
        A5, b5, _ = O.make_problem(P5, m5, n5, B5, seed=5555)
        args5 = _ap.Namespace(GHN_iter_num=K5, GHyp_hidden=100, DADMM_mode="diff", alpha_max=0.1,
                              tau_max=0.99, rho_max=0.99, eta_max=0.99)
        g5 = GM.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A5)[None].to(dev), args5).to(dev).eval()
        gb5 = _gen(B5, P5, 0.5, 7, dev)
        b5t = torch.from_numpy(b5)[..., None].to(dev)

        def f5():
            with torch.no_grad():
                g5(b5t, gb5)
        ms5 = _event_ms(f5, 1, warm=1)
        st("c5_global_forward", g5.last_status)
        out["c5_global_forward"] = {"B": B5, "P": P5, "n": n5, "m": m5, "K": K5, "hidden": 100,
                                    "ms": ms5, "units_per_s": B5 * K5 / (ms5 * 1e-3),
                                    "note": "BASELINE configs[4]'s whole 8-GPU batch on one GPU "
                                            "(graphed eval forward, device-generated graphs)"}
        del g5, b5t, gb5
        torch.cuda.empty_cache()
    except Exception as e:
        out["global_error"] = repr(e)[:300]
    try:
        import unfolded_DLASSO
        from dadmm_hip.ops import backward_raw as _br
        P3, n3, m3, B3, K3 = 16, 512, 64, 4096, 25
        A3, b3, _ = O.make_problem(P3, m3, n3, B3, seed=77)
        mod = unfolded_DLASSO.DLASSO_unfolded(torch.from_numpy(A3)[None].to(dev),
                                              argparse.Namespace(**{**vars(model.args), "GHN_iter_num": K3}))
        mod = mod.to(dev).eval()
        graphs3 = [O.connected_er_graph(P3, 0.3, seed=s) for s in range(B3)]
        b3t = torch.from_numpy(b3)[..., None].to(dev)

        from dadmm_hip.graph import ingest as _ing
        from dadmm_hip.ops import forward_raw as _fr
        t0 = time.perf_counter()
        g3 = _ing(graphs3, P3, B3, dev)
        torch.cuda.synchronize()
        ingest_ms = 1e3 * (time.perf_counter() - t0)
        op3, tab3, b3d = mod.operator(), mod.hyp_table(K3).detach(), b3t[..., 0].contiguous()
        ms = _event_ms(lambda: _fr(op3, b3d, g3, tab3), 5, warm=1)
        st("c3_forward", _fr(op3, b3d, g3, tab3)[2])
        # the training forward (trajectory recording for the adjoint): streamed vs stepwise
        ms_rec = _event_ms(lambda: _fr(op3, b3d, g3, tab3, record=True), 3, warm=1)
        ms_rec_sw = _event_ms(lambda: _fr(op3, b3d, g3, tab3, record=True, path="stepwise"), 3, warm=1)
        _, _, s3r, tr3 = _fr(op3, b3d, g3, tab3, record=True)
        st("c3_record_forward", s3r)
        gY3 = torch.randn(K3, B3, P3, n3, device=dev)
        ms_adj = _event_ms(lambda: _br(op3, g3, tr3, gY3), 3, warm=1)
        del tr3, gY3

        def f3():
            with torch.no_grad():
                mod(b3t, graphs3)
        ms_module = _event_ms(f3, 2, warm=1)
        st("c3_module_forward", mod.last_status)
        out["c3_tiled"] = {"B": B3, "P": P3, "n": n3, "m": m3, "K": K3, "graph_prob": 0.3,
                           "path": "streamed single launch (dadmm_stream.hip) + gated stepwise",
                           "ms_per_forward": ms,
                           "units_per_s": B3 * K3 / (ms * 1e-3),
                           "alg_bytes_per_unit": 4 * P3 * (4 * n3 + m3),
                           "alg_GBs": 4 * P3 * (4 * n3 + m3) * B3 * K3 / (ms * 1e-3) / 1e9,
                           "graph_ingest_ms": ingest_ms,
                           "module_forward_ms_incl_ingest": ms_module,
                           "record_forward_ms": ms_rec, "record_forward_stepwise_ms": ms_rec_sw,
                           "adjoint_ms": ms_adj}
    except Exception as e:
        out["c3_error"] = repr(e)[:300]
    return out


def check_parity(O, model, A, b, G, dev, P, n, m, K, Bs=32):
    """Bit-exactness vs the order-matched fp32 oracle and final-iterate MSE vs fp64 on the
    first Bs problems of the batch (same A, b, graph, inits, hyper-parameters)."""
    rng = np.random.default_rng(99)
    y0, U0, d0 = (1e-2 * rng.standard_normal((3, Bs, P, n))).astype(np.float32)
    bs = b[:Bs].numpy()
    with torch.no_grad():
        Y, _ = model(torch.from_numpy(bs).to(dev)[..., None], [G] * Bs,
                     inits=tuple(torch.from_numpy(v).to(dev) for v in (y0, U0, d0)))
        table = model.hyp_table(K).cpu().numpy()
    Y = Y[..., 0].cpu().numpy()
    Y32, _, _ = O.forward_f32(A, bs, [G] * Bs, table, y0, U0, d0)
    Y64, _, _ = O.forward_f64(A, bs, [G] * Bs, table, y0, U0, d0)
    # north_star's "final-iterate MSE <= 1e-5 vs the CPU reference": the reference's own op
    # sequence replayed in fp32 on the CPU (oracle.ref_torch: Gram form, per-agent GEMVs, the
    # Python compute_delta loop), also at BASELINE configs[0]
    from oracle import ref_torch
    Yr = ref_torch.forward(A, bs, [G] * Bs, table, y0, U0, d0)
    mse = lambda a, c: float(((a[-1] - c[-1]) ** 2).mean())   # noqa: E731
    return {"samples": Bs, "bit_exact_vs_fp32_oracle": bool(np.array_equal(Y, Y32)),
            "max_abs_diff_vs_fp32_oracle": float(np.abs(Y - Y32).max()),
            "final_iter_mse_vs_fp64": mse(Y, Y64),
            "final_iter_mse_vs_reference_form_fp32": mse(Y, Yr),
            "reference_form_fp32_mse_vs_fp64": mse(Yr, Y64),
            "tolerance": 1e-5,
            "configs0": parity_configs0(O, dev)}


def parity_configs0(O, dev):
    """BASELINE configs[0] (P=5, n=200, m=50, B=32, K=15, shared ER(0.5) graph, the reference's
    default hyper-parameter init param = 0): the drop-in module on the GPU vs the reference-form
    fp32 CPU replay (oracle.ref_torch) and the fp64 restatement, final-iterate MSE."""
    import argparse as _ap

    import unfolded_DLASSO
    from oracle import ref_torch
    P, n, m, B, K = 5, 200, 50, 32, 15
    A, b, _ = O.make_problem(P, m, n, B, seed=1200)
    G = O.er_graph(P, 0.5, seed=7)
    rng = np.random.default_rng(99)
    y0, U0, d0 = (1e-2 * rng.standard_normal((3, B, P, n))).astype(np.float32)
    mod = unfolded_DLASSO.DLASSO_unfolded(torch.from_numpy(A)[None].to(dev), _ap.Namespace(
        GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99, rho_max=0.99,
        eta_max=0.99, max_penalty_threshold=0.8, penalty_reduction_factor=0.95)).to(dev).eval()
    with torch.no_grad():
        Y, _ = mod(torch.from_numpy(b).to(dev)[..., None], [G] * B,
                   inits=tuple(torch.from_numpy(v).to(dev) for v in (y0, U0, d0)))
        table = mod.hyp_table(K).cpu().numpy()
    Y = Y[..., 0].cpu().numpy()
    Yr = ref_torch.forward(A, b, [G] * B, table, y0, U0, d0)
    Y64, _, _ = O.forward_f64(A, b, [G] * B, table, y0, U0, d0)
    mse = lambda a, c: float(((a[-1] - c[-1]) ** 2).mean())   # noqa: E731
    return {"P": P, "n": n, "m": m, "B": B, "K": K,
            "final_iter_mse_vs_reference_form_fp32": mse(Y, Yr), "final_iter_mse_vs_fp64": mse(Y, Y64)}


def _host_cpus():
    """(threads this process may run on, CPU model, cgroup CPU quota or None)."""
    try:
        threads = len(os.sched_getaffinity(0))
    except AttributeError:
        threads = os.cpu_count() or 1
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    return threads, model, quota


def cpu_baseline_configs0(O, seconds):
    """The CPU legs at BASELINE configs[0] (P=5, n=200, m=50, B=32, K=15, one shared ER(0.5)
    graph, the reference's default hyper-parameter init param = 0): the batch of 32 problems
    is run repeatedly for a bounded sample; ADMM-iters/s = 32 K / seconds per forward."""
    import argparse as _ap

    import unfolded_DLASSO
    P, n, m, B, K = 5, 200, 50, 32, 15
    A, b, _ = O.make_problem(P, m, n, B, seed=1200)
    G = O.er_graph(P, 0.5, seed=7)
    mod = unfolded_DLASSO.DLASSO_unfolded(torch.from_numpy(A)[None], _ap.Namespace(
        GHN_iter_num=K, DADMM_mode="diff", alpha_max=0.1, tau_max=0.99, rho_max=0.99,
        eta_max=0.99, max_penalty_threshold=0.8, penalty_reduction_factor=0.95)).eval()
    res = cpu_baseline(O, A, torch.from_numpy(b), G, mod, P, n, m, K, seconds, fixed_batch=True)
    res["config"] = {"P": P, "n": n, "m": m, "B": B, "K": K, "graph_prob": 0.5}
    return res


def cpu_baseline(O, A, b, G, model, P, n, m, K, seconds, fixed_batch=False):
    """CPU baseline on the GPU box's host (BASELINE.md's CPU plan), a bounded
    sample of the same workload per leg, scaled to ADMM-iters/s. Legs (all ports of the reference
    forward, fp32; the reference itself may not run here):
      * torch_vectorized: oracle/ref_torch.forward_vectorized — the reference's Gram-form algorithm
        with the per-agent GEMVs batched and compute_delta as a Laplacian product (torch CPU);
      * c_port: oracle_forward_f32 (C, OpenMP over samples, the kernel's factored order);
      * torch_loop_faithful: oracle/ref_torch.forward — the reference's eager op sequence with its
        Python per-edge compute_delta loop (unfolded_DLASSO.py:127-140): its real cost profile;
    each on every host thread this process may use (the affinity mask, capped at the cgroup's CPU
    quota: on the GPU boxes 256 hardware threads but a 16-CPU quota, where 256 software threads
    only thrash) and on 1 thread. The headline object is the fastest leg at that thread count;
    every leg is listed under "legs"."""
    import math

    from oracle import ref_torch
    hw_threads, cpu_model, quota = _host_cpus()
    all_threads = min(hw_threads, max(1, math.ceil(quota))) if quota else hw_threads
    with torch.no_grad():
        table = model.hyp_table(K).cpu().numpy()
    bn = b.numpy()
    rng = np.random.default_rng(7)
    per_leg = seconds / 6.0

    def run_leg(fn, threads, B0, Bmax):
        B0, Bmax = min(B0, len(bn)), min(Bmax, len(bn))
        torch.set_num_threads(threads)
        O.set_threads(threads)
        if fixed_batch:
            B0 = Bmax = len(bn)
        Bs, done, t_total = B0, 0, 0.0
        while t_total < per_leg:
            y0, U0, d0 = (1e-2 * rng.standard_normal((3, Bs, P, n))).astype(np.float32)
            t0 = time.perf_counter()
            fn(A, bn[:Bs], [G] * Bs, table, y0, U0, d0)
            dt = time.perf_counter() - t0
            t_total += dt
            done += Bs
            if dt < 0.2 * per_leg and Bs < Bmax:
                Bs = min(Bs * 2, Bmax)
        return {"value": done * K / t_total, "threads": threads, "problems": done,
                "seconds": round(t_total, 2)}

    legs = {}
    saved = torch.get_num_threads()
    for name, fn, B0, Bmax in (("torch_vectorized", ref_torch.forward_vectorized, 16, 2048),
                               ("c_port", O.forward_f32, 16, 2048),
                               ("torch_loop_faithful", ref_torch.forward, 4, 256)):
        for t in sorted({all_threads, 1}, reverse=True):
            legs[f"{name}@{t}"] = run_leg(fn, t, B0, Bmax)
    torch.set_num_threads(saved)
    best_name = max((k for k in legs if legs[k]["threads"] == all_threads),
                    key=lambda k: legs[k]["value"])
    best = legs[best_name]
    return {"value": best["value"], "unit": "ADMM-iters/s", "cores": all_threads, "kind": "port",
            "sample": f"{best_name.split('@')[0]} on {best['problems']} problems of the same shape "
                      f"(P={P} n={n} m={m} K={K}), {best['seconds']} s, {all_threads} threads",
            "cpu_model": cpu_model, "cgroup_cpu_quota": quota, "hardware_threads": hw_threads,
            "legs": legs}


if __name__ == "__main__":
    main()
