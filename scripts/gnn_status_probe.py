#!/usr/bin/env python3
"""Guard status of GNN eval forwards through the captured-graph plan, interleaved with other
work, to locate a corruption of the plan's guard-flag words: python scripts/gnn_status_probe.py"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hyperparameter-gnn_unfolded-d-admm-main_amd")]
import torch  # noqa: E402

import gnn_dlasso_models_progressive as GM  # noqa: E402
import oracle as O  # noqa: E402
from dadmm_hip.graph import ingest  # noqa: E402
from dadmm_hip.ops import draw_inits  # noqa: E402

dev = torch.device("cuda:0")
B, P, n, m, K = 64, 5, 256, 64, 5
A, b, _ = O.make_problem(P, m, n, B, seed=55)
args = argparse.Namespace(GHN_iter_num=K, GHyp_hidden=100, DADMM_mode="diff", alpha_max=0.1,
                          tau_max=0.99, rho_max=0.99, eta_max=0.99)
g = GM.DLASSO_GNNHyp3_Progressive(torch.from_numpy(A)[None].to(dev), args).to(dev).eval()
graphs = ingest([O.connected_er_graph(P, 0.5, seed=500 + s) for s in range(B)], P, B, dev)
bt = torch.from_numpy(b)[..., None].to(dev)
inits = tuple(torch.randn(B, P, n, device=dev) * 1e-2 for _ in range(3))


def fwd(tag, graph=True, **kw):
    g.use_hip_graph = graph
    with torch.no_grad():
        Y, _ = g(bt, graphs, **kw)
    torch.cuda.synchronize()
    plan = next(iter(g._graph_plans.values())) if g._graph_plans else None
    fl = plan.run_.flags[:6].tolist() if plan is not None else None
    print(f"{tag:28s} graph={graph} status={int(g.last_status.item())} plan flags={fl} "
          f"flags ptr={plan.run_.flags.data_ptr() if plan else 0:#x}", flush=True)
    return Y


def block_state(addr):
    for seg in torch.cuda.memory_snapshot():
        a = seg["address"]
        if a <= addr < a + seg["total_size"]:
            for blk in seg["blocks"]:
                if blk["address"] <= addr < blk["address"] + blk["size"]:
                    return seg.get("segment_pool_id"), blk["state"], blk["size"], hex(blk["address"])
    return None


keep = [fwd("graph 1 (kept)", inits=inits)]
plan = next(iter(g._graph_plans.values()))
for nm in ("flags", "status", "yptr"):
    t = getattr(plan.run_, nm)
    print(nm, hex(t.data_ptr()), t.numel(), block_state(t.data_ptr()), flush=True)
print("steps", hex(plan.steps.data_ptr()), block_state(plan.steps.data_ptr()), flush=True)
with torch.no_grad():   # plan.run step by step
    fl = plan.run_.flags
    fl.zero_(); torch.cuda.synchronize()
    print("zeroed", fl[:6].tolist(), flush=True)
    a_hat = GM.normalized_adjacency(graphs.nbr, P)
    a_hat = (a_hat if not graphs.shared else a_hat[None]).contiguous()
    plan._load(bt[..., 0], graphs, a_hat, *inits); torch.cuda.synchronize()
    print("after _load", fl[:6].tolist(), flush=True)
    Yx = torch.empty((plan.K, plan.B, plan.P, plan.ns), device=dev)
    plan.run_.yptr[1:].copy_(plan.steps + Yx.data_ptr()); torch.cuda.synchronize()
    print("after yptr", fl[:6].tolist(), "yptr", [hex(v) for v in plan.run_.yptr.tolist()], flush=True)
    plan.graph.replay(); torch.cuda.synchronize()
    print("after replay", fl[:16].tolist(), "status", int(plan.run_.status.item()), flush=True)
keep.append(fwd("graph 2 (kept)", inits=inits))
keep.append(fwd("graph 3 (kept)", inits=inits))
del keep
fwd("graph 4", inits=inits)
fwd("graph 5", inits=inits)
with torch.no_grad():
    t = draw_inits((B, P, n), dev)
torch.cuda.synchronize()
fwd("after draw_inits", inits=inits)
fwd("non-graph", graph=False, inits=inits)
fwd("graph after non-graph", inits=inits)
fwd("graph drawn", graph=True)
fwd("graph again", inits=inits)
