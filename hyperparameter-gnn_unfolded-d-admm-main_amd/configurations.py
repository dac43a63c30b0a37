"""Drop-in ``configurations.args_parser``: the flat argparse namespace both drivers and the
modules read (reference configurations.py:3-131).

Same flag names, types, defaults and choices, including the reference's quirks (``--seed`` and
``--GHyp_hidden`` are parsed as float; ``--sequential``/``--valid`` use ``type=bool``). The modules
on the hot path read: GHN_iter_num, DADMM_mode, alpha_max, tau_max, rho_max, eta_max,
max_penalty_threshold, penalty_reduction_factor (and GHyp_hidden for the GNN model).
"""
from __future__ import annotations

import argparse

# (flag, type, default, extra kwargs) — grouped as in the reference
_FLAGS = [
    # problem size and hyper-parameter bounds
    ("m", int, 100, {}), ("n", int, 500, {}),
    ("alpha_max", float, 0.1, {}), ("tau_max", float, 0.99, {}),
    ("rho_max", float, 0.99, {}), ("eta_max", float, 0.99, {}),
    ("init_alpha_frac", float, 0.2, {}), ("init_tau_frac", float, 0.15, {}),
    ("init_rho_frac", float, 0.25, {}), ("init_eta_frac", float, 0.1, {}),
    ("max_penalty_threshold", float, 0.8, {}), ("penalty_reduction_factor", float, 0.95, {}),
    # experiment bookkeeping
    ("exp_name", str, "exp for 5 agents", {}),
    ("method", str, "u-dadmm", {}), ("seq_num", int, 0, {}),
    # data
    ("data", str, "simulated", {"choices": ["mnist", "simulated"]}),
    ("norm_mean", float, 0.5, {}), ("norm_std", float, 0.5, {}),
    ("train_size", int, 200, {}), ("snr", int, 4, {}), ("test_size", int, 32, {}),
    ("batch_size", int, 16, {}),
    # graph
    ("P", int, 5, {}), ("graph_prob", float, 0.5, {}), ("graph_type", str, "erods_renyi", {}),
    # D-ADMM (legacy path values kept for namespace compatibility)
    ("case", str, "dlasso", {"choices": ["dlasso", "dlr"]}),
    ("model", str, "same", {"choices": ["diff", "same"]}),
    ("rho", float, 0.2603, {}), ("alpha", float, 0.3013, {}), ("eta", float, 0.0867, {}),
    ("gamma", float, 1.1797e-07, {}), ("beta", float, 1.2260e-03, {}),
    ("delta", float, 1.2665e-04, {}), ("tau", float, 0.1142, {}),
    ("sequential", bool, False, {}), ("max_iter_seg", int, 2, {}), ("max_iter", int, 25, {}),
    ("num_epochs", int, 10, {}),
    # learning
    ("optimizer", str, "adam", {"choices": ["sgd", "adam"]}),
    ("lr", float, 1e-04, {}), ("momentum", float, 0.5 * 1e-05, {}),
    ("weight_decay", float, 0.0001, {}),
    ("device", str, "cpu", {"choices": ["cuda:0", "cuda:1", "cpu"]}),
    ("valid", bool, True, {}), ("seed", float, 42, {}),
    # GNN hypernetwork / unfolded model
    ("GHyp_hidden", float, 100, {}),
    ("DADMM_mode", str, "diff", {"choices": ["same", "diff"]}),
    ("hyp_mode", str, "unfolded", {"choices": ["GHyp", "unfolded"]}),
    ("GHN_iter_num", int, 15, {}),
    ("save_dir", str, "./results", {}),
]
_STORE_TRUE = ("eval", "lr_scheduler")


def build_parser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser()
    for name, typ, default, extra in _FLAGS:
        parser.add_argument(f"--{name}", type=typ, default=default, **extra)
    for name in _STORE_TRUE:
        parser.add_argument(f"--{name}", action="store_true")
    return parser


def args_parser(argv=None):
    """Parse ``argv`` (default: sys.argv[1:]) into the reference's namespace."""
    return build_parser().parse_args(argv)
