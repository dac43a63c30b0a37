"""dadmm_hip — MI355X (gfx950) unfolded D-ADMM forward behind the reference's module API.

The drop-in modules (``unfolded_DLASSO``, ``gnn_dlasso_models_progressive``, ``gnn_dlasso_utils``,
``gnn_data``, ``configurations``) live next to this package; with its parent directory on
``sys.path`` the reference drivers' imports of those modules resolve to them. The driver files
themselves also import modules the reference does not ship, so the supported drivers are this
repo's ``train_unfolded.py`` / ``train_gnn.py``.
"""
from . import _lib
from .graph import GraphBatch, from_csr, generate_er, ingest, to_networkx
from .ops import PreparedOperator, forward_raw

__all__ = ["_lib", "GraphBatch", "from_csr", "generate_er", "ingest", "to_networkx",
           "PreparedOperator", "forward_raw"]
