"""Extract the reference's shipped data fixtures into tests/golden/ (run from the repo root with
/root/reference present: python tests/golden/make_fixtures.py).

Data only, read without unpickling (oracle.load_fixture_tensor reads the zip member
``*/data/0`` as raw little-endian fp32):
  * results/25_iter_general_learning/A.pt      -> fixture_25_iter_general_learning_A.npy
        [1, 5, 100, 500]: the operator of the reference's published 25-iteration run, at its
        default m = 100, n = 500 (configurations.py:6-9), every sigma(A_p) == 10 (set_A's clamp)
  * results/25_iter_general_learning/model.pt  -> fixture_25_iter_general_learning_seq_hyp_param.npy
        [25, 5, 4]: the trained seq_hyp.param of that run
  * results/P_5_num_epoch_220_*/model.pt        -> fixture_P5_220ep_K15_seq_hyp_param.npy [15, 5, 4]
The GPU box has no /root/reference; the tests read these .npy files.
"""
import glob
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle as O  # noqa: E402

REF = "/root/reference/results"

if __name__ == "__main__":
    run = os.path.join(REF, "25_iter_general_learning")
    A = O.load_fixture_tensor(os.path.join(run, "A.pt")).reshape(1, 5, 100, 500)
    np.save(os.path.join(HERE, "fixture_25_iter_general_learning_A.npy"), A)
    param = O.load_fixture_tensor(os.path.join(run, "model.pt")).reshape(25, 5, 4)
    np.save(os.path.join(HERE, "fixture_25_iter_general_learning_seq_hyp_param.npy"), param)
    p15 = glob.glob(os.path.join(REF, "P_5_num_epoch_220_*", "model.pt"))
    if len(p15) == 1:
        np.save(os.path.join(HERE, "fixture_P5_220ep_K15_seq_hyp_param.npy"),
                O.load_fixture_tensor(p15[0]).reshape(15, 5, 4))
    print("wrote", A.shape, param.shape, len(p15))
