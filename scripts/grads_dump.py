"""Dump the Atari gradient blob of one small step (A/B of builds: FI_LIB_OVERRIDE=...)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from freeimpala_amd.learner import DeviceLearner  # noqa: E402

L = DeviceLearner("atari", seq_len=3, batch=96, num_actions=18, optimizer="sgd", lr=1e-3, max_grad_norm=0.0, seed=4)
L.synth(seed=17)
L.step_resident()
np.save(sys.argv[1], L.tensor("grads"))
L.close()
