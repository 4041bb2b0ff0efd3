import os, sys
sys.path.insert(0, os.getcwd())
os.environ["FI_VERBOSE"] = "1"
from freeimpala_amd.learner import DeviceLearner
L = DeviceLearner("atari", seq_len=100, batch=4096, num_actions=18, optimizer="adam")
L.close()
