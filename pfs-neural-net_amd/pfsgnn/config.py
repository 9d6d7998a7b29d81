"""Constants of the reference configuration (src/config.py:3-30).

``device`` is always the HIP device: this package has no CPU/MPS path.
"""
import torch

device = torch.device("cuda")

# === PATHS === (config.py:12-13)
datafile = "../params/increasing.txt"
checkpoint_path = "../params/model_gnn_"

# === CONSTANTS === (config.py:16-19)
NFIBERS = 2000
NCLASSES = 12
NFIELDS = 10
TOTAL_TIME = 42

# === TRAINING PARAMETERS === (config.py:22-30)
nepochs = 40_000
Fdim = 10
lr = 5e-4
pclass = 0.1
pfiber = 0.1
wutils = 2000.0
wvar = 1.0
sharps = [0.0, 20.0]
min_sharp = 5.0
