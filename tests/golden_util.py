"""Helpers to read the golden fixtures (tests only)."""
import json
import os

import numpy as np
import torch

from synth import synth_weights

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def cfg_of(z):
    return json.loads(bytes(z["cfg"]).decode())


def weights_of(z):
    ks = json.loads(bytes(z["keys"]).decode())
    w = synth_weights([(k, tuple(s)) for k, s in ks], int(z["seed"]))
    return {k: torch.from_numpy(v) for k, v in w.items()}
