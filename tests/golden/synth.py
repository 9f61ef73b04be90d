"""Deterministic synthetic weights shared by the fixture generator and the tests.

Weights are NOT stored in the fixtures: they are regenerated bit-identically
from (state_dict key order, shapes, seed) with numpy's PCG64, then rounded to
fp16-representable values so fp16 device copies are exact.

* conv / linear ``.weight``: U(-1, 1)·√3/√fan_in   (unit-variance-preserving)
* ``.bias`` of conv / linear: U(-1, 1)/√fan_in
* 1-D ``.weight`` (GroupNorm / LayerNorm γ): 1 + 0.1·N(0, 1);  their ``.bias``: 0.1·N(0, 1)
"""
from __future__ import annotations

import math

import numpy as np


def synth_weights(keys_shapes, seed: int, scale: float = 1.0) -> dict:
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    shapes = dict(keys_shapes)
    for key, shape in keys_shapes:
        shape = tuple(int(s) for s in shape)
        if key.endswith(".weight") and len(shape) >= 2:
            fan_in = int(np.prod(shape[1:]))
            w = (rng.random(shape) * 2 - 1) * math.sqrt(3.0) / math.sqrt(fan_in) * scale
        elif key.endswith(".weight"):
            w = 1.0 + 0.1 * rng.standard_normal(shape)
        elif key.endswith(".bias"):
            wkey = key[: -len(".bias")] + ".weight"
            wshape = shapes.get(wkey)
            if wshape is not None and len(wshape) >= 2:
                fan_in = int(np.prod(wshape[1:]))
                w = (rng.random(shape) * 2 - 1) / math.sqrt(fan_in) * scale
            else:
                w = 0.1 * rng.standard_normal(shape)
        else:
            w = rng.standard_normal(shape)
        out[key] = w.astype(np.float16).astype(np.float32)
    return out


def keys_shapes_of(state_dict) -> list:
    return [(k, tuple(v.shape)) for k, v in state_dict.items()]
