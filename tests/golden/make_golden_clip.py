"""Golden vectors for the CLIP text transformer from the installed
``transformers`` CLIPTextModel (the class the reference's FrozenCLIPEmbedder calls,
clip_encoder/modules.py:221-256) — build container only; no network, no pretrained weights:
a small config with the synthetic weights of tests/golden/synth.py.

Run from the repo root:  python tests/golden/make_golden_clip.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, OUT)

TINY_CLIP = dict(vocab_size=1000, hidden_size=128, intermediate_size=512, num_hidden_layers=2,
                 num_attention_heads=2, max_position_embeddings=77, hidden_act="quick_gelu",
                 layer_norm_eps=1e-5, bos_token_id=998, eos_token_id=999, pad_token_id=999)


def main():
    import transformers
    from transformers import CLIPTextConfig, CLIPTextModel
    from synth import synth_weights
    torch.manual_seed(0)
    m = CLIPTextModel(CLIPTextConfig(**TINY_CLIP)).eval()
    sd = m.state_dict()
    keys = [[k, list(v.shape)] for k, v in sd.items() if not k.endswith("position_ids")]
    w = synth_weights(keys, 31)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()}, strict=False)
    g = torch.Generator().manual_seed(32)
    ids = torch.randint(0, 998, (2, 77), generator=g)
    ids[:, 0] = 998                                   # BOS, text, EOS then padding as the tokenizer emits
    ids[0, 9:] = 999
    ids[1, 40:] = 999
    with torch.no_grad():
        y = m(input_ids=ids).last_hidden_state
    np.savez_compressed(os.path.join(OUT, "clip_tiny.npz"), ids=ids.numpy(), y=y.numpy(), seed=np.int64(31),
                        keys=np.frombuffer(json.dumps(keys).encode(), dtype=np.uint8),
                        cfg=np.frombuffer(json.dumps(TINY_CLIP).encode(), dtype=np.uint8),
                        transformers_version=np.frombuffer(transformers.__version__.encode(), dtype=np.uint8))
    print("clip_tiny.npz", os.path.getsize(os.path.join(OUT, "clip_tiny.npz")), "transformers", transformers.__version__)


if __name__ == "__main__":
    main()
