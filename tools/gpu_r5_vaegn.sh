#!/bin/bash
# The one-pass GroupNorm apply at the VAE decoder's >= 128x128 images too (SDK_GN_APPLY_FLAT=2) vs the row form there
# (=1, default): C3 bench lines alternated on one box; the decode share = ms_per_step - 50 x unet_step_ms.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/vaegn
mkdir -p $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "group_norm" --timeout 200 --timeout-method thread > $L/tests.log 2>&1 || { tail -30 $L/tests.log; exit 1; }
tail -1 $L/tests.log
i=0
for f in 1 2 1 2; do
  i=$((i+1))
  SDK_GN_APPLY_FLAT=$f timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > $L/c3_$i.log 2>&1 || { tail -20 $L/c3_$i.log; exit 1; }
  python - $L/c3_$i.log $f <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(f"flat={sys.argv[2]} value {d['value']:.3f} ms_per_step {d['ms_per_step']:.2f} unet {d['unet_step_ms']:.3f} outside-UNet {d['ms_per_step'] - 50 * d['unet_step_ms']:.2f} ms")
PY
done
