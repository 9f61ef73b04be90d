#!/bin/bash
# Re-time the C3 conv problems at REPS (default 12) timed launches per candidate and bench C3 with the result merged
# into the committed table against the committed table, alternated on the same box (gpurun_out/retune12/).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/retune12
mkdir -p $L
SD_AMD_TUNE_REPS=${REPS:-12} timeout -k 10 900 python -u bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache /nonexistent --tuning-out $L/tuneN.json > $L/tune.log 2>&1 || { tail -20 $L/tune.log; exit 1; }
python - <<'PY'
import json
o = json.load(open("configs/conv_tuning_mi355x.json"))
n = json.load(open("gpurun_out/retune12/tuneN.json"))
new = {json.dumps(k): v for k, v in n["entries"]}
merged = [[k, new.get(json.dumps(k), v)] for k, v in o["entries"]]
ch = sum(1 for k, v in o["entries"] if json.dumps(k) in new and new[json.dumps(k)] != v)
o["entries"] = merged
json.dump(o, open("gpurun_out/retune12/merged.json", "w"), indent=0)
print(f"c3 keys re-timed: {len(new)}, changed vs committed: {ch}")
PY
i=0
for t in configs/conv_tuning_mi355x.json $L/merged.json configs/conv_tuning_mi355x.json $L/merged.json; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $t > $L/c3_$i.log 2>&1 || { tail -20 $L/c3_$i.log; exit 1; }
  python - $L/c3_$i.log $t <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(f"{sys.argv[2]}: value {d['value']:.3f} ms_per_step {d['ms_per_step']:.2f} unet {d['unet_step_ms']:.3f}")
PY
done
