#!/bin/bash
# tools/gpu_r5_retune6.sh for C5 and C2: re-time each config's conv problems at 6 reps, merge into the committed
# table, bench the config with both tables alternated on the same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/retune6b
mkdir -p $L
cp configs/conv_tuning_mi355x.json $L/cur.json
for c in c5 c2; do
  SD_AMD_TUNE_REPS=6 timeout -k 10 900 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache /nonexistent --tuning-out $L/tune6_$c.json > $L/tune_$c.log 2>&1 || { tail -20 $L/tune_$c.log; exit 1; }
  python - $L/cur.json $L/tune6_$c.json $L/merged_$c.json <<'PY'
import json, sys
o = json.load(open(sys.argv[1]))
n = json.load(open(sys.argv[2]))
new = {json.dumps(k): v for k, v in n["entries"]}
ch = sum(1 for k, v in o["entries"] if json.dumps(k) in new and new[json.dumps(k)] != v)
o["entries"] = [[k, new.get(json.dumps(k), v)] for k, v in o["entries"]]
json.dump(o, open(sys.argv[3], "w"), indent=0)
print(f"{sys.argv[2]}: keys re-timed {len(new)}, changed vs current {ch}")
PY
  i=0
  for t in $L/cur.json $L/merged_$c.json $L/cur.json $L/merged_$c.json; do
    i=$((i+1))
    timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $t > $L/${c}_$i.log 2>&1 || { tail -20 $L/${c}_$i.log; exit 1; }
    python - $L/${c}_$i.log $t <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        print(f"{sys.argv[2]}: value {d['value']:.3f} ms_per_step {d['ms_per_step']:.2f} unet {d['unet_step_ms']:.3f}")
PY
  done
done
