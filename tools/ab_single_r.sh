#!/bin/bash
# (the BNPP_SLAB_SINGLE_R variant was measured and removed: profiles/r04_single_passes_ab.txt)
# Bench bucket (single-op slab kernel, f32 and the fp64 leg): one pass vs two
# passes of tiles per block (BNPP_SLAB_SINGLE_R=2), interleaved, 3 rounds.
set -o pipefail
R=$PWD
for i in 1 2 3; do
  for e in BNPP_AB_NONE=1 BNPP_SLAB_SINGLE_R=2; do
    env $e timeout -k 10 200 python3 bench.py --no-cpu --no-mar --steps 40 > /tmp/b.json 2>/tmp/b.err || { tail -5 /tmp/b.err; exit 1; }
    python3 - $e <<'PY'
import json, sys
d = json.loads(open('/tmp/b.json').read().strip().splitlines()[-1])
print("%-22s f32 %.4f ms frac %.4f  f64 %.4f ms frac %.4f exact %s" % (sys.argv[1], d['roofline'].get('kernel_ms', d['ms_per_step']), d['roofline']['frac'],
      d['fp64_bucket'].get('kernel_ms', 0), d['fp64_bucket']['frac'], d['fp64_bucket'].get('spot_check_exact')))
PY
  done
done
