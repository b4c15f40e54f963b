#!/bin/bash
# A/B of runtime knobs on the bench bucket (and the 32x32 PR end to end).
# usage: tools/ab_knobs.sh "ENV=.. ENV2=.." "ENV=.." ...
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
    echo "== $cfg"
    env $cfg timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-mar > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    python -c "
import json; l=[x for x in open('gpurun_out/ab.log') if x.startswith('{')]; d=json.loads(l[-1]); print('bench', d['roofline']['kernel_ms'], round(d['roofline']['frac'],4))"
    if [ -n "$AB_VE" ]; then
        env $cfg timeout -k 10 300 python tools/ve_bench.py --only 32x32 > gpurun_out/ab_ve.log 2>&1 || { tail -5 gpurun_out/ab_ve.log; exit 1; }
        python -c "
import json; d=json.loads(open('gpurun_out/ab_ve.log').read().strip().splitlines()[-1]); print('32x32', round(d['gpu_uptime_ms'],1), d['log10Z'])"
    fi
done
