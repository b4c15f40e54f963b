#!/bin/bash
# A/B library variants (tools/build_variant.sh) on the 32x32 bucket-tree MAR, 3 calls each.
# usage: tools/ab_mar.sh base name1 ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = base ]; then L=$PWD/bn-pp_amd/lib/libbnpp.so; else L=$PWD/bn-pp_amd/lib_$v/libbnpp.so; fi
  BNPP_LIB=$L timeout -k 10 200 python tools/mar_grid.py --check 0 --reps 3 > gpurun_out/abm_$v.jsonl 2>gpurun_out/abm_$v.err || { tail -5 gpurun_out/abm_$v.err; exit 1; }
  python -c "
import json; d=[json.loads(x) for x in open('gpurun_out/abm_$v.jsonl') if '\"mar\"' in x]; print('$v', [round(x['uptime_ms'],1) for x in d], d[-1]['p_mid'])"
done
