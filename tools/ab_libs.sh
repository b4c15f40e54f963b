#!/bin/bash
# A/B alternative library builds (tools/build_variant.sh) on the bench bucket
# and, with AB_VE=1, the 32x32 sweep.  usage: tools/ab_libs.sh base name1 name2 ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = base ]; then L=$PWD/bn-pp_amd/lib/libbnpp.so; else L=$PWD/bn-pp_amd/lib_$v/libbnpp.so; fi
  echo "== $v"
  BNPP_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-mar > gpurun_out/ab_$v.log 2>&1 || { tail -5 gpurun_out/ab_$v.log; exit 1; }
  python -c "
import json; l=[x for x in open('gpurun_out/ab_$v.log') if x.startswith('{')]; d=json.loads(l[-1]); print('bench', d['roofline']['kernel_ms'], round(d['roofline']['frac'],4))"
  if [ -n "$AB_VE" ]; then
    BNPP_LIB=$L timeout -k 10 300 python tools/ve_bench.py --only 32x32 > gpurun_out/ab32_$v.jsonl 2>&1 || { tail -5 gpurun_out/ab32_$v.jsonl; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab32_$v.jsonl').read().strip().splitlines()[-1]); print('32x32', round(d['gpu_uptime_ms'],1), d['log10Z'])"
  fi
done
