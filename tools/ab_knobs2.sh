#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python tools/mar_grid.py --check 0 --reps 3 > gpurun_out/abk_$tag.jsonl 2>gpurun_out/abk_$tag.err || { tail -5 gpurun_out/abk_$tag.err; exit 1; }
  python -c "
import json; d=[json.loads(x) for x in open('gpurun_out/abk_$tag.jsonl') if '\"mar\"' in x]; print('$tag', [round(x['uptime_ms'],1) for x in d], d[-1]['p_mid'])"
}
run base BNPP_TIMING=1
run s40 BNPP_TREE_SLOTS=40 BNPP_TIMING=1
run s38 BNPP_TREE_SLOTS=38
run s34 BNPP_TREE_SLOTS=34
run s41 BNPP_TREE_SLOTS=41
run s40b BNPP_TREE_SLOTS=40
