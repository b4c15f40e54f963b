#!/bin/bash
# Eager code-object loading (HIP_ENABLE_DEFERRED_LOADING=0): libbnpp loads and
# runs with every code object loaded at the first HIP call.  (`import torch`
# alone segfaults under this setting on this image -- round 6, first run of this
# script, profiles/r06_nodefer_torch.log -- so the Python run leaves PyTorch out
# with BNPP_NO_TORCH=1.)  Each step under its own time limit, stderr kept; the
# first failure ends the script.
#   1. bin/bnpp on asia: libbnpp alone, no Python
#   2. tools/first_call_phases.py through the Python binding, no PyTorch
set -o pipefail
O=gpurun_out/nodefer
mkdir -p $O
M=tests/golden/models
HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 10 120 bn-pp_amd/bin/bnpp $M/asia.uai -pr > $O/cli.log 2>&1 || exit 1
HIP_ENABLE_DEFERRED_LOADING=0 BNPP_NO_TORCH=1 BNPP_TIMING=1 timeout -k 10 240 \
    python3 -X faulthandler -u tools/first_call_phases.py > $O/first_calls_nodefer.jsonl 2> $O/first_calls_nodefer.err || exit 1
BNPP_NO_TORCH=1 BNPP_TIMING=1 timeout -k 10 240 \
    python3 -X faulthandler -u tools/first_call_phases.py > $O/first_calls_defer.jsonl 2> $O/first_calls_defer.err || exit 1
echo nodefer ok
