#!/bin/bash
# One GPU-box pass for a 10M-record config line (tools/config_lines.py): the index is built in-run on the box's
# 16 CPUs, then each layout / cache variant is measured.  Usage (via gpurun): bash tools/r03_cfg.sh <which> <tag> [args]
set -o pipefail
W=$1; T=$2; shift 2
O=gpurun_out/r03; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1140 python -u tools/config_lines.py --which $W --n 10000000 --out $O/$T.jsonl "$@" > $O/$T.log 2>&1
rc=$?
tail -4 $O/$T.log
exit $rc
