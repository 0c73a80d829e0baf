#!/bin/bash
# Round 5, run 14: the random-row gather ceiling at the configs' own shapes (rows at their packed stride, the fresh
# neighbours per expansion as rows per step, the search kernels' wavefronts per CU), and cfg5's rows padded.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/gather_probe2.jsonl
G=tools/gather_probe
run() { timeout -k 10 60 $G "$@" >> $O || exit 3; }
for rb in 400 416 448 512; do for wpc in 4 5 8; do for rps in 12 16; do run 20 $rb $wpc $rps 1 256; done; done; done
for wpc in 4 6 8; do for rps in 10 16; do run 36 384 $wpc $rps 1 256; done; done
for wpc in 8 12; do for rps in 12 16; do run 0.5 512 $wpc $rps 1 256; done; done
echo ok
