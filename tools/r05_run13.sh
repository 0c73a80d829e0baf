#!/bin/bash
# Round 5, run 13: the random-row gather ceiling (tools/gather_probe.hip) for the BASELINE configs' row sizes and index
# sizes — the rate the search kernels' access pattern can reach at all — beside which the configs' roofline fractions
# are read.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/gather_probe.jsonl
G=tools/gather_probe
run() { timeout -k 10 60 $G "$@" >> $O || exit 3; }
# array sizes: 0.5 GiB (bench: 1M x 512 B, Infinity-Cache-sized), 20 GiB (cfg5 50M x 400 B), 36 GiB (cfg4 100M x 384 B)
for gib in 0.5 20 36; do
  for rb in 384 448 512; do
    for wpc in 4 8 16; do
      for dep in 1 2; do run $gib $rb $wpc 16 $dep 256; done
    done
  done
done
# fewer rows per step (a search expansion has ~8-16 fresh neighbours)
for gib in 0.5 36; do for rps in 4 8; do run $gib 384 8 $rps 1 256; done; done
# adjacency-sized rows (132 B level-0 lists: 128 + header, read as 192 B)
for gib in 0.5 12; do run $gib 192 8 16 1 256; done
echo ok
