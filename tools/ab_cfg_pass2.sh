#!/bin/bash
# Per-pass times of every BASELINE config with and without an env setting (diagnostics, same box).
# usage: bash tools/ab_cfg_pass2.sh <tag> "<env>"
set -o pipefail
O=gpurun_out/$1; E=$2; mkdir -p $O
export TMPDIR=/tmp
for c in suntemple_1080p_q bistro_1080p_full emerald_4k_q bistro_4k_full_n16; do
  for e in RSD_AB_NONE=1 "$E"; do
    echo "$c $e $(env $e timeout -k 10 150 python3 -u tools/pass_time.py $c --frames 100 2>>$O/err.log)" >> $O/cfg.txt || exit 1
  done
done
