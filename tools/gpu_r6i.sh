#!/bin/bash
# diagnostics: walk time over the longest-first rays only / the other rays only, per walk (RSD_TRACE_QRANGE)
set -o pipefail
O=gpurun_out/r6i; mkdir -p $O
for c in emerald_4k_q bistro_1080p_full bistro_4k_full_n16; do
  for w in quad fused; do
    timeout -k 10 300 python tools/env_ab.py RSD_TRACE_QRANGE all long $c --walk $w --n 10 --reps 3 --clean-tiles > $O/qr_${c}_${w}_a.json 2> $O/qr_${c}_${w}_a.err || { tail -3 $O/qr_${c}_${w}_a.err; exit 1; }
    tail -1 $O/qr_${c}_${w}_a.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $w', d['median_us'])"
    timeout -k 10 300 python tools/env_ab.py RSD_TRACE_QRANGE short none $c --walk $w --n 10 --reps 3 --clean-tiles > $O/qr_${c}_${w}_b.json 2> $O/qr_${c}_${w}_b.err || { tail -3 $O/qr_${c}_${w}_b.err; exit 1; }
    tail -1 $O/qr_${c}_${w}_b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c $w', d['median_us'])"
  done
done
