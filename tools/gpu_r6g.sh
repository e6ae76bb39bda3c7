#!/bin/bash
set -o pipefail
O=gpurun_out/r6g
for c in bistro_4k_full_n16 bistro_1080p_full suntemple_1080p_q; do bash tools/lib_ab.sh $O base $c || exit 1; done
