#!/bin/bash
# round 5: row walk wave priority for longest-first rays (RSD_TRACE_PRIO) A/B
set -o pipefail
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_PRIO off on suntemple_1080p_q --n 40 --reps 7 --clean-tiles > $O/prio_c1.json 2> $O/prio_c1.err || exit 1
tail -1 $O/prio_c1.json
timeout -k 10 200 python tools/env_ab.py RSD_TRACE_PRIO off on suntemple_1080p_q --n 40 --reps 7 --clean-tiles > $O/prio_c1b.json 2> $O/prio_c1b.err || exit 1
tail -1 $O/prio_c1b.json
for v in off on off on; do
  RSD_TRACE_PRIO=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('prio $v', d['value'], d['ms_per_step'], d.get('sd_kernel_ms'))"
done
