# round-5 batch g: pass-1 XCD chunk A/B (RSD_PASS1_XCD) at configs[1] and configs[3]
mkdir -p gpurun_out/r5g
for c in 4 16 64; do
  timeout -k 10 120 python tools/env_ab.py RSD_PASS1_XCD 0 $c --what pass1 --n 40 --reps 6 > gpurun_out/r5g/xcd_c1_$c.json 2>&1 || exit 1
done
timeout -k 10 200 python tools/env_ab.py RSD_PASS1_XCD 0 16 emerald_4k_q --what pass1 --n 20 --reps 4 > gpurun_out/r5g/xcd_c3_16.json 2>&1
