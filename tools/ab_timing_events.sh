set -o pipefail
O=gpurun_out/abev; mkdir -p $O
for rep in 1 2; do
for t in hip torch off; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 0 --timing-events $t > $O/s20_${t}_$rep.json 2>$O/err_$t.log || exit 1
done; done
for t in hip torch; do
timeout -k 10 200 python -u bench.py --cpu-baseline-seconds 0 --timing-events $t > $O/s200_${t}.json 2>$O/err200_$t.log || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --cpu-baseline-seconds 0 > $O/prof.log 2>&1
