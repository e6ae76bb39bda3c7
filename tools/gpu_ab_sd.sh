set -o pipefail
mkdir -p gpurun_out/ab1
export TMPDIR=/tmp
for cfg in "" "RSD_TRACE_WAVES_PER_CU=10" "RSD_TRACE_WAVES_PER_CU=12 RSD_TRACE_POOL=128" "RSD_TRACE_WAVES_PER_CU=16 RSD_TRACE_POOL=128" "RSD_TRACE_ENTRY=off"; do
  echo "== $cfg" >> gpurun_out/ab1/sd_time.txt
  env $cfg timeout -k 10 120 python3 -u tools/sd_time.py >> gpurun_out/ab1/sd_time.txt 2>&1 || exit 1
  env $cfg timeout -k 10 120 python3 -u tools/sd_time.py >> gpurun_out/ab1/sd_time.txt 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab1/prof -o run -- python3 -u tools/sd_time.py > gpurun_out/ab1/prof.log 2>&1
