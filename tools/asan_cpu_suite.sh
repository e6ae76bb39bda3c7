#!/bin/bash
# The CPU test suite (pytest -m "not gpu") against ASan + UBSan builds of the oracle and of librsd's
# host code (sanitizers on the CPU side).  Leak checking is off (the Python interpreter
# and torch keep allocations to exit); any ASan / UBSan report aborts the test process.
# usage: bash tools/asan_cpu_suite.sh [log]   (build container; no GPU needed)
set -o pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/round3/asan_cpu_suite.log}
mkdir -p "$(dirname "$LOG")"
make -C oracle asan > /dev/null && make -C ray-traced-stochastic-depth-map_amd -j8 asan > /dev/null || exit 1
ASAN_LIB=$(gcc -print-file-name=libasan.so)
UBSAN_LIB=$(gcc -print-file-name=libubsan.so)
{
  echo "# $(date -u +%FT%TZ)  ASan+UBSan CPU suite: oracle/_build/librsd_oracle_asan.so, librsd_asan.so"
  echo "# LD_PRELOAD=$ASAN_LIB:$UBSAN_LIB ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1"
} > "$LOG"
export LD_PRELOAD="$ASAN_LIB:$UBSAN_LIB" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:verify_asan_link_order=0 \
  UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 RSD_LIB_VARIANT=asan RSD_ORACLE_VARIANT=asan
# the instrumented libraries are the ones loaded (their paths, and the sanitizer runtime in the maps)
python - >> "$LOG" 2>&1 <<'PY'
import sys
sys.path[:0] = ["ray-traced-stochastic-depth-map_amd", "."]
from rsd import abi
from oracle import oracle as O
abi.lib(); O.lib()
maps = open("/proc/self/maps").read()
print("# loaded:", abi.LIB_PATH.name, O._LIB_PATH.name, "| libasan mapped:", "libasan" in maps, "| libubsan mapped:", "libubsan" in maps)
PY
python -m pytest tests -m "not gpu" -q -p no:cacheprovider >> "$LOG" 2>&1
rc=$?
echo "# exit $rc" >> "$LOG"
tail -3 "$LOG"
exit $rc
