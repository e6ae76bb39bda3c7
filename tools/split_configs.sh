#!/bin/bash
# SD-trace setup / walk split (tools/setup_split.sh) of several configs with the bench's clean tiles, each under the
# same env settings.  usage: bash tools/split_configs.sh <tag> "<config ...>" [env settings ("-": none) ...]
set -o pipefail
TAG=$1; CFGS=$2; shift 2
[ $# -eq 0 ] && set -- -
for c in $CFGS; do
  SD_TIME_ARGS="$c --clean-tiles" bash tools/setup_split.sh ${TAG}_$c "$@" || exit 1
done
