#!/bin/bash
# runs every built tools/microbench/tgemm_* variant (GPU)
cd "$(dirname "$0")"
for b in tgemm_*; do
  case $b in *.hip|*.sh) continue;; esac
  echo "== $b"; timeout -k 5 60 ./$b ${1:-24576} || exit 1
done
