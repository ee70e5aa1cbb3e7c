#!/bin/bash
# A/B phase times of the in-tree library under environment settings.
# Usage (repo root on the GPU box): bash tools/ab_env.sh F "VAR=1" "VAR2=x" ...   ("-": none)
F=$1; shift
for e in "$@"; do
  [ "$e" = "-" ] && e=""
  echo "== [$e] $F"; env $e timeout -k 10 200 python tools/phase_time.py $F 3 || exit 1
  echo "== [$e] 1"; env $e timeout -k 10 100 python tools/phase_time.py 1 3 || exit 1
done
