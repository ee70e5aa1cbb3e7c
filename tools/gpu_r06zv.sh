#!/bin/bash
# r06zv: enc_pack waves prioritised by their bit count (ab/pemit) and dec_place's
# bookkeeping loads issued together (ab/pspec) vs the working tree; 512 x 4K, one 4K frame.
set -e
for rep in 1 2; do for d in - ab/pemit ab/pspec; do
  if [ "$d" = "-" ]; then unset NICE_LIB_PATH; else export NICE_LIB_PATH=$d/libnice_hip.so; fi
  echo "== [$d] 512"
  timeout -k 10 200 python tools/phase_time.py 512 3 2>&1 | grep -E "F=|rror" | sed -e "s/'enc_tailruns.*'enc_pack'/ pack/" -e "s/'dec_scan.*'dec_place'/ place/" | cut -c1-170
done; done
for d in - ab/pspec; do
  if [ "$d" = "-" ]; then unset NICE_LIB_PATH; else export NICE_LIB_PATH=$d/libnice_hip.so; fi
  echo "== [$d] 1"
  timeout -k 10 200 python tools/phase_time.py 1 5 2>&1 | grep -E "decode F=|rror" | sed -e "s/'dec_scan.*'dec_place'/ place/" | cut -c1-170
done
