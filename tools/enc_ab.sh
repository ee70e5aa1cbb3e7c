#!/bin/bash
# Encode/decode phase times + stream digests of several ab/ builds, two
# alternating passes: bash tools/enc_ab.sh NF DIR...
NF=$1; shift
for pass in 1 2; do
  for d in "$@"; do
    NF=$NF NICE_LIB_PATH=$d/libnice_hip.so timeout -k 10 200 python tools/enc_time.py 2>&1 | grep digest | \
      python3 -c "import sys,re,ast
for l in sys.stdin:
    ph=ast.literal_eval(l[l.index('{'):]); print(l.split(']')[0]+']', re.search(r'encode [0-9.]+ ms',l).group(0), re.search(r'digest=\w+',l).group(0), 'classify', ph.get('enc_classify'), 'pack', ph.get('enc_pack'), 'ok' in l and l.split('ok=')[1].split()[0])"
  done
done
