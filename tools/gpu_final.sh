#!/bin/bash
# End-of-round check of the committed tree: the GPU suite, smoke(), the default bench line.
set -e
O=gpurun_out/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
cat $O/smoke.log | tail -2
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cut -c1-400 $O/bench.json
