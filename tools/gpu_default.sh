#!/bin/bash
# The driver's round-end commands on the current tree: smoke(), then the default bench line.
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 2>&1 | tail -1 | cut -c1-400
