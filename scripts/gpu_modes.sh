#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u scripts/step_modes2.py > $O/modes_$TAG.json 2> $O/modes_$TAG.err || { tail -20 $O/modes_$TAG.err; exit 1; }
cat $O/modes_$TAG.json
echo EXIT 0
