#!/bin/bash
# GPU box: bench.py under each stream-priority setting, two rounds in turn (no DCN / CPU legs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-run}; shift
mkdir -p gpurun_out
for round in 1 2; do
  for p in none detect criterion; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-dcn --steps 200 --priority $p \
      >> gpurun_out/prio_$TAG.json 2>> gpurun_out/prio_$TAG.err || { echo "EXIT $p"; exit 1; }
  done
done
echo "EXIT 0"
